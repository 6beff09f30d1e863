"""Round 4's k_min<0> defect: tools/mir_emu.py on the
machine IR after every pass of an llc -print-after-all dump, counting the
oracle cases whose stored record is wrong or holds an undefined word.
Investigation tool (the oracle is the checker, as in tests/).

    llc -mtriple=amdgcn-amd-amdhsa -mcpu=gfx950 -O3 -print-after-all IN.ll -o /dev/null 2> dump.txt
    python tools/kmin_mir_stages.py dump.txt [cases]
"""
import sys, re
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tools')); sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'tests'))
import mir_emu
from test_kmin_isa_emulation import cases, DST
cs = cases(int(sys.argv[2]) if len(sys.argv) > 2 else 300)
t = open(sys.argv[1]).read()
parts = re.split(r'\n(?=# \*\*\* IR Dump After )', t)
started = False
for idx, p in enumerate(parts):
    head = p.split('\n', 1)[0]
    m = re.search(r'\(([\w-]+)\) \*\*\*', head)
    name = m.group(1) if m else head[:40]
    if name == 'amdgpu-isel':
        started = True
    if not started or '# Machine code for function' not in p:
        continue
    fn = mir_emu.Function(p.split('# Machine code for function', 1)[1])
    mach = mir_emu.Machine(fn)
    bad = undef = 0; words = [0] * 4; err = None
    for rec, a, want in cs:
        mem = {DST + 4 * k: rec[k] for k in range(4)}
        try:
            st = mach.run({0: DST, 0x20: a}, mem)
        except Exception as e:
            err = type(e).__name__ + ' ' + str(e)[:100] + ' @ ' + str(getattr(mach, 'last', ''))[:100]; break
        got = [mem.get(DST + 4 * k) for k in range(4)]
        if got != want:
            bad += 1
            if None in got: undef += 1
            for k in range(4): words[k] += got[k] != want[k]
    print('%3d %-34s bad %4d undef %4d words %s %s' % (idx, name, bad, undef, words, ('FAULT ' + err) if err else ''), flush=True)
