"""Which <2 x i32> value of the SLP IR does the AMDGPU backend lower wrong?
  Investigation tool, not product
code.

    python tools/w3_phi_variants.py   # writes build/w3phi/*.ll, *.co, *.s and a manifest

Starts from the committed k_min<0> IR after SLP (profiles/r04/codegen/
kmin_slp.ll, wrong through llc at every optimisation level, right once opt's
scalarizer splits every vector operation), names its values (instnamer),
then rewrites chosen <2 x i32> phi nodes as two i32 phi nodes -- the
incoming vectors split by extractelement at the end of each predecessor,
the pair rebuilt by insertelement after the block's phis, so every other
vector operation stays as SLP left it.  One variant per phi and one with
all of them; each through llc -O0 and -O3 into a code object that
tools/w3_module_check.hip runs on the reproducer's cases on the GPU.
"""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
SRC = os.path.join(ROOT, "profiles", "r04", "codegen", "kmin_slp.ll")
OUT = os.path.join(ROOT, "build", "w3phi")  # travels to the GPU box (build/w3 does not)
TRIPLE = ["-mtriple=amdgcn-amd-amdhsa", "-mcpu=gfx950"]

PHI = re.compile(r"^  (%[\w.]+) = phi <2 x i32> (.*)$")
INC = re.compile(r"\[ ([^,\]]+), (%[\w.]+) \]")
CONST = re.compile(r"^<i32 (-?\d+), i32 (-?\d+)>$")


def elements(v):
    """The two i32 operands of incoming vector value v: constants inline,
    else None (extract in the predecessor)."""
    v = v.strip()
    m = CONST.match(v)
    if m:
        return m.group(1), m.group(2)
    if v.startswith("splat (i32 "):
        c = v[len("splat (i32 "):-1]
        return c, c
    if v in ("zeroinitializer",):
        return "0", "0"
    if v in ("poison", "undef"):
        return v, v
    return None


def scalarize(lines, names):
    """Rewrite the <2 x i32> phis named in `names` (e.g. {"%i810"})."""
    block_of_line, label_line = {}, {}
    cur = None
    for k, ln in enumerate(lines):
        m = re.match(r"^([\w.]+):", ln)
        if m:
            cur = "%" + m.group(1)
            label_line[cur] = k
        block_of_line[k] = cur
    inserts_before_term = {}  # pred block -> lines
    after_phis = {}           # block -> lines
    out_lines = list(lines)
    for k, ln in enumerate(lines):
        m = PHI.match(ln)
        if not m or m.group(1) not in names:
            continue
        name, body = m.group(1), m.group(2)
        base = name[1:]
        a_inc, b_inc = [], []
        for val, pred in INC.findall(body):
            el = elements(val)
            if el is None:
                e0, e1 = f"%{base}.x0.{pred[1:]}", f"%{base}.x1.{pred[1:]}"
                inserts_before_term.setdefault(pred, []).extend([
                    f"  {e0} = extractelement <2 x i32> {val}, i64 0",
                    f"  {e1} = extractelement <2 x i32> {val}, i64 1"])
                el = (e0, e1)
            a_inc.append(f"[ {el[0]}, {pred} ]")
            b_inc.append(f"[ {el[1]}, {pred} ]")
        out_lines[k] = (f"  %{base}.s0 = phi i32 {', '.join(a_inc)}\n"
                        f"  %{base}.s1 = phi i32 {', '.join(b_inc)}")
        after_phis.setdefault(block_of_line[k], []).extend([
            f"  %{base}.v0 = insertelement <2 x i32> poison, i32 %{base}.s0, i64 0",
            f"  {name} = insertelement <2 x i32> %{base}.v0, i32 %{base}.s1, i64 1"])
    # place the inserts: extracts before each predecessor's terminator, the
    # rebuilt vectors after the last phi of their block
    term = re.compile(r"^  (br|switch|ret|unreachable)\b")
    result = []
    k = 0
    n = len(out_lines)
    while k < n:
        ln = out_lines[k]
        blk = block_of_line.get(k)
        if term.match(ln) and blk in inserts_before_term:
            result.extend(inserts_before_term.pop(blk))
        result.append(ln)
        if blk in after_phis and " = phi " in ln and not (k + 1 < n and " = phi " in out_lines[k + 1]):
            result.extend(after_phis.pop(blk))
        k += 1
    assert not inserts_before_term and not after_phis, (inserts_before_term.keys(), after_phis.keys())
    return result


def run(cmd):
    subprocess.run(cmd, check=True)


def main():
    os.makedirs(OUT, exist_ok=True)
    named = os.path.join(OUT, "kmin_slp_named.ll")
    run([os.path.join(LLVM, "opt"), "-passes=instnamer", SRC, "-S", "-o", named])
    with open(named) as f:
        lines = f.read().split("\n")
    phis = [PHI.match(ln).group(1) for ln in lines if PHI.match(ln)]
    variants = {"none": set(), "all": set(phis)}
    for p in phis:
        variants["only_" + p[1:]] = {p}
    manifest = {"phis": phis, "variants": {}}
    for vname, names in variants.items():
        ll = os.path.join(OUT, f"kmin_{vname}.ll")
        with open(ll, "w") as f:
            f.write("\n".join(scalarize(lines, names)))
        run([os.path.join(LLVM, "opt"), "-passes=verify", ll, "-disable-output"])
        for o in ("0", "3"):
            obj = os.path.join(OUT, f"kmin_{vname}_O{o}.o")
            co = os.path.join(OUT, f"kmin_{vname}_O{o}.co")
            run([os.path.join(LLVM, "llc"), f"-O{o}"] + TRIPLE + ["-filetype=obj", ll, "-o", obj])
            run([os.path.join(LLVM, "ld.lld"), "-shared", obj, "-o", co])
            run([os.path.join(LLVM, "llc"), f"-O{o}"] + TRIPLE + [ll, "-o", co[:-3] + ".s"])
            os.remove(obj)
            manifest["variants"][f"{vname}_O{o}"] = {"scalarized": sorted(names), "co": os.path.relpath(co, ROOT)}
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(json.dumps(manifest, indent=1))


if __name__ == "__main__":
    sys.exit(main())
