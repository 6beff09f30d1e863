# Round 5, VERDICT r4 item 1, continued: the uint2-prefix mismatch counts vary
# run to run for one code object (r05o) -- a timing effect, not a fixed
# miscompiled value.  Each code object three times: llc -O3, -O3 with
# s_nop 15 before every instruction (and with every s_waitcnt zero), the
# bisect limits either side of the uint2 kernel's dead-mi-elimination (95 /
# 96) and of the rows kernel's passes (35 / 36, 58 / 59); k_min<0> with
# s_nop 15.
set -u
D=gpurun_out/r05p
mkdir -p $D
M="build/infomod/O3.co build/infomod/O3snop15.co build/infomod/O3snop15waitzero.co build/infomod/bisect_095.co build/infomod/bisect_096.co build/infomod/bisect_035.co build/infomod/bisect_036.co build/infomod/bisect_058.co build/infomod/bisect_059.co"
for i in 1 2 3; do
  timeout -k 10 600 build/info_prefix_repro 20000 $M > $D/modules_$i.jsonl 2>&1 || { tail -5 $D/modules_$i.jsonl; exit 1; }
  python3 -c "
import json
print(' | '.join('%s %s' % (json.loads(l)['kernel'].split('/')[-1], json.loads(l)['mismatching_lanes']) for l in open('$D/modules_$i.jsonl')))"
done
timeout -k 10 300 build/w3phi/w3_module_check 20000 build/w3phi/kmin_none_O3.co build/w3phi/kmin_slp_O3snop15.co > $D/kmin.json 2>&1 || { tail -5 $D/kmin.json; exit 1; }
python3 -c "
import json; d=json.load(open('$D/kmin.json'))
for k,v in d['modules'].items(): print(k, v['mismatch'], v['by_word'])"
