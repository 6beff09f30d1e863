# Round 5, VERDICT r4 item 1: which llc stage brings the uint2-prefix defect
# -- the reproducer's own kernels, then k_sweep_uint2<512, 2> / k_sweep_rows
# <512, 2> from the device IR through llc -O0, -O3, GlobalISel and every
# opt-bisect limit over llc's 135 optional passes (tools/info_modules.sh).
set -u
D=gpurun_out/r05o
mkdir -p $D
timeout -k 10 120 build/info_prefix_repro 20000 > $D/repro.jsonl 2>&1 || { cat $D/repro.jsonl; exit 1; }
cat $D/repro.jsonl
timeout -k 10 600 build/info_prefix_repro 20000 $(ls build/infomod/*.co) > $D/modules.jsonl 2>&1 || { tail -5 $D/modules.jsonl; exit 1; }
python3 -c "
import json
for l in open('$D/modules.jsonl'):
    d=json.loads(l); print(d['kernel'].split('/')[-1], d['mismatching_lanes'])" | awk '{printf \"%s %s %s | \", \$1, \$2, \$3} END {print \"\"}'
