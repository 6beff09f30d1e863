# Round 5, VERDICT r4 item 1 on round 4's deterministic k_min<0> defect: the
# SLP IR through llc's late IR passes, scalarized (opt's scalarizer, a
# semantics-preserving split of every vector op) right before each of them
# and right before instruction selection, then compiled from that point on
# (-start-before); the unscalarized IR from the same points as controls.
set -u
D=gpurun_out/r05w
mkdir -p $D
timeout -k 10 600 build/w3phi/w3_module_check 20000 build/w3phi/kmin_none_O3.co build/w3phi/kmin_pre_isel_ir.co build/w3phi/kmin_pre_isel_scal.co $(ls build/w3phi/kmin_scalbefore_*.co build/w3phi/kmin_vecbefore_*.co) > $D/kmin_stages.json 2>&1 || { tail -5 $D/kmin_stages.json; exit 1; }
python3 -c "
import json; d=json.load(open('$D/kmin_stages.json'))
for k,v in d['modules'].items(): print(k.split('/')[-1], v['mismatch'], v['by_word'])"
