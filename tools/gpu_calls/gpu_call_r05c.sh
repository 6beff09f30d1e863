# Round 5: the section-12 codegen investigation -- the
# uint2-prefix reproducer of round 4's k_info_sweep sighting, and k_min<0>'s
# SLP IR with single <2 x i32> phis split into i32 pairs (tools/
# w3_phi_variants.py), each variant's code object on the reproducer's cases.
set -u
D=gpurun_out/r05c
mkdir -p $D
timeout -k 10 120 build/info_prefix_repro 100000 > $D/info_prefix_repro.jsonl 2>&1 || { cat $D/info_prefix_repro.jsonl; exit 1; }
cat $D/info_prefix_repro.jsonl
timeout -k 10 300 build/w3phi/w3_module_check 20000 $(ls build/w3phi/*.co) > $D/w3_phi_variants.json 2>&1 || { tail -5 $D/w3_phi_variants.json; exit 1; }
python3 -c "
import json; d=json.load(open('$D/w3_phi_variants.json'))
for k,v in d['modules'].items(): print(k, v['mismatch'], v['by_word'])"
