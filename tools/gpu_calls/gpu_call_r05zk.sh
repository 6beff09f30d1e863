#!/bin/bash
# Round 5, VERDICT r4 item 1: round 4's k_min<0> defect with chosen <2 x i32>
# phis split into i32 pairs (tools/kmin_phi_split.sh), each code object run on
# the reproducer's 20,000 cases against the per-lane rules.
set -u
D=gpurun_out/r05zk
mkdir -p $D
timeout -k 10 300 build/w3phi/w3_module_check 20000 build/w3phi/kmin_none_O3.co $(ls build/w3phi/phisplit/kmin_phi_*.co) > $D/kmin_phis.json 2>&1 || { tail -5 $D/kmin_phis.json; exit 1; }
python3 -c "
import json; d=json.load(open('$D/kmin_phis.json'))
for k,v in d['modules'].items(): print(k.split('/')[-1], v['mismatch'], v['by_word'])"
