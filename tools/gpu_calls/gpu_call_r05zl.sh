#!/bin/bash
# Round 5, VERDICT r4 item 1: round 4's k_min<0> defect named on the CPU
# (tools/kmin_ir_bisect.py: structurizecfg) -- the same code objects on the
# GPU: the -O3 control, the build with -structurizecfg-skip-uniform-regions,
# the IR scalarized right before / right after structurizecfg, and the build
# without amdgpu-codegenprepare's large-PHI splitting; 20,000 cases each.
set -u
D=gpurun_out/r05zl
mkdir -p $D
timeout -k 10 300 build/w3phi/w3_module_check 20000 build/w3phi/kmin_none_O3.co build/w3phi/irbisect/kmin_skipuniform.co build/w3phi/irbisect/kmin_vec_through_unify-loop-exits_scal.co build/w3phi/irbisect/kmin_vec_through_structurizecfg_scal.co build/w3phi/irbisect/kmin_nobreakphis.co > $D/kmin_structurizer.json 2>&1 || { tail -5 $D/kmin_structurizer.json; exit 1; }
python3 -c "
import json; d=json.load(open('$D/kmin_structurizer.json'))
for k,v in d['modules'].items(): print(k.split('/')[-1], v['mismatch'], v['by_word'])"
