# Round 4, third call: the group-Philox step after the PrefRng fix (no LDS
# alloca): its tests, the c2 A/B; the word-3 modules through GlobalISel.
set -u
D=gpurun_out/r04c
mkdir -p $D
timeout -k 10 200 python -u -m pytest tests/test_gpu_step_group.py -x -v --timeout 150 --timeout-method thread > $D/pytest_group.log 2>&1 || { tail -60 $D/pytest_group.log; exit 1; }
tail -2 $D/pytest_group.log
timeout -k 10 90 python -u tools/ab_step.py --batch 65536 --obs 0 --rounds 9 "" COUP_STEP_TPL=1 COUP_STEP_TPL=2 COUP_STEP_TPL=4 > $D/ab_c2_tpl.jsonl 2> $D/ab_c2_tpl.err || { tail -5 $D/ab_c2_tpl.err; exit 1; }
cut -c1-100 $D/ab_c2_tpl.jsonl
timeout -k 10 60 build/w3/w3_module_check 20000 build/w3/kmin_slp_O3gisel.co build/w3/kmin_noslp_O3gisel.co > $D/w3_modules_gisel.json 2> $D/w3_modules_gisel.err || { tail -5 $D/w3_modules_gisel.err; exit 1; }
cut -c1-400 $D/w3_modules_gisel.json
