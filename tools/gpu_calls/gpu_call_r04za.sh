# Round 4, after the final call: plain instead of non-temporal stores in the
# split writers (the probe had plain ahead at 4 passes) -- equality tests,
# then same-process A/B at the c3 and c3i sizes.
set -u
D=gpurun_out/r04za
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_obs_split.py -x -q --timeout 800 --timeout-method thread > $D/pytest_split.log 2>&1 || { tail -60 $D/pytest_split.log; exit 1; }
tail -2 $D/pytest_split.log
timeout -k 10 200 python -u tools/ab_step.py --batch 1048576 --obs 1 --rounds 9 COUP_OBS_SPLIT=0 "" COUP_OBS_SPLIT=18 COUP_OBS_SPLIT=19 > $D/ab_c3_plain.jsonl 2> $D/ab_c3_plain.err || { tail -5 $D/ab_c3_plain.err; exit 1; }
cut -c1-100 $D/ab_c3_plain.jsonl
timeout -k 10 300 python -u tools/ab_step.py --batch 262144 --obs 0 --info 1 --rounds 7 COUP_INFO_SPLIT=0 "" COUP_INFO_SPLIT=6 > $D/ab_c3i_plain.jsonl 2> $D/ab_c3i_plain.err || { tail -5 $D/ab_c3i_plain.err; exit 1; }
cut -c1-100 $D/ab_c3i_plain.jsonl
