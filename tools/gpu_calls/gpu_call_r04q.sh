# Round 4, seventeenth call: shapes of the split observation writer
# (COUP_OBS_SPLIT 3-7: two threads decode a lane's rows; 64-512 threads per
# block, 1-2 passes) -- equality tests, then the c3-size A/B.
set -u
D=gpurun_out/r04q
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_obs_split.py -x -q --timeout 300 --timeout-method thread > $D/pytest_split.log 2>&1 || { tail -60 $D/pytest_split.log; exit 1; }
tail -2 $D/pytest_split.log
timeout -k 10 200 python -u tools/ab_step.py --batch 1048576 --obs 1 --rounds 7 COUP_OBS_SPLIT=0 COUP_OBS_SPLIT=1 COUP_OBS_SPLIT=3 COUP_OBS_SPLIT=4 COUP_OBS_SPLIT=5 COUP_OBS_SPLIT=6 COUP_OBS_SPLIT=7 COUP_OBS_SPLIT=8 > $D/ab_c3_split.jsonl 2> $D/ab_c3_split.err || { tail -5 $D/ab_c3_split.err; exit 1; }
cut -c1-100 $D/ab_c3_split.jsonl
