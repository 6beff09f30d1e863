# Round 4, nineteenth call: the row-decoding split writer at 512-1024
# threads per block (the fastest so far: 512 x 2 passes) -- equality tests,
# then the c3-size A/B.
set -u
D=gpurun_out/r04s
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_obs_split.py -x -q --timeout 500 --timeout-method thread > $D/pytest_split.log 2>&1 || { tail -60 $D/pytest_split.log; exit 1; }
tail -2 $D/pytest_split.log
timeout -k 10 200 python -u tools/ab_step.py --batch 1048576 --obs 1 --rounds 9 COUP_OBS_SPLIT=0 COUP_OBS_SPLIT=11 COUP_OBS_SPLIT=14 COUP_OBS_SPLIT=15 COUP_OBS_SPLIT=16 COUP_OBS_SPLIT=17 > $D/ab_c3_split.jsonl 2> $D/ab_c3_split.err || { tail -5 $D/ab_c3_split.err; exit 1; }
cut -c1-100 $D/ab_c3_split.jsonl
