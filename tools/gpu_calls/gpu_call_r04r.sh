# Round 4, eighteenth call: more shapes of the row-decoding split writer
# around the fastest one (256 threads x 2 passes): equality tests, then the
# c3-size A/B (same process).
set -u
D=gpurun_out/r04r
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_gpu_obs_split.py -x -q --timeout 400 --timeout-method thread > $D/pytest_split.log 2>&1 || { tail -60 $D/pytest_split.log; exit 1; }
tail -2 $D/pytest_split.log
timeout -k 10 200 python -u tools/ab_step.py --batch 1048576 --obs 1 --rounds 7 COUP_OBS_SPLIT=0 COUP_OBS_SPLIT=4 COUP_OBS_SPLIT=8 COUP_OBS_SPLIT=9 COUP_OBS_SPLIT=10 COUP_OBS_SPLIT=11 COUP_OBS_SPLIT=12 COUP_OBS_SPLIT=13 > $D/ab_c3_split.jsonl 2> $D/ab_c3_split.err || { tail -5 $D/ab_c3_split.err; exit 1; }
cut -c1-100 $D/ab_c3_split.jsonl
