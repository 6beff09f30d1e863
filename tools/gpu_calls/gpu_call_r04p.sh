# Round 4, sixteenth call: the split observation step (rules step without
# tensors + k_obs_sweep in address order) -- its equality tests against the
# fused step, the headline parity test, then same-process A/B at 2^20, 2^18
# and 2^16 lanes.
set -u
D=gpurun_out/r04p
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_obs_split.py tests/test_gpu_headline.py -x -v --timeout 200 --timeout-method thread > $D/pytest_split.log 2>&1 || { tail -60 $D/pytest_split.log; exit 1; }
tail -3 $D/pytest_split.log
timeout -k 10 150 python -u tools/ab_step.py --batch 1048576 --obs 1 --rounds 9 COUP_OBS_SPLIT=0 COUP_OBS_SPLIT=1 COUP_OBS_SPLIT=2 > $D/ab_c3_split.jsonl 2> $D/ab_c3_split.err || { tail -5 $D/ab_c3_split.err; exit 1; }
cut -c1-110 $D/ab_c3_split.jsonl
timeout -k 10 120 python -u tools/ab_step.py --batch 262144 --obs 1 --rounds 9 COUP_OBS_SPLIT=0 COUP_OBS_SPLIT=1 > $D/ab_2e18_split.jsonl 2> $D/ab_2e18_split.err || { tail -5 $D/ab_2e18_split.err; exit 1; }
cut -c1-110 $D/ab_2e18_split.jsonl
timeout -k 10 120 python -u tools/ab_step.py --batch 65536 --obs 1 --rounds 9 COUP_OBS_SPLIT=0 COUP_OBS_SPLIT=1 > $D/ab_2e16_split.jsonl 2> $D/ab_2e16_split.err || { tail -5 $D/ab_2e16_split.err; exit 1; }
cut -c1-110 $D/ab_2e16_split.jsonl
