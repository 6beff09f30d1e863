# Round 4, eighth call: the 6-player step storing its non-reset lanes before
# the reset phase (COUP_NP_EARLY_STORE): its invariance test, then a
# same-process A/B against the shipped form at 2^20 lanes.
set -u
D=gpurun_out/r04h
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_nplayer.py -x -q -k "reset_schedule" --timeout 200 --timeout-method thread > $D/pytest_np.log 2>&1 || { tail -40 $D/pytest_np.log; exit 1; }
tail -2 $D/pytest_np.log
timeout -k 10 150 python -u tools/ab_step.py --players 6 --obs 0 --rounds 9 "" COUP_NP_EARLY_STORE=1 > $D/ab_np_early.jsonl 2> $D/ab_np_early.err || { tail -5 $D/ab_np_early.err; exit 1; }
cut -c1-120 $D/ab_np_early.jsonl
