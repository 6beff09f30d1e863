# Round 3: the 6-player step with two groups per block and the next group's
# records loaded ahead (COUP_NP_GROUPS=2): invariance tests, then a
# same-process A/B against one group per block.
set -u
D=gpurun_out/r03u
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_nplayer.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 300 python -u tools/ab_step.py --players 6 --obs 0 --rounds 9 --steps 20 COUP_NP_GROUPS=1 COUP_NP_GROUPS=2 > $D/ab_groups.jsonl 2> $D/ab.err || { tail -20 $D/ab.err; exit 1; }
cat $D/ab_groups.jsonl
