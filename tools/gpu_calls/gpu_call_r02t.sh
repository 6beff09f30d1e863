# Regroup block size A/B: 6-player step and rollout, 3/4-player step; parity.
set -u
mkdir -p gpurun_out/r02t
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nplayer.py > gpurun_out/r02t/nplayer.log 2>&1 || { tail -20 gpurun_out/r02t/nplayer.log; exit 1; }
tail -1 gpurun_out/r02t/nplayer.log
V="COUP_NP_SORT_THREADS=256 COUP_NP_SORT_THREADS=512 COUP_NP_SORT_THREADS=1024"
timeout -k 10 300 python -u tools/ab_step.py --players 6 --obs 0 --rounds 7 --fused 20 $V > gpurun_out/r02t/ab_rollout6.log 2>&1 || { tail gpurun_out/r02t/ab_rollout6.log; exit 1; }
grep variant gpurun_out/r02t/ab_rollout6.log
for p in 3 4; do
  timeout -k 10 300 python -u tools/ab_step.py --players $p --obs 0 --rounds 7 $V > gpurun_out/r02t/ab_step$p.log 2>&1 || { tail gpurun_out/r02t/ab_step$p.log; exit 1; }
  grep variant gpurun_out/r02t/ab_step$p.log
done
