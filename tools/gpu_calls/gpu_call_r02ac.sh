# 2-player regroup block size: parity, step / rollout A/B at 2^20 lanes.
set -u
mkdir -p gpurun_out/r02ac
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "regroup" > gpurun_out/r02ac/parity.log 2>&1 || { tail -20 gpurun_out/r02ac/parity.log; exit 1; }
tail -1 gpurun_out/r02ac/parity.log
V="COUP_SORT_THREADS=256 COUP_SORT_THREADS=512 COUP_SORT_THREADS=1024"
timeout -k 10 300 python -u tools/ab_step.py --players 2 --obs 0 --rounds 7 $V > gpurun_out/r02ac/ab_step2.log 2>&1 || { tail gpurun_out/r02ac/ab_step2.log; exit 1; }
grep variant gpurun_out/r02ac/ab_step2.log
timeout -k 10 300 python -u tools/ab_step.py --players 2 --obs 0 --rounds 7 --fused 20 $V > gpurun_out/r02ac/ab_rollout2.log 2>&1 || { tail gpurun_out/r02ac/ab_rollout2.log; exit 1; }
grep variant gpurun_out/r02ac/ab_rollout2.log
