# Round 2, session 2: register budget of the regrouped 6-player trajectory (64 VGPRs with 42 spilled, vs 80 VGPRs
# without spills at fewer waves) -- parity of the variants, then traj_ab alternating processes.
set -u
D=gpurun_out/r02s2x
mkdir -p $D
COUP_TRAJ_WAVES=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_trajectory.py -x -q --timeout 150 --timeout-method thread -k "6p or players" > $D/pytest_w4.log 2>&1 || { tail -20 $D/pytest_w4.log; exit 1; }
COUP_TRAJ_WAVES=6 COUP_NP_SORT_THREADS=512 timeout -k 10 300 python -u -m pytest tests/test_gpu_trajectory.py -x -q --timeout 150 --timeout-method thread -k "6p or players" > $D/pytest_w6.log 2>&1 || { tail -20 $D/pytest_w6.log; exit 1; }
tail -1 $D/pytest_w4.log $D/pytest_w6.log
for i in 1 2 3; do
  for v in "8 1024" "4 1024" "6 512" "8 512"; do
    set -- $v
    COUP_TRAJ_WAVES=$1 COUP_NP_SORT_THREADS=$2 timeout -k 10 300 python -u tools/traj_ab.py --players 6 --rounds 3 2>/dev/null | grep '"trajectory"' | sed "s/^/waves=$1 block=$2 /" >> $D/traj_waves.log || exit 1
  done
done
cat $D/traj_waves.log
