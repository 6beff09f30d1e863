# Round 2, session 2: regrouped 6-player trajectory with a wave-0 scan of the bins (COUP_TRAJ_SCAN=1) vs per-thread
# bins_below -- parity of the scan variant, then traj_ab for both, alternating processes.
set -u
D=gpurun_out/r02s2q
mkdir -p $D
COUP_TRAJ_SCAN=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_trajectory.py -x -v --timeout 150 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
for i in 1 2 3; do
  for v in 0 1; do
    COUP_TRAJ_SCAN=$v timeout -k 10 300 python -u tools/traj_ab.py --players 6 --rounds 3 2>/dev/null | grep '"trajectory"' | sed "s/^/scan=$v /" >> $D/traj_scan.log || exit 1
  done
done
cat $D/traj_scan.log
