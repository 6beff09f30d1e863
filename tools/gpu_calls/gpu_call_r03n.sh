# Round 3: per-wave bin prefix (wave_bins_below) in the N-player sorted step,
# rollout and trajectory kernels; N-player parity, then same-process A/B of
# the prefix forms (COUP_NP_SCAN=0/1) for the 6-player step, trajectory and rollout.
set -u
D=gpurun_out/r03n
mkdir -p $D
timeout -k 10 700 python -u -m pytest tests/test_gpu_nplayer.py tests/test_gpu_trajectory.py -m gpu -x -v --timeout 200 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 300 python -u tools/ab_step.py --players 6 --obs 0 --rounds 9 --steps 20 COUP_NP_SCAN=0 COUP_NP_SCAN=1 > $D/ab_np_scan.jsonl 2> $D/ab_np.err || { tail -20 $D/ab_np.err; exit 1; }
cat $D/ab_np_scan.jsonl
timeout -k 10 300 python -u tools/traj_ab.py --players 6 --steps 100 --rounds 7 > $D/traj_ab_6p.jsonl 2> $D/traj_ab.err || { tail -20 $D/traj_ab.err; exit 1; }
cat $D/traj_ab_6p.jsonl
