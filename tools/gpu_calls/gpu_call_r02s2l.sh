# Round 2, session 2: 2-player regrouped trajectory -- parity, then traj_ab at 2^20 and 2^16 (2 players).
set -u
D=gpurun_out/r02s2l
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_trajectory.py -x -v --timeout 150 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 300 python -u tools/traj_ab.py --players 2 > $D/traj_ab.jsonl 2>$D/err.log || { tail $D/err.log; exit 1; }
COUP_REGROUP=0 timeout -k 10 300 python -u tools/traj_ab.py --players 2 >> $D/traj_ab.jsonl 2>>$D/err.log || { tail $D/err.log; exit 1; }
cat $D/traj_ab.jsonl
