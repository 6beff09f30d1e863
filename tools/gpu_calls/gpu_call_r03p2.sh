# Round 3: debug the unchecked SyncVectorEnv test (loop envs on the launch path).
set -u
D=gpurun_out/r03p2
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_unchecked.py -m gpu -x -v --timeout 200 --timeout-method thread -k sync_vector > $D/pytest.log 2>&1 || { grep -E "^E|Failed|t=" $D/pytest.log | head -20; exit 1; }
tail -2 $D/pytest.log
