# Round 5: the rules trajectory with its outputs staged by lane
# (COUP_MANY_STAGE) and longer chunks (COUP_TRAJ_CHUNK 16 / 20): equality
# tests, then the same-process A/B.
set -u
D=gpurun_out/r05m
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_step_many.py > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
timeout -k 10 400 python -u tools/pipe_ab.py > $D/pipe_ab.jsonl 2> $D/pipe_ab.err || { tail -20 $D/pipe_ab.err; exit 1; }
cat $D/pipe_ab.jsonl
