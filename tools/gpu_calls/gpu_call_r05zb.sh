# Round 5: the rules trajectories beside the writers once more, with the
# writer's waves at a higher issue priority (s_setprio) and the rules' blocks
# capped per CU by dynamic LDS (measurement build), against the shipped
# one-stream form; plus the step-many product tests.
set -u
D=gpurun_out/r05zb
mkdir -p $D
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_step_many.py > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
export COUP_LIB_PATH=build/variants/libcoup_mi355x.so
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/ab_variants/test_ab_overlap.py -k priority > $D/pytest_ab.log 2>&1 || { tail -40 $D/pytest_ab.log; exit 1; }
tail -2 $D/pytest_ab.log
timeout -k 10 600 python -u tools/pipe_ab.py traj8:COUP_PIPE=1 traj8p:COUP_PIPE=1,COUP_WRITER_PRIO=2 \
  over4:COUP_PIPE=3,COUP_TRAJ_CHUNK=4 over4p:COUP_PIPE=3,COUP_TRAJ_CHUNK=4,COUP_WRITER_PRIO=2 \
  over4pl:COUP_PIPE=3,COUP_TRAJ_CHUNK=4,COUP_WRITER_PRIO=2,COUP_OVERLAP_LDS=98304 \
  over8pl:COUP_PIPE=3,COUP_WRITER_PRIO=2,COUP_OVERLAP_LDS=98304 \
  over8l:COUP_PIPE=3,COUP_OVERLAP_LDS=98304 > $D/pipe_ab.jsonl 2> $D/pipe_ab.err || { tail -20 $D/pipe_ab.err; exit 1; }
cut -c1-120 $D/pipe_ab.jsonl
