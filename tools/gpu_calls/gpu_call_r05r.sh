# Round 5: the rules trajectory's block / register-budget shapes (measurement
# build: equality, then the same-process A/B), then the c2 and c4 profiles of
# coup_step_many's one-launch trajectory form (tools/profile_gpu.sh).
set -u
D=gpurun_out/r05r
mkdir -p $D
export COUP_LIB_PATH=build/variants/libcoup_mi355x.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/ab_variants/test_ab_overlap.py -k shapes > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 400 python -u tools/pipe_ab.py serial:COUP_PIPE=0 traj8:COUP_PIPE=1 t512w8:COUP_MANY_SHAPE=1 t512w6:COUP_MANY_SHAPE=2 t256w8:COUP_MANY_SHAPE=3 t1024w4:COUP_MANY_SHAPE=4 > $D/pipe_ab.jsonl 2> $D/pipe_ab.err || { tail -20 $D/pipe_ab.err; exit 1; }
cat $D/pipe_ab.jsonl | cut -c1-120
unset COUP_LIB_PATH
for c in c2 c4; do
  timeout -k 10 900 bash tools/profile_gpu.sh r05 $c > gpurun_out/profile_r05_$c.log 2>&1 || { tail -30 gpurun_out/profile_r05_$c.log; exit 1; }
  tail -2 gpurun_out/profile_r05_$c.log
done
