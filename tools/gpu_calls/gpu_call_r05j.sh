# Round 5: the overlapped rules-trajectory forms in the measurement build
# (unmasked and CU-masked second streams): their equality tests, then a
# same-process A/B of graph replays and of eager calls (a graph replay may
# drop a stream's CU mask).
set -u
D=gpurun_out/r05j
mkdir -p $D
export COUP_LIB_PATH=build/variants/libcoup_mi355x.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/ab_variants/test_ab_overlap.py > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
timeout -k 10 400 python -u tools/pipe_ab.py > $D/pipe_ab_graph.jsonl 2> $D/pipe_ab_graph.err || { tail -20 $D/pipe_ab_graph.err; exit 1; }
cat $D/pipe_ab_graph.jsonl
timeout -k 10 400 python -u tools/pipe_ab.py --eager > $D/pipe_ab_eager.jsonl 2> $D/pipe_ab_eager.err || { tail -20 $D/pipe_ab_eager.err; exit 1; }
cat $D/pipe_ab_eager.jsonl
