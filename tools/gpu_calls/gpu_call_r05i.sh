# Round 5: the overlapped rules-trajectory form (COUP_PIPE=3: the rules
# trajectory of chunk c + 1 on a second stream beside chunk c's writers) --
# its equality tests, then a same-process A/B against the serial and
# one-stream forms.
set -u
D=gpurun_out/r05i
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_step_many.py > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
timeout -k 10 400 python -u tools/pipe_ab.py > $D/pipe_ab.jsonl 2> $D/pipe_ab.err || { tail -20 $D/pipe_ab.err; exit 1; }
cat $D/pipe_ab.jsonl
