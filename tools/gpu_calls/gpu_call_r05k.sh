# Round 5: coup_step_many's fused trajectory (COUP_PIPE=4: one launch, the
# rules kernel writing every step's observations in address order block by
# block) -- equality tests (product + measurement-build shapes), then the
# same-process A/B against the serial and rules-trajectory forms.
set -u
D=gpurun_out/r05k
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_step_many.py > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
COUP_LIB_PATH=build/variants/libcoup_mi355x.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/ab_variants/test_ab_overlap.py -k fused > $D/pytest_ab.log 2>&1 || { tail -40 $D/pytest_ab.log; exit 1; }
tail -3 $D/pytest_ab.log
COUP_LIB_PATH=build/variants/libcoup_mi355x.so timeout -k 10 400 python -u tools/pipe_ab.py > $D/pipe_ab.jsonl 2> $D/pipe_ab.err || { tail -20 $D/pipe_ab.err; exit 1; }
cat $D/pipe_ab.jsonl
