# Round 3: reference-faithful unchecked ApplyAction (COUP_SLOT_UNCHECKED /
# COUP_FLAG_UNCHECKED): the new tests first, then the whole GPU suite, smoke()
# and the default bench line (the uniform kernels must be unchanged).
set -u
D=gpurun_out/r03p
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_unchecked.py tests/test_policy_prefixes.py tests/test_rust_abi.py tests/test_gpu_cpp_api.py -m gpu -x -v --timeout 200 --timeout-method thread > $D/pytest_new.log 2>&1 || { tail -60 $D/pytest_new.log; exit 1; }
tail -2 $D/pytest_new.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $D/bench_default.json 2> $D/bench_default.err || { tail -5 $D/bench_default.err; exit 1; }
cut -c1-200 $D/bench_default.json
