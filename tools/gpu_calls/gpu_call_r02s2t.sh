# Round 2, session 2: coup_slot_op and coup_slot_ops answered through host-polled completion flags instead of a stream
# synchronisation -- the per-game State suites (Python, C++, Rust ABI, codegen reproducer), then the facade latency.
set -u
D=gpurun_out/r02s2t
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_slot_pool.py tests/test_gpu_facade.py tests/test_gpu_cpp_api.py tests/test_rust_abi.py tests/test_gpu_codegen_hazard.py tests/test_gpu_vector_env.py tests/test_gpu_rule_branches.py -x -v --timeout 200 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 400 python -u tools/facade_latency.py > $D/facade_latency.json 2> $D/facade.err || { tail -3 $D/facade.err; exit 1; }
python -c "import json; d=json.load(open('$D/facade_latency.json')); print({k: v for k, v in d.items() if k.startswith(('pool', 'rl_', 'children_n1_', 'children_n7_'))})"
