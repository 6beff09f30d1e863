set -u
mkdir -p gpurun_out/r02c
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "rust_abi or slot_pool or cpp_api or slot_ops" > gpurun_out/r02c/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/r02c/pytest_gpu.log
if grep -q "Timeout +++" gpurun_out/r02c/pytest_gpu.log; then exit 3; fi
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/facade_latency.py > gpurun_out/r02c/facade_latency.json 2>gpurun_out/r02c/facade.err || exit $?
cat gpurun_out/r02c/facade_latency.json
exit $rc
