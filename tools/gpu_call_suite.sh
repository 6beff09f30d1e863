# Full GPU suite, then one driver-style bench line.  usage: tools/gpu_call_suite.sh TAG
set -u
TAG=${1:-r02}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/$TAG/pytest_gpu.log
if grep -q "Timeout +++" gpurun_out/$TAG/pytest_gpu.log; then exit 3; fi
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench_c3.json 2>gpurun_out/$TAG/bench.err || exit $?
cut -c1-300 gpurun_out/$TAG/bench_c3.json
exit $rc
