set -u
mkdir -p gpurun_out/r02a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r02a/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/r02a/pytest_gpu.log
if grep -q "Timeout +++" gpurun_out/r02a/pytest_gpu.log; then echo "pytest timeout: stopping"; exit 3; fi
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
bash tools/profile_gpu.sh r02 c3 --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02a/profile.log 2>&1
prc=$?
tail -30 gpurun_out/r02a/profile.log
exit $(( rc > prc ? rc : prc ))
