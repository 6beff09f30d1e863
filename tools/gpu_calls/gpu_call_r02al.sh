# Packed int32 collective payload: 2-process HIP tests and the default bench line.
set -u
mkdir -p gpurun_out/r02al
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_dist.py > gpurun_out/r02al/dist.log 2>&1 || { tail -20 gpurun_out/r02al/dist.log; exit 1; }
tail -1 gpurun_out/r02al/dist.log
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02al/bench.json 2>gpurun_out/r02al/bench.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/r02al/bench.json').read().splitlines()[-1]); print(d['value'], d['episodes'], d['roofline']['kernel_ms'])"
