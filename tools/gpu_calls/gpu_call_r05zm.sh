# Round 5, end of session: the k_min<0> structurizer code objects on the GPU
# (tools/gpu_calls/gpu_call_r05zl.sh), then the whole GPU suite on the final
# tree, smoke() and the driver's default line twice.
set -u
D=gpurun_out/r05zm
mkdir -p $D
bash tools/gpu_calls/gpu_call_r05zl.sh || exit 1
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > $D/bench_default_$i.json 2> $D/bench_default_$i.err || { tail -20 $D/bench_default_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_default_$i.json')); r=d['roofline']; print('c3', d['value'], r['frac'], r['kernel_ms'], r.get('store_ceiling_ms'), d['power_warm'])"
done
