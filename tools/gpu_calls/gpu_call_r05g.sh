# Round 5: the driver's c3 bench line with the power warm-up (twice, and once
# with it off), then the whole GPU suite and the other configs (r05b).
set -u
D=gpurun_out/r05g
mkdir -p $D
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > $D/bench_c3_$i.json 2> $D/bench_c3_$i.err || { tail -20 $D/bench_c3_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_c3_$i.json')); r=d['roofline']; print('c3', d['value'], r['frac'], r['kernel_ms'], r.get('store_ceiling_ms'), d['power_warm'])"
done
timeout -k 10 300 python -u bench.py --power-warm-ms 0 > $D/bench_c3_nowarm.json 2> $D/bench_c3_nowarm.err || { tail -20 $D/bench_c3_nowarm.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_c3_nowarm.json')); r=d['roofline']; print('c3 no warm', d['value'], r['frac'], r['kernel_ms'], r.get('store_ceiling_ms'))"
bash tools/gpu_calls/gpu_call_r05b.sh
