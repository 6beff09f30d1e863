# Round 2, session 2: every bench config on one box, driver-style K = 20 for the per-step configs and K = 100 for
# the fused ones, for DESIGN's measured table.
set -u
D=gpurun_out/r02s2s
mkdir -p $D
for a in "c3 20" "c3i 20" "c2 20" "c2r 100" "c2t 100" "c4 20" "c4r 100" "c4t 100"; do
  set -- $a
  timeout -k 10 300 python -u bench.py --config $1 --steps $2 --warmup 5 > $D/bench_$1.json 2> $D/bench_$1.err || { tail $D/bench_$1.err; exit 1; }
  python -c "import json; d=json.load(open('$D/bench_$1.json')); r=d['roofline']; c=d.get('cpu_baseline',{}); print('$1', '%.3e' % d['value'], round(r['kernel_ms']*1e3/d['config']['fused_steps_per_launch'],2), 'us/step frac', round(r['frac'],3), 'ceil', r['store_ceiling_ms'], 'cpu', '%.2e' % c.get('value',0), c.get('all_cores',{}).get('value'))"
done
