# Round 5: the c2 line with and without the power warm-up, alternating on one
# box (r05h's c2 line after the warm-up measured 12.9 us per step against
# round 4's 7.6-7.8), then the default c3 line.
set -u
D=gpurun_out/r05l
mkdir -p $D
for i in 1 2; do
  for w in 0 40; do
    timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline --power-warm-ms $w > $D/bench_c2_w${w}_$i.json 2> $D/bench_c2_w${w}_$i.err || { tail -20 $D/bench_c2_w${w}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/bench_c2_w${w}_$i.json')); r=d['roofline']; print('c2 warm $w', d['value'], r['kernel_ms'], d['power_warm'])"
  done
done
timeout -k 10 300 python -u bench.py > $D/bench_c3.json 2> $D/bench_c3.err || { tail -20 $D/bench_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_c3.json')); r=d['roofline']; print('c3', d['value'], r['frac'], r['kernel_ms'], d['power_warm'])"
