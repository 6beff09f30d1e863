# Round 4, twenty-fifth call: the split c3 step replayed from a HIP graph
# (the default) against K eager launches, same box, two lines each.
set -u
D=gpurun_out/r04y
mkdir -p $D
for g in on off on off; do
  timeout -k 10 300 python -u bench.py --graph $g --no-cpu-baseline > $D/bench_$g.json 2> $D/bench_$g.err || { tail -20 $D/bench_$g.err; exit 1; }
  python -c "import json; d=json.loads(open('$D/bench_$g.json').readline()); print('$g', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
