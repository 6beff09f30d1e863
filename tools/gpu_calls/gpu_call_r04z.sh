# Round 4, twenty-sixth call: the driver's default c3 line with the split
# step (default) and with the fused step (COUP_OBS_SPLIT=0), alternating on
# one box.
set -u
D=gpurun_out/r04z
mkdir -p $D
for v in split fused split fused; do
  if [ $v = fused ]; then export COUP_OBS_SPLIT=0; else unset COUP_OBS_SPLIT; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $D/bench_$v.json 2> $D/bench_$v.err || { tail -20 $D/bench_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('$D/bench_$v.json').readline()); print('$v', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['kernel'])"
done
