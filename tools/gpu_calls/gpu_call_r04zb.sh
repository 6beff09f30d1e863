# Round 4: the launcher form of the driver's scaling run with the split c3
# step -- bench.py --gpus 2 starting its own ranks (gloo, both on the one
# GPU of this box), after one plain line.
set -u
D=gpurun_out/r04zb
mkdir -p $D
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline > $D/bench_2ranks.json 2> $D/bench_2ranks.err || { tail -30 $D/bench_2ranks.err; exit 1; }
python -c "import json; d=json.loads(open('$D/bench_2ranks.json').readline()); print(d['n_gpus'], d['value'], d['config']['parallelism'], d['roofline']['kernel'], d['episodes']['finished'])"
