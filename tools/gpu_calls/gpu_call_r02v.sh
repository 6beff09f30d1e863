# Why bench c4 (graph) reads 39 us where ab_step (eager) reads 36 us.
set -u
mkdir -p gpurun_out/r02v
for g in on off; do
  timeout -k 10 200 python -u bench.py --config c4 --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --graph $g > gpurun_out/r02v/bench_c4_$g.json 2> gpurun_out/r02v/bench_c4_$g.err || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['roofline']['kernel_ms'])" gpurun_out/r02v/bench_c4_$g.json
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r02v/prof -o run --output-format csv -- python3 bench.py --config c4 --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02v/prof.log 2>&1 || exit $?
find gpurun_out/r02v/prof -name '*kernel_stats.csv' -exec cut -c1-160 {} \;
