# c4 kernel durations: ab_step (eager, 512) vs bench (graph) under rocprof.
set -u
mkdir -p gpurun_out/r02x
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r02x/ab -o run --output-format csv -- python3 tools/ab_step.py --players 6 --obs 0 --rounds 3 COUP_NP_SORT_THREADS=512 > gpurun_out/r02x/ab.log 2>&1 || exit $?
grep variant gpurun_out/r02x/ab.log
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r02x/bench -o run --output-format csv -- python3 bench.py --config c4 --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02x/bench.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r02x/bench_s1 -o run --output-format csv -- python3 bench.py --config c4 --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --seed 1 > gpurun_out/r02x/bench_s1.log 2>&1 || exit $?
