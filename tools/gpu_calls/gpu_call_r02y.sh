# c4: local-reset variant (parity + A/B), c4 bench eager default.
set -u
mkdir -p gpurun_out/r02y
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nplayer.py > gpurun_out/r02y/nplayer.log 2>&1 || { tail -20 gpurun_out/r02y/nplayer.log; exit 1; }
tail -1 gpurun_out/r02y/nplayer.log
timeout -k 10 300 python -u tools/ab_step.py --players 6 --obs 0 --rounds 9 COUP_NP_LOCAL_RESET=0 COUP_NP_LOCAL_RESET=1 COUP_NP_LOCAL_RESET=1,COUP_NP_SORT_THREADS=1024 > gpurun_out/r02y/ab_local_reset.log 2>&1 || { tail gpurun_out/r02y/ab_local_reset.log; exit 1; }
grep variant gpurun_out/r02y/ab_local_reset.log
timeout -k 10 200 python -u bench.py --config c4 --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02y/bench_c4.json 2> gpurun_out/r02y/bench_c4.err || exit $?
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['roofline']['kernel_ms'], d['config']['hip_graph'])" gpurun_out/r02y/bench_c4.json
