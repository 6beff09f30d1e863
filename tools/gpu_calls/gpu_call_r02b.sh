set -u
mkdir -p gpurun_out/r02b
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "episode_stats or c2_bench or gpu_dist or traffic_ceiling" > gpurun_out/r02b/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/r02b/pytest_gpu.log
if grep -q "Timeout +++" gpurun_out/r02b/pytest_gpu.log; then exit 3; fi
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/boxinfo.sh > gpurun_out/r02b/box.txt 2>&1
timeout -k 10 300 python -u tools/ab_step.py --rounds 7 --steps 20 STATS=0 STATS=1 STATS=1,COUP_EP_MODE=1 STATS=1,COUP_EP_MODE=2 CEIL=1 > gpurun_out/r02b/ab_epstats.jsonl 2>gpurun_out/r02b/ab.err || exit $?
cat gpurun_out/r02b/ab_epstats.jsonl
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02b/bench_c3.json 2>gpurun_out/r02b/bench.err || exit $?
cut -c1-400 gpurun_out/r02b/bench_c3.json
exit $rc
