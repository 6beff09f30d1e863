# Round 6: the c3 profile of the final tree (balanced 10-step rules chunks):
# tools/profile_gpu.sh (the driver's command traced, FETCH / WRITE / SQ passes
# in runs of their own), smoke(), and the driver's default line.
set -u
. tools/gpu_calls/attempt.sh r06za
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 500 bash tools/profile_gpu.sh r06 c3 > $D/profile_c3.log 2>&1 || { tail -30 $D/profile_c3.log; exit 1; }
tail -2 $D/profile_c3.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_default.json 2> $D/bench_default.err || { tail -20 $D/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_default.json')); r=d['roofline']; print('c3', d['value'], r['frac'], r['kernel_ms'], r['kernel'] == r['kernel_launched'])"
