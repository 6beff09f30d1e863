# Round 5: the final bench form (graph replays of coup_step_many for c2 / c3 /
# c4, no gate before a replay, power warm-up): the dist tests, the three
# profiles (each with before / after lines), c3i's line.
set -u
D=gpurun_out/r05u
mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_dist.py > $D/pytest_dist.log 2>&1 || { tail -40 $D/pytest_dist.log; exit 1; }
tail -2 $D/pytest_dist.log
for c in c3 c2 c4; do
  timeout -k 10 900 bash tools/profile_gpu.sh r05 $c > gpurun_out/profile_r05_$c.log 2>&1 || { tail -30 gpurun_out/profile_r05_$c.log; exit 1; }
  python3 -c "
import json
for w in ('before','after'):
    d=[json.loads(l) for l in open('gpurun_out/prof/r05/$c/bench_'+w+'.json') if l.startswith('{')][-1]
    print('$c', w, d['value'], d['roofline']['kernel_ms'], d['config']['gate_steps'], d['config']['hip_graph'])"
done
timeout -k 10 300 python -u bench.py --config c3i --no-cpu-baseline > $D/bench_c3i.json 2> $D/bench_c3i.err || { tail -20 $D/bench_c3i.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_c3i.json')); r=d['roofline']; print('c3i', d['value'], r['frac'], r['kernel_ms'], r.get('store_ceiling_ms'))"
