# Round 5: after the gate moved ahead of the graph replay -- the dist tests
# (deterministic games with --gate-steps 0), then the c2 / c4 / c3 profiles
# (each with its before / after lines).
set -u
D=gpurun_out/r05s
mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_dist.py > $D/pytest_dist.log 2>&1 || { tail -40 $D/pytest_dist.log; exit 1; }
tail -2 $D/pytest_dist.log
for c in c2 c4 c3; do
  timeout -k 10 900 bash tools/profile_gpu.sh r05 $c > gpurun_out/profile_r05_$c.log 2>&1 || { tail -30 gpurun_out/profile_r05_$c.log; exit 1; }
  python3 -c "
import json
for w in ('before','after'):
    d=[json.loads(l) for l in open('gpurun_out/prof/r05/$c/bench_'+w+'.json') if l.startswith('{')][-1]
    print('$c', w, d['value'], d['roofline']['kernel_ms'], d['config']['gate_steps'])"
done
