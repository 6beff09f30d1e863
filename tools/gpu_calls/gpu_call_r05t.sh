# Round 5: c2 / c4 time coup_step_many eagerly (one trajectory launch behind a
# gate; no graph), c3 through its graph with a 1.5x gate: the dist tests, then
# the three profiles again.
set -u
D=gpurun_out/r05t
mkdir -p $D
true
true
for c in c2 c4 c3; do
  timeout -k 10 900 bash tools/profile_gpu.sh r05 $c > gpurun_out/profile_r05_$c.log 2>&1 || { tail -30 gpurun_out/profile_r05_$c.log; exit 1; }
  python3 -c "
import json
for w in ('before','after'):
    d=[json.loads(l) for l in open('gpurun_out/prof/r05/$c/bench_'+w+'.json') if l.startswith('{')][-1]
    print('$c', w, d['value'], d['roofline']['kernel_ms'], d['config']['gate_steps'], d['config']['hip_graph'])"
done
