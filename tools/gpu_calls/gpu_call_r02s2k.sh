# Round 2, session 2: 2-player coup_step_trajectory with ObservationTensor write-out -- parity, then c3 and c3t lines.
set -u
D=gpurun_out/r02s2k
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_trajectory.py -x -v --timeout 150 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
for a in "c3 20" "c3t 20" "c3t 100" "c3 100"; do
  set -- $a
  timeout -k 10 300 python -u bench.py --config $1 --steps $2 --warmup 5 --no-cpu-baseline > $D/bench_$1_$2.json 2> $D/bench_$1_$2.err || { tail $D/bench_$1_$2.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$D/bench_$1_$2.json')); r=d['roofline']; print('$1 K=$2', '%.3e' % d['value'], round(r['kernel_ms']*1e3/ (d['config']['fused_steps_per_launch']), 2), 'us/step frac', round(r['frac'],3), 'ceiling', r['store_ceiling_ms'], r['kernel'])"
done
