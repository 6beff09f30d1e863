# Round 5: coup_step_many's tensor-free form (ONE trajectory launch for the K
# steps, outputs over the [B] buffers) -- its equality tests, then c2 / c4
# lines with it (the graph path) and without it (COUP_PIPE=0: one coup_step
# per step), alternating, and the c4t line.
set -u
D=gpurun_out/r05q
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_step_many.py > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
for i in 1 2; do
  for c in c2 c4; do
    for p in 1 0; do
      COUP_PIPE=$p timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $D/bench_${c}_pipe${p}_$i.json 2> $D/bench_${c}_pipe${p}_$i.err || { tail -20 $D/bench_${c}_pipe${p}_$i.err; exit 1; }
      python3 -c "import json; d=json.load(open('$D/bench_${c}_pipe${p}_$i.json')); r=d['roofline']; print('$c pipe=$p', d['value'], round(r['kernel_ms']*1e3/d['config']['fused_steps_per_launch'],2), 'us/step', r['kernel'], r['step_form'])"
    done
  done
done
timeout -k 10 300 python -u bench.py --config c4t --no-cpu-baseline > $D/bench_c4t.json 2> $D/bench_c4t.err || { tail -20 $D/bench_c4t.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_c4t.json')); r=d['roofline']; print('c4t', d['value'], r['kernel_ms'], r['kernel'])"
