# Round 5: the whole GPU suite on the pruned product library (the A/B
# variants' suite runs inside it against build/variants/), then the other
# configs' bench lines and the writers' store ceilings shape by shape.
set -u
D=gpurun_out/r05b
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
for c in c3i c2 c4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $D/bench_$c.json 2> $D/bench_$c.err || { tail -20 $D/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_$c.json')); r=d['roofline']; print('$c', d['value'], r['frac'], r['kernel_ms'], r.get('store_ceiling_ms'), r['kernel'])"
done
COUP_LIB_PATH=build/variants/libcoup_mi355x.so timeout -k 10 300 python -u tools/sweep_ab.py > $D/sweep_ab.jsonl 2> $D/sweep_ab.err || { tail -20 $D/sweep_ab.err; exit 1; }
cat $D/sweep_ab.jsonl
