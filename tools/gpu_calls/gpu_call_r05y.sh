# Round 5: the c3i writer with sc1 nt buffer stores (shipped now) -- the info
# parity tests (split vs fused, the bench path against the oracle), a
# same-process A/B (measurement build: nt / sc1 / the shipped sc1 nt), and
# the driver-form c3i lines.
set -u
D=gpurun_out/r05y
mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_obs_split.py tests/test_gpu_headline.py -k "info" > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
COUP_LIB_PATH=build/variants/libcoup_mi355x.so timeout -k 10 900 python -u tools/ab_step.py --batch 262144 --obs 0 --info 1 --rounds 9 nt:COUP_WRITER_POL=0 sc1:COUP_WRITER_POL=2 sc1nt:COUP_WRITER_POL=-1 > $D/c3i_ab.jsonl 2> $D/c3i_ab.err || { tail -20 $D/c3i_ab.err; exit 1; }
cut -c1-160 $D/c3i_ab.jsonl
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config c3i --no-cpu-baseline > $D/bench_c3i_$i.json 2> $D/bench_c3i_$i.err || { tail -20 $D/bench_c3i_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_c3i_$i.json')); r=d['roofline']; print('c3i', d['value'], r['frac'], r['kernel_ms'], r.get('store_ceiling_ms'))"
done
