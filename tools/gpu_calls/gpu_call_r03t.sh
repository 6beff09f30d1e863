# Round 3: the tree built without the SLP vectorizer -- whole GPU suite,
# smoke(), then the measurement set on one box: box identity, the driver's
# default c3 line (store ceiling in the same process), c4 / c4t / c2 lines,
# and the c3 profile with the bench command.
set -u
D=gpurun_out/r03t
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
bash tools/boxinfo.sh > $D/box.txt 2>&1 || true
timeout -k 10 300 python -u bench.py > $D/bench_c3.json 2> $D/bench_c3.err || { tail -5 $D/bench_c3.err; exit 1; }
cut -c1-250 $D/bench_c3.json
for c in c4 c4t c2; do
  st=20; [ $c = c4t ] && st=100
  timeout -k 10 300 python -u bench.py --gpus 1 --config $c --steps $st --warmup 5 --no-cpu-baseline > $D/bench_$c.json 2> $D/bench_$c.err || { tail -5 $D/bench_$c.err; exit 1; }
  cut -c1-200 $D/bench_$c.json
done
timeout -k 10 900 bash tools/profile_gpu.sh r03 c3 --gpus 1 --steps 20 --warmup 5 > $D/prof_c3.log 2>&1 || { tail -20 $D/prof_c3.log; exit 1; }
grep -E "kernel_ms|rocprof_minus|timed_kernel" $D/prof_c3.log | head
