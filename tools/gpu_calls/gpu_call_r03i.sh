# Round 3 measurement set on one box: box identity; the driver's default c3
# line (store ceiling in the same process); the store-order probe (chunk
# orders vs an unconstrained sweep); the c4 line (per-launch kernel times),
# c4t, c2; a c3 line again; the c4 profile with the exact bench command.
set -u
D=gpurun_out/r03i
mkdir -p $D
bash tools/boxinfo.sh > $D/box.txt 2>&1 || true
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_c3.json 2> $D/bench_c3.err || { tail -5 $D/bench_c3.err; exit 1; }
cut -c1-300 $D/bench_c3.json
timeout -k 10 200 ./build/store_probe > $D/store_probe.jsonl 2> $D/store_probe.err || { tail -5 $D/store_probe.err; exit 1; }
tail -4 $D/store_probe.jsonl
for c in c4 c4t c2; do
  st=20; [ $c = c4t ] && st=100
  timeout -k 10 300 python -u bench.py --gpus 1 --config $c --steps $st --warmup 5 > $D/bench_$c.json 2> $D/bench_$c.err || { tail -5 $D/bench_$c.err; exit 1; }
  cut -c1-200 $D/bench_$c.json
done
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $D/bench_c3_again.json 2> $D/bench_c3b.err || { tail -5 $D/bench_c3b.err; exit 1; }
cut -c1-200 $D/bench_c3_again.json
timeout -k 10 900 bash tools/profile_gpu.sh r03 c4 --gpus 1 --steps 20 --warmup 5 > $D/prof_c4.log 2>&1 || { tail -20 $D/prof_c4.log; exit 1; }
grep -E "kernel_ms|rocprof_minus|timed_kernel" $D/prof_c4.log | head
