# Round 4, first call: the packed episode word (new tests first), the
# bench.py --gpus launcher and the config-5 rehearsal, the c4 bench-path pin,
# the group-Philox step (tests + c2 A/B), the c3 / c2 lines, the rest of the
# GPU suite, and the facade latencies.
set -u
D=gpurun_out/r04a
mkdir -p $D
NEW="tests/test_gpu_step_group.py tests/test_gpu_episode_word.py tests/test_gpu_headline.py tests/test_gpu_dist.py tests/test_gpu_server.py"
timeout -k 10 450 python -u -m pytest $NEW -x -v --timeout 200 --timeout-method thread > $D/pytest_new.log 2>&1 || { tail -60 $D/pytest_new.log; exit 1; }
tail -3 $D/pytest_new.log
timeout -k 10 90 python -u tools/ab_step.py --batch 65536 --obs 0 --rounds 7 "" COUP_STEP_TPL=1 COUP_STEP_TPL=2 COUP_STEP_TPL=4 > $D/ab_c2_tpl.jsonl 2> $D/ab_c2_tpl.err || { tail -5 $D/ab_c2_tpl.err; exit 1; }
cat $D/ab_c2_tpl.jsonl | cut -c1-120
timeout -k 10 100 python -u bench.py > $D/bench_c3.json 2> $D/bench_c3.err || { tail -5 $D/bench_c3.err; exit 1; }
cut -c1-400 $D/bench_c3.json
timeout -k 10 100 python -u bench.py --config c2 --steps 20 --warmup 5 > $D/bench_c2.json 2> $D/bench_c2.err || { tail -5 $D/bench_c2.err; exit 1; }
cut -c1-400 $D/bench_c2.json
IGN=""; for f in $NEW; do IGN="$IGN --ignore=$f"; done
timeout -k 10 300 python -u -m pytest tests -m gpu $IGN -x -q --timeout 200 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 130 python -u tools/facade_latency.py --rounds 2 --ops 500 > $D/facade_latency.json 2> $D/facade_latency.err || { tail -5 $D/facade_latency.err; exit 1; }
cut -c1-300 $D/facade_latency.json
