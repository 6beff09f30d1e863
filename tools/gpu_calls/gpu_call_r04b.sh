# Round 4, second call: r04a stopped at a too-strict launch-count assertion
# (the destroy-stops-the-wave test); the server tests again, the c2 group-step
# A/B, the c3 / c2 lines, the rest of the GPU suite, the facade latencies, and
# the word-3 code-object check (tools/w3_module_check.hip).
set -u
D=gpurun_out/r04b
mkdir -p $D
timeout -k 10 240 python -u -m pytest tests/test_gpu_server.py tests/test_gpu_unchecked.py -x -v --timeout 150 --timeout-method thread > $D/pytest_server.log 2>&1 || { tail -60 $D/pytest_server.log; exit 1; }
tail -2 $D/pytest_server.log
timeout -k 10 120 build/w3/w3_module_check 20000 build/w3/kmin_noslp_O0.co build/w3/kmin_noslp_O1.co build/w3/kmin_noslp_O2.co build/w3/kmin_noslp_O3.co build/w3/kmin_slp_O0.co build/w3/kmin_slp_O1.co build/w3/kmin_slp_O2.co build/w3/kmin_slp_O3.co build/w3/kmin_slpscal_O3.co > $D/w3_modules.json 2> $D/w3_modules.err || { tail -5 $D/w3_modules.err; exit 1; }
python -c "import json;d=json.load(open('$D/w3_modules.json'));print({k.split('/')[-1]:(v['mismatch'],v['by_word']) for k,v in d['modules'].items()})"
timeout -k 10 90 python -u tools/ab_step.py --batch 65536 --obs 0 --rounds 9 "" COUP_STEP_TPL=1 COUP_STEP_TPL=2 COUP_STEP_TPL=4 > $D/ab_c2_tpl.jsonl 2> $D/ab_c2_tpl.err || { tail -5 $D/ab_c2_tpl.err; exit 1; }
cut -c1-100 $D/ab_c2_tpl.jsonl
timeout -k 10 100 python -u bench.py > $D/bench_c3.json 2> $D/bench_c3.err || { tail -5 $D/bench_c3.err; exit 1; }
cut -c1-300 $D/bench_c3.json
timeout -k 10 100 python -u bench.py --config c2 --steps 20 --warmup 5 > $D/bench_c2.json 2> $D/bench_c2.err || { tail -5 $D/bench_c2.err; exit 1; }
cut -c1-300 $D/bench_c2.json
NEW="tests/test_gpu_step_group.py tests/test_gpu_episode_word.py tests/test_gpu_headline.py tests/test_gpu_dist.py tests/test_gpu_server.py tests/test_gpu_unchecked.py"
IGN=""; for f in $NEW; do IGN="$IGN --ignore=$f"; done
timeout -k 10 300 python -u -m pytest tests -m gpu $IGN -x -q --timeout 200 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 130 python -u tools/facade_latency.py --rounds 2 --ops 500 > $D/facade_latency.json 2> $D/facade_latency.err || { tail -5 $D/facade_latency.err; exit 1; }
cut -c1-300 $D/facade_latency.json
COUP_LIB_PATH=build/trace/libcoup_trace.so timeout -k 10 120 python -u tools/np_wave_trace.py --out $D/np_wave_trace.json > $D/np_wave_trace.txt 2>&1 || { tail -5 $D/np_wave_trace.txt; exit 1; }
tail -15 $D/np_wave_trace.txt
