# Round 4, fourth call: the whole GPU suite and smoke() with k_step_group<1>
# as the default rules-bound step; the llc opt-bisect of the word-3 defect
# (69 code objects of k_min<0> from the SLP IR, 4000 cases each); the c2
# step's per-wave timeline (trace build, k_step).
set -u
D=gpurun_out/r04d
mkdir -p $D
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
MODS=""; for n in $(seq 0 68); do MODS="$MODS build/w3/bisect/b$n.co"; done
timeout -k 10 240 build/w3/w3_module_check 4000 $MODS > $D/w3_bisect.json 2> $D/w3_bisect.err || { tail -5 $D/w3_bisect.err; exit 1; }
python -c "import json;d=json.load(open('$D/w3_bisect.json'));print([(k.split('/')[-1][:-3],v['mismatch']) for k,v in d['modules'].items()])"
COUP_LIB_PATH=build/trace/libcoup_trace.so COUP_STEP_TPL=0 timeout -k 10 120 python -u tools/wave_trace.py --obs 0 --batch 65536 --bin-us 0.5 > $D/wave_trace_c2.txt 2>&1 || { tail -5 $D/wave_trace_c2.txt; exit 1; }
head -1 $D/wave_trace_c2.txt | cut -c1-1500
