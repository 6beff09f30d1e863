# Round 5, first call: the pipelined split observation step (coup_step_many,
# k_step_obs_pipe) -- its equality tests and the c3 headline check against the
# oracle; the section-12 codegen checks (the uint2-prefix reproducer, k_min<0>
# with single <2 x i32> phis split); a same-process A/B of the step forms in
# the driver's form; the driver's bench line; smoke(); the c3 profile.
set -u
D=gpurun_out/r05a
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py \
  tests/test_gpu_headline.py::test_c3_headline_kernel_full_batch_slices_match_oracle \
  tests/test_gpu_codegen_hazard.py > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
timeout -k 10 120 build/info_prefix_repro 100000 > $D/info_prefix_repro.jsonl 2>&1 || { cat $D/info_prefix_repro.jsonl; exit 1; }
cat $D/info_prefix_repro.jsonl
timeout -k 10 300 build/w3phi/w3_module_check 20000 $(ls build/w3phi/*.co) > $D/w3_phi_variants.json 2>&1 || { tail -5 $D/w3_phi_variants.json; exit 1; }
python3 -c "
import json; d=json.load(open('$D/w3_phi_variants.json'))
for k,v in d['modules'].items(): print(k, v['mismatch'], v['by_word'])"
timeout -k 10 300 python -u tools/pipe_ab.py > $D/pipe_ab.jsonl 2> $D/pipe_ab.err || { tail -20 $D/pipe_ab.err; exit 1; }
cat $D/pipe_ab.jsonl
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_c3.json 2> $D/bench_c3.err || { tail -20 $D/bench_c3.err; exit 1; }
cat $D/bench_c3.json
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 900 bash tools/profile_gpu.sh r05 c3 > $D/profile.log 2>&1 || { tail -30 $D/profile.log; exit 1; }
tail -5 $D/profile.log
