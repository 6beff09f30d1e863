# Round 5: coup_step_many's rules-trajectory form (k_trajectory_sorted<1024,
# true> per chunk of steps + k_obs_sweep_rows<512, 2> per step) -- its
# equality tests and the c3 headline check against the oracle; a
# same-process A/B against the serial split step and chunk lengths; the
# driver's bench line; smoke(); the tensor-like vs index-bit store ceilings.
set -u
D=gpurun_out/r05d
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_step_many.py \
  tests/test_gpu_headline.py::test_c3_headline_kernel_full_batch_slices_match_oracle > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
timeout -k 10 300 python -u tools/pipe_ab.py > $D/pipe_ab.jsonl 2> $D/pipe_ab.err || { tail -20 $D/pipe_ab.err; exit 1; }
cat $D/pipe_ab.jsonl
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_c3.json 2> $D/bench_c3.err || { tail -20 $D/bench_c3.err; exit 1; }
cat $D/bench_c3.json
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python -u tools/sweep_ab.py > $D/sweep_ab.jsonl 2> $D/sweep_ab.err || { tail -20 $D/sweep_ab.err; exit 1; }
cat $D/sweep_ab.jsonl
