# Round 4, twentieth call: the split observation step as the default from
# 2^20 lanes (k_step_sorted<true, 512> + k_obs_sweep_rows<512, 2>) -- the
# whole GPU suite, smoke(), the driver's default bench line, the c3 profile
# (trace + PMC passes), and the fused/split A/B at 2^19 lanes.
set -u
D=gpurun_out/r04t
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
cut -c1-300 $D/bench.json
bash tools/profile_gpu.sh r04 c3 > $D/profile_c3.log 2>&1 || { tail -30 $D/profile_c3.log; exit 1; }
tail -5 $D/profile_c3.log
timeout -k 10 150 python -u tools/ab_step.py --batch 524288 --obs 1 --rounds 7 COUP_OBS_SPLIT=0 COUP_OBS_SPLIT=11 > $D/ab_2e19_split.jsonl 2> $D/ab_2e19_split.err || { tail -5 $D/ab_2e19_split.err; exit 1; }
cut -c1-100 $D/ab_2e19_split.jsonl
