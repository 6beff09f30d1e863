# Round 4, twenty-first call: the split InformationStateTensor step
# (COUP_INFO_SPLIT 1-5: the history-keeping rules step, then k_info_sweep in
# address order) -- equality tests against the fused writer, then the c3i
# A/B at 2^18 lanes.
set -u
D=gpurun_out/r04u
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_gpu_obs_split.py -x -q -k info --timeout 400 --timeout-method thread > $D/pytest_info_split.log 2>&1 || { tail -60 $D/pytest_info_split.log; exit 1; }
tail -2 $D/pytest_info_split.log
timeout -k 10 300 python -u tools/ab_step.py --batch 262144 --obs 0 --info 1 --rounds 7 COUP_INFO_SPLIT=0 COUP_INFO_SPLIT=1 COUP_INFO_SPLIT=2 COUP_INFO_SPLIT=3 COUP_INFO_SPLIT=4 COUP_INFO_SPLIT=5 > $D/ab_c3i_split.jsonl 2> $D/ab_c3i_split.err || { tail -5 $D/ab_c3i_split.err; exit 1; }
cut -c1-100 $D/ab_c3i_split.jsonl
