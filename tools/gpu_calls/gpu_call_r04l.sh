# Round 4, twelfth call: k_step_group<1> with the next episode's deal
# computed up front (COUP_RESET_AHEAD): its tests, then the c2 A/B at 65,536
# lanes and at 2^20 lanes (a config-5 rank's shard).
set -u
D=gpurun_out/r04l
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_step_group.py -x -v --timeout 150 --timeout-method thread > $D/pytest_group.log 2>&1 || { tail -60 $D/pytest_group.log; exit 1; }
tail -2 $D/pytest_group.log
timeout -k 10 120 python -u tools/ab_step.py --batch 65536 --obs 0 --rounds 11 COUP_STEP_TPL=0 "" COUP_RESET_AHEAD=1 > $D/ab_c2_ra.jsonl 2> $D/ab_c2_ra.err || { tail -5 $D/ab_c2_ra.err; exit 1; }
cut -c1-110 $D/ab_c2_ra.jsonl
timeout -k 10 120 python -u tools/ab_step.py --batch 1048576 --obs 0 --rounds 7 COUP_STEP_TPL=0 "" COUP_RESET_AHEAD=1 > $D/ab_c5_ra.jsonl 2> $D/ab_c5_ra.err || { tail -5 $D/ab_c5_ra.err; exit 1; }
cut -c1-110 $D/ab_c5_ra.jsonl
# then the facade rows after the host-side list / tensor speed-ups
timeout -k 10 400 python -u tools/facade_latency.py > $D/facade.json 2> $D/facade.err || { tail -20 $D/facade.err; exit 1; }
python -c "
import json; d=json.load(open('$D/facade.json'))['rows_us']
for k,v in d.items():
    if k.startswith(('vector','rl_env','host_')): print(k, v['median'])"
