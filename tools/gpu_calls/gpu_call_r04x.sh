# Round 4, twenty-fourth call: the split c3 step's rules kernel choice at 2^20
# lanes (regrouped in 512-lane blocks by default; in place: k_step_group<1>;
# 256 / 1024-lane blocks), then the default bench line.
set -u
D=gpurun_out/r04x
mkdir -p $D
timeout -k 10 200 python -u tools/ab_step.py --batch 1048576 --obs 1 --rounds 9 "" COUP_REGROUP=0 COUP_SORT_THREADS=256 COUP_SORT_THREADS=1024 > $D/ab_c3_rules.jsonl 2> $D/ab_c3_rules.err || { tail -5 $D/ab_c3_rules.err; exit 1; }
cut -c1-100 $D/ab_c3_rules.jsonl
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$D/bench.json').readline()); print(d['value'], d['roofline'])"
