# Round 5: the store sweep beside a writer-like sweep (load -> LDS -> barrier -> stores, no decode)
# Sweep shapes with a dependent integer chain of 8 / 24 / 64 ops ahead of each
# store (measurement build), beside the plain sweeps, on both tensor buffers.
set -u
D=gpurun_out/r05ze
mkdir -p $D
COUP_LIB_PATH=build/variants/libcoup_mi355x.so timeout -k 10 600 python -u tools/sweep_ab.py > $D/sweep_ab.jsonl 2> $D/sweep_ab.err || { tail -20 $D/sweep_ab.err; exit 1; }
python3 -c "
import json
for l in open('$D/sweep_ab.jsonl'):
    d=json.loads(l); print(d['buffer'], d['threads'], d['passes'], 'res' if d['resident'] else '', d['data'], d['pace_ops'], 'WL' if d.get('writerlike') else '', d['median_us'], d['tb_per_s'])"
