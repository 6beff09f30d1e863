#!/bin/bash
# Round 5: is the store rate a function of the data's all-zero lines?  The
# share of zero segments in the writers' real tensors, then the density sweep
# shapes beside the plain ones (measurement build).
set -o pipefail
O=gpurun_out/r05zg
mkdir -p $O
timeout -k 10 300 python3 -u tools/obs_zero_lines.py > $O/zero_lines.jsonl 2> $O/zero_lines.err &&
cat $O/zero_lines.jsonl &&
COUP_LIB_PATH=build/variants/libcoup_mi355x.so timeout -k 10 600 python3 -u tools/sweep_ab.py --only 0,1,16,17,18,19,20,21,22,23,24,25,26 > $O/sweep_ab.jsonl 2> $O/sweep_ab.err &&
python3 -c "
import json
for l in open('$O/sweep_ab.jsonl'):
    d = json.loads(l); print(d['buffer'], d['threads'], 'WL' if d['writerlike'] else '', 'dens', d['dens'], d['median_us'], d['tb_per_s'])
"
