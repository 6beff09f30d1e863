#!/bin/bash
# Round 5: the 2-player rules trajectory at c3's 2^20 lanes without records or
# per-step outputs (c2's bare form at c3's batch) beside c3 itself: how much of
# c3's 19.6 us of rules per step is rules compute?
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zh
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2big -o run -- python3 -u bench.py --config c2 --batch 1048576 --steps 20 --warmup 5 --no-cpu-baseline > $O/c2big.json 2> $O/c2big.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o run -- python3 -u bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline > $O/c3.json 2> $O/c3.err &&
tail -1 $O/c2big.json | cut -c1-300 && tail -1 $O/c3.json | cut -c1-300 &&
for d in c2big c3; do echo "== $d"; find $O/$d -name '*kernel_stats.csv' -exec cut -d, -f1-8 {} \; | head -8; done
