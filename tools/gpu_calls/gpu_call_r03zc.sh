#!/bin/bash
# Round 3, final tree: run-to-run spread on one box -- c4 (6-player step) and
# c3 (headline) three times each, no CPU baseline.
set -o pipefail
O=gpurun_out/r03zc
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 240 python -u bench.py --config c4 --steps 100 --warmup 10 --no-cpu-baseline \
      > $O/c4_$i.json 2> $O/c4_$i.err || exit $?
  timeout -k 10 240 python -u bench.py --config c3 --steps 100 --warmup 10 --no-cpu-baseline \
      > $O/c3_$i.json 2> $O/c3_$i.err || exit $?
done
echo done
