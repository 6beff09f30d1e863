#!/bin/bash
# Round 5: does the store sweep's per-kernel duration drop when an idle kernel
# follows each sweep (dirty lines draining after the kernel ends), as the
# observation writer's does when the rules kernel follows it?
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zf
mkdir -p $O
COUP_LIB_PATH=build/variants/libcoup_mi355x.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/back2back -o run -- python3 -u tools/sweep_ab.py --only 0,16 --rounds 5 > $O/back2back.jsonl 2> $O/back2back.err &&
COUP_LIB_PATH=build/variants/libcoup_mi355x.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/gap100k -o run -- python3 -u tools/sweep_ab.py --only 0,16 --rounds 5 --gap-sleep 100000 > $O/gap100k.jsonl 2> $O/gap100k.err &&
COUP_LIB_PATH=build/variants/libcoup_mi355x.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/gap400k -o run -- python3 -u tools/sweep_ab.py --only 0,16 --rounds 5 --gap-sleep 400000 > $O/gap400k.jsonl 2> $O/gap400k.err &&
for d in back2back gap100k gap400k; do echo "== $d"; cat $O/$d.jsonl; find $O/$d -name '*kernel_stats.csv' -exec grep -h -E 'store_sweep|sleep' {} \; ; done
