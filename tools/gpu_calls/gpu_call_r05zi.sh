#!/bin/bash
# Round 5: where the 2-player rules trajectory's cycles go at 2^20 lanes
# (bare form, c2 at c3's batch): SQ counter passes, each in a run of its own.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zi
mkdir -p $O
B="python3 -u bench.py --config c2 --batch 1048576 --steps 20 --warmup 5 --settle 8 --power-warm-ms 0 --no-cpu-baseline"
timeout -k 10 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $O/p1 -o run -- $B > $O/p1.json 2> $O/p1.err &&
timeout -k 10 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --output-format csv -d $O/p2 -o run -- $B > $O/p2.json 2> $O/p2.err &&
ls -R $O | head -20
