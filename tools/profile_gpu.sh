#!/bin/bash
# Profile one bench.py config on the GPU box (run from the repo root through
# gpurun).  Three separate rocprofv3 runs, as MI355X_MICROARCH.md's rocprofv3
# section prescribes: a kernel trace with --stats, then one PMC pass per TCC
# counter (FETCH_SIZE and WRITE_SIZE do not fit in one pass), then one SQ +
# GRBM pass for the issue mix (VALU busy, wave wait share).  Outputs land
# in gpurun_out/prof/<tag>/<config>/; tools/traffic.py condenses them into
# profiles/<tag>/<config>/ and profiles/traffic.json.
# The trace pass runs the bench command exactly as given (the driver's is
# `bench.py --gpus 1 --steps 20 --warmup 5`), so the line it prints and the
# trace's kernel average come from one process; a plain bench line runs
# before and after the passes on the same lease, and the box is recorded.
#   usage: tools/profile_gpu.sh <tag> <config> [bench.py args...]
set -euo pipefail
TAG=${1:-r02}
CFG=${2:-c3}
shift 2 || true
ARGS=${*:-"--gpus 1 --steps 20 --warmup 5"}
R=$(pwd)
OUT=$R/gpurun_out/prof/$TAG/$CFG
mkdir -p "$OUT"
bash "$R/tools/boxinfo.sh" > "$OUT/box.txt" 2>&1 || true
timeout -k 10 300 python3 "$R/bench.py" --config "$CFG" $ARGS > "$OUT/bench_before.json" 2> "$OUT/bench_before.err"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 "$R/bench.py" --config "$CFG" $ARGS > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
  -- python3 "$R/bench.py" --config "$CFG" $ARGS --no-cpu-baseline > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run \
  -- python3 "$R/bench.py" --config "$CFG" $ARGS --no-cpu-baseline > "$OUT/write.log" 2>&1
# issue mix: a failed pass (e.g. a counter this ROCm does not list) only
# drops the issue block from the summary
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_INSTS_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq" -o run \
  -- python3 "$R/bench.py" --config "$CFG" $ARGS --no-cpu-baseline > "$OUT/sq.log" 2>&1 || echo "SQ pass failed (rc=$?)"
cd "$R"
timeout -k 10 300 python3 "$R/bench.py" --config "$CFG" $ARGS --no-cpu-baseline > "$OUT/bench_after.json" \
  2> "$OUT/bench_after.err"
python3 tools/traffic.py "$OUT" --config "$CFG" $ARGS
