#!/bin/bash
# Profile the benchmark's step kernel on the GPU box (run from the repo root
# through gpurun).  Three separate rocprofv3 runs, as MI355X_MICROARCH.md's
# rocprofv3 section prescribes: a kernel trace with --stats, then one PMC pass
# per TCC counter group (FETCH_SIZE and WRITE_SIZE do not fit in one pass).
# Outputs land in gpurun_out/prof/<tag>/; tools/traffic.py condenses them.
#   usage: tools/profile_gpu.sh <tag> [bench.py args...]
set -euo pipefail
TAG=${1:-r01}
shift || true
ARGS=${*:-"--steps 20 --warmup 3"}
R=$(pwd)
OUT=$R/gpurun_out/prof/$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 "$R/bench.py" $ARGS --no-cpu-baseline > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
  -- python3 "$R/bench.py" $ARGS --no-cpu-baseline > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run \
  -- python3 "$R/bench.py" $ARGS --no-cpu-baseline > "$OUT/write.log" 2>&1
cd "$R"
python3 tools/traffic.py "$OUT" $ARGS
