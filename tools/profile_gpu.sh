#!/bin/bash
# Profile one bench.py config on the GPU box (run from the repo root through
# gpurun).  Three separate rocprofv3 runs, as MI355X_MICROARCH.md's rocprofv3
# section prescribes: a kernel trace with --stats, then one PMC pass per TCC
# counter (FETCH_SIZE and WRITE_SIZE do not fit in one pass).  Outputs land
# in gpurun_out/prof/<tag>/<config>/; tools/traffic.py condenses them into
# profiles/<tag>/<config>/ and profiles/traffic.json.
#   usage: tools/profile_gpu.sh <tag> <config> [bench.py args...]
set -euo pipefail
TAG=${1:-r01}
CFG=${2:-c3}
shift 2 || true
ARGS=${*:-"--steps 20 --warmup 3"}
R=$(pwd)
OUT=$R/gpurun_out/prof/$TAG/$CFG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 "$R/bench.py" --config "$CFG" $ARGS --no-cpu-baseline > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
  -- python3 "$R/bench.py" --config "$CFG" $ARGS --no-cpu-baseline > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run \
  -- python3 "$R/bench.py" --config "$CFG" $ARGS --no-cpu-baseline > "$OUT/write.log" 2>&1
cd "$R"
python3 tools/traffic.py "$OUT" --config "$CFG" $ARGS
