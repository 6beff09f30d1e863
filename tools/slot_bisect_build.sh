#!/bin/bash
# Build the k_slot reproducer (tools/slot_inline_repro.hip) WITH the SLP
# vectorizer (the product builds without it: the defect's trigger) and LLVM's
# -opt-bisect-limit=N for each N given: passes past N are skipped (in the
# device and the host compilations alike; the host code only gets slower).
# Running the binaries on a GPU finds the first device pass after which
# the inline k_slot miscompiles.
#   tools/slot_bisect_build.sh N1 N2 ...   -> build/bisect/repro_N
# The pass numbers of the k_min<0> kernel come from a device-only compile
# with -mllvm -opt-bisect-limit=-1 (profiles/r03/codegen/k_min0_passes.txt).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/build/bisect"
for n in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DCOUP_RULES_V1 -I "$R/include" -I "$R/open_spiel_coup_amd/csrc" \
    -mllvm -opt-bisect-limit="$n" "$R/tools/slot_inline_repro.hip" "$R/open_spiel_coup_amd/csrc/coup_nplayer.hip" \
    -o "$R/build/bisect/repro_$n" 2>/dev/null &
done
wait
