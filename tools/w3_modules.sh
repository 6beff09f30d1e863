#!/bin/bash
# Code objects of the reproducer's k_min<0> (tools/slot_inline_repro.hip) for
# tools/w3_module_check.hip: the device IR of the
# reproducer as hipcc -O3 leaves it, with the SLP vectorizer (as the product
# built before round 3) and without it (as it builds now); k_min<0> kept
# alone (internalize + globaldce: no change to its body); then llc at
# -O0..-O3 for each, and the SLP IR once more after opt's scalarizer (vector
# operations split back into scalar ones, a semantics-preserving IR rewrite)
# at -O3.  Also the host checker.  Outputs under build/w3/ (git-ignored; the
# .co files travel to the GPU box with the snapshot).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
B=/opt/rocm/llvm/bin
O="$R/build/w3"
K=_Z5k_minILi0EEvN4coup8SlotArgsE
mkdir -p "$O"
for v in slp noslp; do
  F=""
  [ "$v" = noslp ] && F="-fno-slp-vectorize"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DCOUP_RULES_V1 $F -I "$R/include" \
    -I "$R/open_spiel_coup_amd/csrc" --cuda-device-only -emit-llvm -S "$R/tools/slot_inline_repro.hip" \
    -o "$O/repro_$v.ll" 2>/dev/null
  $B/opt -passes='internalize,globaldce' -internalize-public-api-list=$K "$O/repro_$v.ll" -S -o "$O/kmin_$v.ll"
done
$B/opt -passes='scalarizer<load-store>' "$O/kmin_slp.ll" -S -o "$O/kmin_slpscal.ll"
for v in slp noslp slpscal; do
  for o in 0 1 2 3; do
    [ "$v" = slpscal ] && [ "$o" != 3 ] && continue
    $B/llc -O$o -mtriple=amdgcn-amd-amdhsa -mcpu=gfx950 -filetype=obj "$O/kmin_$v.ll" -o "$O/kmin_${v}_O$o.o"
    $B/ld.lld -shared "$O/kmin_${v}_O$o.o" -o "$O/kmin_${v}_O$o.co"
    $B/llc -O$o -mtriple=amdgcn-amd-amdhsa -mcpu=gfx950 "$O/kmin_$v.ll" -o "$O/kmin_${v}_O$o.s"
  done
done
# the SLP IR once more through GlobalISel instead of SelectionDAG
for v in slp noslp; do
  $B/llc -O3 -global-isel -mtriple=amdgcn-amd-amdhsa -mcpu=gfx950 -filetype=obj "$O/kmin_$v.ll" -o "$O/kmin_${v}_O3gisel.o"
  $B/ld.lld -shared "$O/kmin_${v}_O3gisel.o" -o "$O/kmin_${v}_O3gisel.co"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -std=c++17 -I "$R/include" \
  -I "$R/open_spiel_coup_amd/csrc" -I "$R/tools" "$R/tools/w3_module_check.hip" \
  "$R/open_spiel_coup_amd/csrc/coup_nplayer.hip" -o "$O/w3_module_check"
rm -f "$O"/repro_*.ll "$O"/*.o
