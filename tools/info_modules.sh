#!/bin/bash
# Code objects of tools/info_prefix_repro.hip's k_sweep_uint2<512, 2> (round
# 4's first k_info_sweep: the prefix words stored as uint2) and, as the
# control, k_sweep_rows<512, 2>, for `build/info_prefix_repro N *.co`
# (VERDICT r4 item 1): the device IR as hipcc -O3
# -fno-slp-vectorize leaves it, the two kernels kept alone (internalize +
# globaldce), then llc at -O0 and -O3, -O3 through GlobalISel, and -O3 with
# -opt-bisect-limit at every limit over llc's optional passes (the machine
# passes an opt-bisect may skip) -- which names the pass if one of them
# brings the defect -- and -O3 / -O0 with an s_nop before every instruction
# or every s_waitcnt forced to zero.  Outputs under build/infomod/ (the .co files travel).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
B=/opt/rocm/llvm/bin
O="$R/build/infomod"
K1=_Z13k_sweep_uint2ILi512ELi2EEvPK15HIP_vector_typeIjLj4EEPKhPfl
K2=_Z12k_sweep_rowsILi512ELi2EEvPK15HIP_vector_typeIjLj4EEPKhPfl
T="-mtriple=amdgcn-amd-amdhsa -mcpu=gfx950"
rm -rf "$O"
mkdir -p "$O"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -std=c++17 -I "$R/include" \
  -I "$R/open_spiel_coup_amd/csrc" --cuda-device-only -emit-llvm -S "$R/tools/info_prefix_repro.hip" \
  -o "$O/repro.ll" 2>/dev/null
$B/opt -passes='internalize,globaldce' -internalize-public-api-list=$K1,$K2 "$O/repro.ll" -S -o "$O/sweep.ll"
co() {  # co <name> <llc flags...>
  local name=$1
  shift
  $B/llc $T "$@" -filetype=obj "$O/sweep.ll" -o "$O/$name.o" 2>/dev/null
  $B/ld.lld -shared "$O/$name.o" -o "$O/$name.co"
  rm -f "$O/$name.o"
}
co O0 -O0
co O3 -O3
co O3gisel -O3 -global-isel
# the hazard / wait hypotheses: an s_nop before every instruction (covers any
# missing wait states of the hazard recognizer), and every s_waitcnt forced
# to zero (covers a missing memory-counter wait)
co O3snop4 -O3 -amdgpu-snop-padding=4
co O3waitzero -O3 -amdgpu-waitcnt-forcezero
co O0snop4 -O0 -amdgpu-snop-padding=4
co O3snop15 -O3 -amdgpu-snop-padding=15
co O3snop15waitzero -O3 -amdgpu-snop-padding=15 -amdgpu-waitcnt-forcezero
# the optional passes of an -O3 llc run, in order (opt-bisect's numbering)
$B/llc $T -O3 -opt-bisect-limit=-1 -filetype=null "$O/sweep.ll" 2> "$O/passes.txt" || true
N=$(grep -c "BISECT: running pass" "$O/passes.txt" || true)
for ((l = 0; l <= N; l++)); do
  co "bisect_$(printf %03d $l)" -O3 -opt-bisect-limit=$l
done
$B/llc $T -O3 "$O/sweep.ll" -o "$O/O3.s"
echo "$N optional passes; $(ls "$O"/*.co | wc -l) code objects in $O"
