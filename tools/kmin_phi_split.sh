#!/bin/bash
# Round 4's k_min<0> defect: which of the SLP IR's five <2 x i32> phis carry
# it?  Variants of the committed IR with chosen phis split into i32 pairs
# (tools/kmin_phi_split.py), compiled by llc -O3 into code objects that
# build/w3phi/w3_module_check runs on the GPU (call r05zk).  Investigation tool.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
B=/opt/rocm/llvm/bin
T="-mtriple=amdgcn-amd-amdhsa -mcpu=gfx950"
S="$R/profiles/r04/codegen/kmin_slp.ll"
O="$R/build/w3phi/phisplit"
mkdir -p "$O"
PHIS="810 811 812 813 850"
gen() {  # name phis...
  local n=$1; shift
  python3 "$R/tools/kmin_phi_split.py" "$S" "$O/$n.ll" "$@"
  $B/opt -passes=verify "$O/$n.ll" -S -o /dev/null
  $B/llc $T -O3 -filetype=obj "$O/$n.ll" -o "$O/$n.o"
  $B/ld.lld -shared "$O/$n.o" -o "$O/kmin_phi_$n.co"
  $B/llc $T -O3 "$O/$n.ll" -o "$O/$n.s"
  rm -f "$O/$n.o"
}
gen none
gen all $PHIS
for p in $PHIS; do
  gen only$p $p
  gen allbut$p $(for q in $PHIS; do [ $q = $p ] || echo $q; done)
done
ls "$O"/*.co
