#!/bin/bash
# Round 4's deterministic k_min<0> defect, stage by
# stage through llc's late IR pipeline: the committed SLP IR
# (profiles/r04/codegen/kmin_slp.ll) is stopped before each late IR pass and
# before instruction selection (-stop-before; the IR taken out of the MIR
# wrapper), scalarized there by opt's scalarizer (a semantics-preserving
# split of every vector operation) or left as it is, and compiled from that
# point on (-start-before).  build/w3phi/w3_module_check runs the code
# objects on the GPU (call r05w).  Investigation tool.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
B=/opt/rocm/llvm/bin
T="-mtriple=amdgcn-amd-amdhsa -mcpu=gfx950"
SRC="$R/profiles/r04/codegen/kmin_slp.ll"
O="$R/build/w3phi/irstage"
mkdir -p "$O"
unwrap() {  # MIR file with an embedded IR module -> plain IR
  python3 - "$1" "$2" <<'PY'
import sys
lines = open(sys.argv[1]).read().split('\n')
if not lines[0].startswith('--- |'):
    open(sys.argv[2], 'w').write('\n'.join(lines))
    sys.exit(0)
out = []
for l in lines[1:]:
    if l.startswith('...') or l.startswith('---'):
        break
    out.append(l[2:] if l.startswith('  ') else l)
open(sys.argv[2], 'w').write('\n'.join(out) + '\n')
PY
}
for P in lowerswitch flattencfg sink amdgpu-late-codegenprepare amdgpu-unify-divergent-exit-nodes fix-irreducible \
         unify-loop-exits structurizecfg amdgpu-annotate-uniform si-annotate-control-flow \
         amdgpu-rewrite-undef-for-phi lcssa amdgpu-isel; do
  $B/llc $T -O3 -stop-before=$P "$SRC" -o "$O/raw_$P.ll"
  unwrap "$O/raw_$P.ll" "$O/ir_$P.ll"
  $B/opt -passes='scalarizer<load-store>' "$O/ir_$P.ll" -S -o "$O/scal_$P.ll"
  for v in ir scal; do
    $B/llc $T -O3 -start-before=$P -filetype=obj "$O/${v}_$P.ll" -o "$O/${v}_$P.o"
    name=$([ $v = ir ] && echo vecbefore || echo scalbefore)
    $B/ld.lld -shared "$O/${v}_$P.o" -o "$R/build/w3phi/kmin_${name}_$P.co"
  done
done
rm -f "$O"/*.o
