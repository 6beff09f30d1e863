#!/bin/bash
# Round 5: the timing-dependent uint2-prefix fault against the structurizer
# finding -- an undefined register read returns whatever an earlier wave left
# in that register, which would vary with co-resident workgroups and timing.
# The reproducer's kernels (build/infomod2, from tools/info_prefix_repro.hip)
# at -O3, with -structurizecfg-skip-uniform-regions, and scalarized before /
# after structurizecfg; twice each.
set -u
D=gpurun_out/r05zp
mkdir -p $D
for i in 1 2; do
  timeout -k 10 300 build/info_prefix_repro 20000 build/infomod2/O3.co build/infomod2/O3skipuniform.co build/infomod2/scal_after_unify-loop-exits.co build/infomod2/scal_after_structurizecfg.co > $D/mods_$i.jsonl 2>&1 || { tail -5 $D/mods_$i.jsonl; exit 1; }
  python3 -c "
import json
for l in open('$D/mods_$i.jsonl'):
    if l.startswith('{'):
        d = json.loads(l); print($i, d['kernel'].split('/')[-1], d['mismatching_lanes'])"
done
