#!/bin/bash
# A/B two builds of libcoup_mi355x.so on one GPU box: alternate processes
# (base, new, base, new, ...) running tools/ab_step.py with the default
# knobs, so box-to-box variance cancels.  Measurement tool only.
#   usage: tools/ab_builds.sh <base.so> <new.so> <rounds> [ab_step.py args...]
set -euo pipefail
BASE=$1; NEW=$2; R=$3; shift 3
for i in $(seq 1 "$R"); do
  for tag in base new; do
    lib=$BASE; [ "$tag" = new ] && lib=$NEW
    out=$(COUP_LIB_PATH=$lib timeout -k 10 120 python tools/ab_step.py --rounds 2 "$@" COUP_OBS_MODE=4 | grep variant)
    echo "$tag $out"
  done
done
