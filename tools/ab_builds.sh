#!/bin/bash
# A/B several builds of libcoup_mi355x.so on one GPU box: alternate processes
# (lib1, lib2, ..., lib1, lib2, ...) running tools/ab_step.py with the
# default knobs, so box-to-box variance cancels.  Measurement tool only.
#   usage: tools/ab_builds.sh <rounds> <lib1.so> <lib2.so> [more.so ...] [-- ab_step.py args...]
set -euo pipefail
R=$1; shift
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
for i in $(seq 1 "$R"); do
  for lib in "${LIBS[@]}"; do
    out=$(COUP_LIB_PATH=$lib timeout -k 10 120 python tools/ab_step.py --rounds 2 "$@" COUP_OBS_MODE=9 | grep variant)
    echo "$(basename "$lib") $out"
  done
done
