# Round 6: profiles of the shipped tree (tools/profile_gpu.sh: the driver's
# command traced, then FETCH / WRITE / SQ passes in runs of their own) for c3,
# and for c4 / c2, whose kernels changed (the line's VALU issue fraction reads
# profiles/traffic.json).
set -u
. tools/gpu_calls/attempt.sh r06q
for c in c3 c4 c2; do
  timeout -k 10 400 bash tools/profile_gpu.sh r06 $c > $D/profile_$c.log 2>&1 || { tail -30 $D/profile_$c.log; exit 1; }
  tail -2 $D/profile_$c.log
done
