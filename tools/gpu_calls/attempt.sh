# Source from a GPU-call script: `. tools/gpu_calls/attempt.sh NAME` sets D to a
# directory no earlier attempt used, gpurun_out/NAME/<UTC time>-<pid>, so a retry
# never overwrites a failed attempt's logs (call r05j's crash
# log was lost that way).
D="gpurun_out/${1:?call name}/$(date -u +%Y%m%dT%H%M%S)-$$"
mkdir -p "$D"
echo "attempt dir: $D"
