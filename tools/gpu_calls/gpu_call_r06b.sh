# Round 6: the c3 every-lane failure of call r06a -- which stage differs first.
set -u
. tools/gpu_calls/attempt.sh r06b
timeout -k 10 300 python -u tools/every_lane_diag.py > $D/diag.jsonl 2> $D/diag.err || { tail -20 $D/diag.err; cat $D/diag.jsonl; exit 1; }
cat $D/diag.jsonl
