# Round 2, session 2: per-op State latency with host-polled completion flags vs stream synchronisation
# (COUP_SLOT_SYNC=1), alternating processes on one box.
set -u
D=gpurun_out/r02s2v
mkdir -p $D
for i in 1 2; do
  for v in 0 1; do
    COUP_SLOT_SYNC=$v timeout -k 10 300 python -u tools/facade_latency.py 2>/dev/null > $D/facade_sync$v.$i.json || exit 1
    python -c "import json; d=json.load(open('$D/facade_sync$v.$i.json')); print('sync=$v', {k: v for k, v in d.items() if k.startswith(('pool', 'rl_', 'children_n1_', 'children_n7_', 'children_n64_us', 'apply'))})"
  done
done
