# Round 5: the bench's first-replay gap (replay_probe: the timed K-step graph's
# first replay against later ones, back to back and after idle gaps; once
# under a kernel trace for per-dispatch durations), then the whole GPU suite
# (r05b) on the product library.
set -u
D=gpurun_out/r05e
mkdir -p $D
timeout -k 10 300 python -u tools/replay_probe.py > $D/replay_probe.jsonl 2> $D/replay_probe.err || { tail -20 $D/replay_probe.err; exit 1; }
cat $D/replay_probe.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/trace -o run -- python3 -u tools/replay_probe.py --replays 3 > $D/replay_probe_traced.jsonl 2> $D/replay_probe_traced.err || { tail -20 $D/replay_probe_traced.err; exit 1; }
cat $D/replay_probe_traced.jsonl
bash tools/gpu_calls/gpu_call_r05b.sh
