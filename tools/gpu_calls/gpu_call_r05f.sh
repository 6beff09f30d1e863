# Round 5: the c3 step's dependence on the GPU's power state (tools/dpm_probe.py:
# idle-gapped vs back-to-back replays of the bench's graph, and the store-only
# sweep, with the GPU metrics sampled read-only), then the whole GPU suite.
set -u
D=gpurun_out/r05f
mkdir -p $D
timeout -k 10 300 python -u tools/dpm_probe.py > $D/dpm_probe.jsonl 2> $D/dpm_probe.err || { tail -20 $D/dpm_probe.err; exit 1; }
grep '"mean_us"\|"box"' $D/dpm_probe.jsonl
bash tools/gpu_calls/gpu_call_r05b.sh
