# Round 4, fifteenth call: the split-step premise again (tools/split_probe.hip)
# with one block per sweep chunk, LDS bitmaps and sc1 stores -- alone and
# overlapped with the bare step, beside the fused c3 step.
set -u
D=gpurun_out/r04o
mkdir -p $D
timeout -k 10 120 build/split/split_probe > $D/split_probe.jsonl 2> $D/split_probe.err || { tail -5 $D/split_probe.err; cat $D/split_probe.jsonl; exit 1; }
cat $D/split_probe.jsonl
