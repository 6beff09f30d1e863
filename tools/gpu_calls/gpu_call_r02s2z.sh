# Round 2, session 2: 6-player step, 512- vs 1024-lane regrouping blocks, interleaved in one process, two processes.
set -u
D=gpurun_out/r02s2z
mkdir -p $D
for i in 1 2; do
  timeout -k 10 300 python -u tools/ab_step.py --players 6 --obs 0 --rounds 11 --steps 20 COUP_NP_SORT_THREADS=512 COUP_NP_SORT_THREADS=1024 >> $D/ab_np_block.jsonl 2>$D/ab.err || { tail $D/ab.err; exit 1; }
done
cat $D/ab_np_block.jsonl
