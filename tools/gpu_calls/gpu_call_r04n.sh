# Round 4, fourteenth call: the 6-player step (c4, 2^20 lanes) with 512-lane
# regrouping blocks again (moved to 1024 at the end of round 2, before the
# 4-thread reset groups and the packed episode word).
set -u
D=gpurun_out/r04n
mkdir -p $D
timeout -k 10 150 python -u tools/ab_step.py --players 6 --obs 0 --rounds 9 "" COUP_NP_SORT_THREADS=512 > $D/ab_c4_sort512.jsonl 2> $D/ab_c4_sort512.err || { tail -5 $D/ab_c4_sort512.err; exit 1; }
cut -c1-110 $D/ab_c4_sort512.jsonl
