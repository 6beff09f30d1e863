# Round 6: the rules trajectory's chunk length on the shipped kernel.  The
# c3 trace (r06q) puts a fixed ~14 us on each chunk launch (130 us per 8-step
# chunk, 71-73 us per 4-step one); K = 20 runs as 8 + 8 + 4.  Chunks of 10
# (two launches) and 7 (7 + 7 + 6) against the default, alternating processes.
set -u
. tools/gpu_calls/attempt.sh r06w
P=open_spiel_coup_amd/libcoup_mi355x.so
L="$P $P:COUP_TRAJ_CHUNK=10 $P:COUP_TRAJ_CHUNK=7"
timeout -k 10 700 python -u tools/bench_ab.py --rounds 5 $L -- --config c3 --steps 20 --warmup 5 > $D/ab_c3.jsonl 2> $D/ab_c3.err || { tail -20 $D/ab_c3.err; exit 1; }
grep median $D/ab_c3.jsonl
