# Round 6: the reverted 8-byte observation-record build (commit d56e9d4, as a
# measurement library) against the shipped tree, alternating processes of the
# driver's c3 command: words at 10-step chunks and at one 20-step launch.
set -u
. tools/gpu_calls/attempt.sh r06ze
P=open_spiel_coup_amd/libcoup_mi355x.so
W=build/libab/words.so
timeout -k 10 800 python -u tools/bench_ab.py --rounds 4 $P $W $W:COUP_TRAJ_CHUNK=20 -- --config c3 --steps 20 --warmup 5 > $D/ab_c3.jsonl 2> $D/ab_c3.err || { tail -20 $D/ab_c3.err; exit 1; }
grep median $D/ab_c3.jsonl
