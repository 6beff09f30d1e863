# Round 6: the 6-player trajectory (c4's one launch): regrouping blocks of
# 512 / 256 lanes (measurement build, COUP_NP_SORT_THREADS) against the
# shipped 1024 after the packed-record carry, and the Philox rounds' share
# (COUP_ABLATE_PHILOX_ROUNDS=5, wrong streams); alternating processes.
set -u
. tools/gpu_calls/attempt.sh r06zc
P=open_spiel_coup_amd/libcoup_mi355x.so
V=build/variants/libcoup_mi355x.so
L="$P $V:COUP_NP_SORT_THREADS=512 $V:COUP_NP_SORT_THREADS=256 build/libab/philox5.so"
timeout -k 10 700 python -u tools/bench_ab.py --rounds 3 $L -- --config c4 --steps 20 --warmup 5 > $D/ab_c4.jsonl 2> $D/ab_c4.err || { tail -20 $D/ab_c4.err; exit 1; }
grep median $D/ab_c4.jsonl
# c3 with one 20-step rules launch (16-byte records: 320 MB at 2^20) against the 10-step default
P=open_spiel_coup_amd/libcoup_mi355x.so
timeout -k 10 600 python -u tools/bench_ab.py --rounds 3 $P $P:COUP_TRAJ_CHUNK=20 -- --config c3 --steps 20 --warmup 5 > $D/ab_c3_chunk20.jsonl 2> $D/ab_c3_chunk20.err || { tail -20 $D/ab_c3_chunk20.err; exit 1; }
grep median $D/ab_c3_chunk20.jsonl
