# Round 6: c2 (65,536 lanes, tensor-free, one trajectory launch per K steps)
# in place (k_step_trajectory, one wave per SIMD: latency-bound) against the
# regrouped trajectory at this size -- 64 / 128 / 256 blocks of 1024 / 512 /
# 256 lanes (measurement build knobs COUP_REGROUP=1, COUP_SORT_THREADS);
# alternating processes of the driver's c2 command.
set -u
. tools/gpu_calls/attempt.sh r06t
V=build/variants/libcoup_mi355x.so
L="open_spiel_coup_amd/libcoup_mi355x.so $V:COUP_REGROUP=1 $V:COUP_REGROUP=1,COUP_SORT_THREADS=512 $V:COUP_REGROUP=1,COUP_SORT_THREADS=256"
timeout -k 10 600 python -u tools/bench_ab.py --rounds 3 $L -- --config c2 --steps 20 --warmup 5 > $D/ab_c2.jsonl 2> $D/ab_c2.err || { tail -20 $D/ab_c2.err; exit 1; }
grep median $D/ab_c2.jsonl
