# Round 6: confirm the reset / deal waves at s_setprio 3 (-DCOUP_TRAJ_PRIO=3)
# against the product with more rounds: c3 x 6, the bare trajectory at 2^20 x 4.
set -u
. tools/gpu_calls/attempt.sh r06v
L="open_spiel_coup_amd/libcoup_mi355x.so build/libab/prio3.so"
timeout -k 10 600 python -u tools/bench_ab.py --rounds 6 $L -- --config c3 --steps 20 --warmup 5 > $D/ab_c3.jsonl 2> $D/ab_c3.err || { tail -20 $D/ab_c3.err; exit 1; }
echo "== c3"; grep median $D/ab_c3.jsonl
timeout -k 10 600 python -u tools/bench_ab.py --rounds 4 $L -- --config c2 --batch 1048576 --steps 20 --warmup 5 > $D/ab_c2big.jsonl 2> $D/ab_c2big.err || { tail -20 $D/ab_c2big.err; exit 1; }
echo "== c2big"; grep median $D/ab_c2big.jsonl
