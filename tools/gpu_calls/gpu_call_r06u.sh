# Round 6: the rules trajectory with its slow waves raised in priority
# (measurement builds -DCOUP_TRAJ_PRIO=2 / 3: s_setprio in the reset group's
# waves and in waves with deals, back to 0 at the next step), so the VALU
# arbiter serves the block's critical path first; alternating processes
# against the product, the bare trajectory at 2^20 and c3.
set -u
. tools/gpu_calls/attempt.sh r06u
L="open_spiel_coup_amd/libcoup_mi355x.so build/libab/prio2.so build/libab/prio3.so"
for c in "c2 --batch 1048576" "c3"; do
  n=$(echo $c | tr -d ' -')
  timeout -k 10 600 python -u tools/bench_ab.py --rounds 4 $L -- --config $c --steps 20 --warmup 5 > $D/ab_$n.jsonl 2> $D/ab_$n.err || { tail -20 $D/ab_$n.err; exit 1; }
  echo "== $c"; grep median $D/ab_$n.jsonl
done
