# Round 6: what the rules trajectory's critical waves cost, by ablation
# (measurement builds, wrong results, alternating processes against the
# product; c3 and the bare trajectory at 2^20): the reset group without its
# deals (COUP_ABLATE_TRAJ_RESET), the Philox products from full-rate 24-bit
# multiplies (COUP_ABLATE_PHILOX_FULLRATE), 5 Philox rounds instead of 10.
set -u
. tools/gpu_calls/attempt.sh r06s
L="open_spiel_coup_amd/libcoup_mi355x.so build/libab/ablreset.so build/libab/fullrate.so build/libab/philox5.so"
for c in "c2 --batch 1048576" "c3"; do
  n=$(echo $c | tr -d ' -')
  timeout -k 10 600 python -u tools/bench_ab.py --rounds 3 $L -- --config $c --steps 20 --warmup 5 > $D/ab_$n.jsonl 2> $D/ab_$n.err || { tail -20 $D/ab_$n.err; exit 1; }
  echo "== $c"; grep median $D/ab_$n.jsonl
done
