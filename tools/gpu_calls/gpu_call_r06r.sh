# Round 6: (1) c2 (k_step_trajectory in place, 65,536 lanes) read 5.9 us per
# step in call r06q's profile against round 5's 4.4-4.6: alternating processes
# of the round-start build (base), the shipped tree with rounds 1-5's Rng word
# select (chain, -DCOUP_RNG_SELECT_CHAIN) and the shipped tree, for c2, c2r and
# c4; (2) the 6-player trajectory's Philox evaluations and phase timing
# (COUP_COUNT_PHILOX / COUP_TRAJ_PHASES builds).
set -u
. tools/gpu_calls/attempt.sh r06r
L="build/libab/base.so build/libab/chain.so open_spiel_coup_amd/libcoup_mi355x.so"
for c in "c2" "c2r" "c4"; do
  timeout -k 10 400 python -u tools/bench_ab.py --rounds 3 $L -- --config $c --steps 20 --warmup 5 > $D/ab_$c.jsonl 2> $D/ab_$c.err || { tail -20 $D/ab_$c.err; exit 1; }
  echo "== $c"; grep median $D/ab_$c.jsonl
done
COUP_LIB_PATH=build/libab/count.so timeout -k 10 120 python -u tools/philox_count.py --players 6 --steps 10 > $D/count_6p.json 2> $D/count_6p.err || { tail -20 $D/count_6p.err; exit 1; }
cat $D/count_6p.json
COUP_LIB_PATH=build/libab/count.so timeout -k 10 120 python -u tools/philox_count.py --players 2 --steps 10 > $D/count_2p.json 2> $D/count_2p.err || { tail -20 $D/count_2p.err; exit 1; }
cat $D/count_2p.json
COUP_LIB_PATH=build/libab/phases.so timeout -k 10 120 python -u tools/traj_phases.py --players 6 > $D/traj_phases_6p.jsonl 2> $D/traj_phases_6p.err || { tail -20 $D/traj_phases_6p.err; exit 1; }
cat $D/traj_phases_6p.jsonl
