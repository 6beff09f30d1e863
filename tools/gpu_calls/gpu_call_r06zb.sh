# Round 6: the c3 step's fixed per-step cost -- the same split form (rules
# trajectory + k_obs_sweep_rows<512, 2>, COUP_OBS_SPLIT=11) at 2^18, 2^19 and
# 2^20 lanes, alternating processes: T(B) = a + b B puts a launch-and-tail
# cost a per step beside the per-lane work.
set -u
. tools/gpu_calls/attempt.sh r06zb
P=open_spiel_coup_amd/libcoup_mi355x.so
for b in 262144 524288 1048576; do
  timeout -k 10 400 python -u tools/bench_ab.py --rounds 3 $P:COUP_OBS_SPLIT=11 -- --config c3 --batch $b --steps 20 --warmup 5 > $D/c3_$b.jsonl 2> $D/c3_$b.err || { tail -20 $D/c3_$b.err; exit 1; }
  echo "$b $(grep median $D/c3_$b.jsonl)"
done
