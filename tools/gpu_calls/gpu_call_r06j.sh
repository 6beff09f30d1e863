# Round 6: the rules trajectory with its packed record carried across the
# step loop (v1, -DCOUP_NO_RNG_CARRY) and with the Philox block carried
# through the regroup plus miss-sorted keys (v2, the product build), against
# the round's previous product build (base): parity of the trajectory /
# step_many / every-lane / headline tests on the product build, then
# alternating-process bench lines (c3 and the bare rules trajectory at 2^20).
set -u
. tools/gpu_calls/attempt.sh r06j
timeout -k 10 600 python -u -m pytest tests/test_gpu_every_lane.py tests/test_gpu_step_many.py tests/test_gpu_trajectory.py \
  tests/test_gpu_headline.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
L="build/libab/base.so build/libab/v1.so open_spiel_coup_amd/libcoup_mi355x.so"
timeout -k 10 600 python -u tools/bench_ab.py --rounds 4 $L -- --config c3 --steps 20 --warmup 5 > $D/ab_c3.jsonl 2> $D/ab_c3.err || { tail -20 $D/ab_c3.err; exit 1; }
grep median $D/ab_c3.jsonl
timeout -k 10 400 python -u tools/bench_ab.py --rounds 4 $L -- --config c2 --batch 1048576 --steps 20 --warmup 5 > $D/ab_c2big.jsonl 2> $D/ab_c2big.err || { tail -20 $D/ab_c2big.err; exit 1; }
grep median $D/ab_c2big.jsonl
# the 6-player trajectory with its packed record carried (no spills): base against the product build
timeout -k 10 400 python -u tools/bench_ab.py --rounds 3 build/libab/base.so open_spiel_coup_amd/libcoup_mi355x.so -- --config c4 --steps 20 --warmup 5 > $D/ab_c4.jsonl 2> $D/ab_c4.err || { tail -20 $D/ab_c4.err; exit 1; }
grep median $D/ab_c4.jsonl
# wave-level Philox evaluations per wave-step, without / with the carry (COUP_COUNT_PHILOX builds)
for v in count_v1 count_v2; do
  COUP_LIB_PATH=build/libab/$v.so timeout -k 10 120 python -u tools/philox_count.py --steps 10 > $D/$v.json 2> $D/$v.err || { tail -20 $D/$v.err; exit 1; }
  echo "$v $(cat $D/$v.json)"
done
