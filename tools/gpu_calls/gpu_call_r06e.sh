# Round 6: the rules trajectory's attribution / first cut:
# the DPP wave-scan bin prefix (COUP_BINS_DPP) -- its parity tests, then bench
# lines alternating the base library, the DPP one and a measurement build pricing
# the Philox products (full-rate 24-bit multiplies, wrong streams).
set -o pipefail
. tools/gpu_calls/attempt.sh r06e
COUP_LIB_PATH=build/ab_r06dpp/libcoup_mi355x.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_every_lane.py tests/test_gpu_step_many.py tests/test_gpu_trajectory.py > $D/dpp_tests.log 2>&1 || { tail -30 $D/dpp_tests.log; exit 1; }
tail -1 $D/dpp_tests.log
for r in 1 2; do
  for lib in base dpp mix; do
    export COUP_LIB_PATH=build/ab_r06$lib/libcoup_mi355x.so
    for c in "c3" "c2 --batch 1048576" "c4" "c2"; do
      n=$(echo $c | tr -d ' -')
      timeout -k 10 120 python3 -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $D/${n}_${lib}_$r.json 2> $D/${n}_${lib}_$r.err || { tail -5 $D/${n}_${lib}_$r.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['value']/1e9,3), round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3/d['config']['fused_steps_per_launch'],2))" $D/${n}_${lib}_$r.json "$c" $lib
    done
  done
done
