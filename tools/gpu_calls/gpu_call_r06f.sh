# Round 6: the DPP bin prefix in the N-player kernels (COUP_NP_BINS_DPP) and the
# rules trajectory without output-pointer tests (COUP_TRAJ_FULL): parity on
# each build, then bench lines alternating them with the 2-player-DPP build.
set -o pipefail
. tools/gpu_calls/attempt.sh r06f
for lib in full; do
  COUP_LIB_PATH=build/ab_r06$lib/libcoup_mi355x.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_every_lane.py tests/test_gpu_step_many.py tests/test_gpu_trajectory.py tests/test_gpu_nplayer.py -k "not c3_every_lane" > $D/${lib}_tests.log 2>&1 || { tail -30 $D/${lib}_tests.log; exit 1; }
  echo "$lib: $(tail -1 $D/${lib}_tests.log)"
done
for r in 1 2; do
  for lib in dpp npdpp full; do
    export COUP_LIB_PATH=build/ab_r06$lib/libcoup_mi355x.so
    for c in "c3" "c2 --batch 1048576" "c4" "c4r"; do
      n=$(echo $c | tr -d ' -')
      timeout -k 10 120 python3 -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $D/${n}_${lib}_$r.json 2> $D/${n}_${lib}_$r.err || { tail -5 $D/${n}_${lib}_$r.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['value']/1e9,3), round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3/d['config']['fused_steps_per_launch'],2))" $D/${n}_${lib}_$r.json "$c" $lib
    done
  done
done
