#!/bin/bash
# Round 5: the Rng block carried through the regroup (k_trajectory_sorted,
# k_rollout_sorted): parity tests on the new library, then bench lines
# alternating the previous library (build/ab_base) and the new one.
set -o pipefail
O=gpurun_out/r05zj
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_trajectory.py tests/test_gpu_step_many.py tests/test_gpu_parity.py tests/test_gpu_properties.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then export COUP_LIB_PATH=build/ab_base/libcoup_mi355x.so; else unset COUP_LIB_PATH; fi
    for c in "c3" "c2" "c2 --batch 1048576" "c2r"; do
      n=$(echo $c | tr -d ' -')
      timeout -k 10 120 python3 -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/${n}_${lib}_$r.json 2> $O/${n}_${lib}_$r.err || exit 1
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['value']/1e9,3), round(d['ms_per_step']*1e3,2))" $O/${n}_${lib}_$r.json "$c" $lib
    done
  done
done
