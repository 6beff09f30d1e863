#!/bin/bash
# Round 5: the product library built with -structurizecfg-skip-uniform-regions (r05zn part 2 only).
# reproducer built with SLP on (the construct that made -fno-slp-vectorize
# necessary), with and without the flag, and with the product's flags.
# (2) The product library built with the flag (build/structflag): the main
# parity tests through it and the c3 / c2 / c4 lines beside the shipped
# library's, alternating.
set -u
D=gpurun_out/r05zo
mkdir -p $D
for v in; do
  timeout -k 10 120 build/structflag/slot_repro_$v 200000 > $D/slot_$v.jsonl 2> $D/slot_$v.err || { tail -5 $D/slot_$v.err; exit 1; }
  python3 -c "
import json,sys
for l in open('$D/slot_$v.jsonl'):
    if not l.startswith('{'): continue
    d=json.loads(l)
    if 'slot_variants' in d: print('$v', 'slot', {k: v['mismatch'] for k, v in d['slot_variants'].items()})
    else: print('$v', 'uniform', d.get('uniform_inline_mismatch'), d.get('uniform_call_mismatch'))"
done
COUP_LIB_PATH=build/structflag/libcoup_mi355x.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_properties.py tests/test_gpu_step_many.py tests/test_gpu_trajectory.py tests/test_gpu_headline.py tests/test_gpu_slot_pool.py tests/test_gpu_nplayer.py > $D/tests_flag.log 2>&1 || { tail -30 $D/tests_flag.log; exit 1; }
tail -1 $D/tests_flag.log
for r in 1 2; do
  for lib in base flag; do
    if [ $lib = flag ]; then export COUP_LIB_PATH=build/structflag/libcoup_mi355x.so; else unset COUP_LIB_PATH; fi
    for c in c3 c2 c4; do
      timeout -k 10 200 python3 -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $D/${c}_${lib}_$r.json 2> $D/${c}_${lib}_$r.err || exit 1
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['value']/1e9,3), round(d['ms_per_step']*1e3,2))" $D/${c}_${lib}_$r.json $c $lib
    done
  done
done
