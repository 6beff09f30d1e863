# Round 4, thirteenth call: confirmation of the tree after the host-side
# facade changes and the reset-ahead revert -- the whole GPU suite, smoke(),
# and the driver's default bench line.
set -u
D=gpurun_out/r04m
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
cut -c1-600 $D/bench.json
# c2 (65,536 lanes) with the lanes regrouped by decision in 256- / 512-lane
# blocks, against the shipped group step (round 2 measured regrouping slower
# below 2^18 lanes, before PrefRng and the packed episode word)
timeout -k 10 120 python -u tools/ab_step.py --batch 65536 --obs 0 --rounds 11 "" COUP_REGROUP=1,COUP_SORT_THREADS=256 COUP_REGROUP=1,COUP_SORT_THREADS=512 > $D/ab_c2_regroup.jsonl 2> $D/ab_c2_regroup.err || { tail -5 $D/ab_c2_regroup.err; exit 1; }
cut -c1-110 $D/ab_c2_regroup.jsonl
