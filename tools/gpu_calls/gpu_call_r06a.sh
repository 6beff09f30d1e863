# Round 6, first call: the every-lane parity tests at the bench sizes (VERDICT r5
# item 1), the step_many / trajectory / capi tests touched by the launch log and
# the traj_rec allocation change, smoke(), and the driver's default line.
set -u
. tools/gpu_calls/attempt.sh r06a
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_every_lane.py > $D/every_lane.log 2>&1 || { tail -40 $D/every_lane.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $D/every_lane.log | tail -6
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_step_many.py tests/test_gpu_trajectory.py tests/test_gpu_parity.py tests/test_gpu_headline.py \
  tests/test_gpu_ab_variants.py > $D/pytest_subset.log 2>&1 || { tail -40 $D/pytest_subset.log; exit 1; }
tail -2 $D/pytest_subset.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench.json')); r=d['roofline']; print('c3', d['value'], r['frac'], r['kernel_ms'], r['kernel'] == r['kernel_launched'], r.get('valu_issue_frac'), r['bound'])"
