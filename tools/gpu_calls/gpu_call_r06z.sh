# Round 6: the shipped tree (balanced 10-step chunks, in-place last-step
# resets) on the whole GPU suite; then whether the Infinity Cache absorbs
# part of a split writer's stores when one tensor buffer is rewritten every
# step (tools/mall_probe.py: one buffer against two alternating ones, c3 and c3i).
set -u
. tools/gpu_calls/attempt.sh r06z
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 200 python -u tools/mall_probe.py > $D/mall_c3.json 2> $D/mall_c3.err || { tail -20 $D/mall_c3.err; exit 1; }
cat $D/mall_c3.json
timeout -k 10 300 python -u tools/mall_probe.py --info --rounds 5 > $D/mall_c3i.json 2> $D/mall_c3i.err || { tail -20 $D/mall_c3i.err; exit 1; }
cat $D/mall_c3i.json
