# Round 3, first call: the new headline-size parity tests (c3 at 2^20, c3i at
# 2^18), the coup_slot_ops flag fix, the one-rank RCCL tests; then the c4
# profile of the shipped 6-player step (1024-lane blocks) with the driver's command.
set -u
D=gpurun_out/r03a
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_slot_pool.py tests/test_gpu_dist.py -x -v -s --timeout 200 --timeout-method thread > $D/pytest_new.log 2>&1 || { tail -40 $D/pytest_new.log; exit 1; }
tail -3 $D/pytest_new.log
timeout -k 10 900 bash tools/profile_gpu.sh r03 c4 --gpus 1 --steps 20 --warmup 5 > $D/prof_c4.log 2>&1 || { tail -20 $D/prof_c4.log; exit 1; }
tail -5 $D/prof_c4.log
