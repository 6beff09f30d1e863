set -u
mkdir -p gpurun_out/r02e
timeout -k 10 120 build/slot_inline_repro 200000 > gpurun_out/r02e/repro.txt 2>&1 || exit $?
tail -3 gpurun_out/r02e/repro.txt | cut -c1-600
COUP_LIB_PATH=build/libcoup_inline.so timeout -k 10 300 python -u -m pytest tests/test_gpu_slot_pool.py -q --timeout 150 --timeout-method thread -k "tree_walk_clones or illegal_action" > gpurun_out/r02e/inline_pool.log 2>&1
echo "inline-variant pool tests rc=$?"
tail -3 gpurun_out/r02e/inline_pool.log
bash tools/gpu_call_suite.sh r02e
