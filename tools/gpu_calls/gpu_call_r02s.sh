# c4: 128- vs 256-lane regroup blocks (parity + interleaved A/B + timeline).
set -u
mkdir -p gpurun_out/r02s
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nplayer.py > gpurun_out/r02s/nplayer.log 2>&1 || { tail -20 gpurun_out/r02s/nplayer.log; exit 1; }
tail -1 gpurun_out/r02s/nplayer.log
timeout -k 10 300 python -u tools/ab_step.py --players 6 --obs 0 --rounds 9 COUP_NP_SORT_THREADS=256 COUP_NP_SORT_THREADS=512 COUP_NP_SORT_THREADS=1024 > gpurun_out/r02s/ab_sort_threads.log 2>&1 || { tail gpurun_out/r02s/ab_sort_threads.log; exit 1; }
cat gpurun_out/r02s/ab_sort_threads.log
COUP_NP_SORT_THREADS=1024 COUP_LIB_PATH=ab/trace.so timeout -k 10 120 python -u tools/np_wave_trace.py --out gpurun_out/r02s/np_wave_trace_1024.json > gpurun_out/r02s/np_wave_trace_1024.log || exit $?
head -1 gpurun_out/r02s/np_wave_trace_1024.log | cut -c1-400
