# 6-player step: wave-priority variants (ab/prio<mask>.so, -DCOUP_NP_PRIO) against the default, alternating processes.
set -u
mkdir -p gpurun_out/r02ak
COUP_LIB_PATH=ab/prio7.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nplayer.py -k "regrouped_step" > gpurun_out/r02ak/parity_prio7.log 2>&1 || { tail -20 gpurun_out/r02ak/parity_prio7.log; exit 1; }
tail -1 gpurun_out/r02ak/parity_prio7.log
timeout -k 10 600 bash tools/ab_builds.sh 3 open_spiel_coup_amd/libcoup_mi355x.so ab/prio1.so ab/prio3.so ab/prio7.so -- --players 6 --obs 0 > gpurun_out/r02ak/ab_prio.log 2>&1 || { tail gpurun_out/r02ak/ab_prio.log; exit 1; }
grep variant gpurun_out/r02ak/ab_prio.log | cut -c1-110
