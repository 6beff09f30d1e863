# Ballot sort (default) vs LDS-atomic sort (ab/lds_atomic.so): N-player parity, 6-player step / rollout A/B.
set -u
mkdir -p gpurun_out/r02z
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nplayer.py > gpurun_out/r02z/nplayer.log 2>&1 || { tail -20 gpurun_out/r02z/nplayer.log; exit 1; }
tail -1 gpurun_out/r02z/nplayer.log
timeout -k 10 400 bash tools/ab_builds.sh 4 open_spiel_coup_amd/libcoup_mi355x.so ab/lds_atomic.so -- --players 6 --obs 0 > gpurun_out/r02z/ab_sort_step6.log 2>&1 || { tail gpurun_out/r02z/ab_sort_step6.log; exit 1; }
cat gpurun_out/r02z/ab_sort_step6.log | cut -c1-150
timeout -k 10 400 bash tools/ab_builds.sh 4 open_spiel_coup_amd/libcoup_mi355x.so ab/lds_atomic.so -- --players 6 --obs 0 --fused 20 > gpurun_out/r02z/ab_sort_rollout6.log 2>&1 || { tail gpurun_out/r02z/ab_sort_rollout6.log; exit 1; }
cat gpurun_out/r02z/ab_sort_rollout6.log | cut -c1-150
