# Refined regroup keys default (plain keys: ab/plain.so): N-player parity under both builds, 6-player step and rollout A/B.
set -u
mkdir -p gpurun_out/r02ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nplayer.py > gpurun_out/r02ab/nplayer.log 2>&1 || { tail -20 gpurun_out/r02ab/nplayer.log; exit 1; }
tail -1 gpurun_out/r02ab/nplayer.log
COUP_LIB_PATH=ab/plain.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nplayer.py > gpurun_out/r02ab/nplayer_plain.log 2>&1 || { tail -20 gpurun_out/r02ab/nplayer_plain.log; exit 1; }
tail -1 gpurun_out/r02ab/nplayer_plain.log
timeout -k 10 400 bash tools/ab_builds.sh 4 open_spiel_coup_amd/libcoup_mi355x.so ab/plain.so -- --players 6 --obs 0 > gpurun_out/r02ab/ab_keys_step6.log 2>&1 || { tail gpurun_out/r02ab/ab_keys_step6.log; exit 1; }
grep variant gpurun_out/r02ab/ab_keys_step6.log | cut -c1-120
timeout -k 10 400 bash tools/ab_builds.sh 4 open_spiel_coup_amd/libcoup_mi355x.so ab/plain.so -- --players 6 --obs 0 --fused 20 > gpurun_out/r02ab/ab_keys_rollout6.log 2>&1 || { tail gpurun_out/r02ab/ab_keys_rollout6.log; exit 1; }
grep variant gpurun_out/r02ab/ab_keys_rollout6.log | cut -c1-120
