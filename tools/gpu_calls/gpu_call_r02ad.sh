# 2-player sorted kernels at 512 / 1024-lane blocks with refined keys: parity (default and plain-key builds), key A/B.
set -u
mkdir -p gpurun_out/r02ad
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_nplayer.py > gpurun_out/r02ad/parity.log 2>&1 || { tail -20 gpurun_out/r02ad/parity.log; exit 1; }
tail -1 gpurun_out/r02ad/parity.log
COUP_LIB_PATH=ab/plain.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "regroup or oracle or golden" > gpurun_out/r02ad/parity_plain.log 2>&1 || { tail -20 gpurun_out/r02ad/parity_plain.log; exit 1; }
tail -1 gpurun_out/r02ad/parity_plain.log
timeout -k 10 400 bash tools/ab_builds.sh 3 open_spiel_coup_amd/libcoup_mi355x.so ab/plain.so -- --players 2 --obs 0 > gpurun_out/r02ad/ab_keys_step2.log 2>&1 || { tail gpurun_out/r02ad/ab_keys_step2.log; exit 1; }
grep variant gpurun_out/r02ad/ab_keys_step2.log | cut -c1-110
timeout -k 10 400 bash tools/ab_builds.sh 3 open_spiel_coup_amd/libcoup_mi355x.so ab/plain.so -- --players 2 --obs 0 --fused 20 > gpurun_out/r02ad/ab_keys_rollout2.log 2>&1 || { tail gpurun_out/r02ad/ab_keys_rollout2.log; exit 1; }
grep variant gpurun_out/r02ad/ab_keys_rollout2.log | cut -c1-110
