# Round 5, last tree: the c3 profile again (tools/profile_gpu.sh: the driver's
# command traced, then FETCH_SIZE / WRITE_SIZE / SQ passes in runs of their own).
set -u
timeout -k 10 900 bash tools/profile_gpu.sh r05 c3 > gpurun_out/profile_r05_c3_zq.log 2>&1 || { tail -30 gpurun_out/profile_r05_c3_zq.log; exit 1; }
tail -3 gpurun_out/profile_r05_c3_zq.log
