# Round 5: the c3 profile of the shipped form (coup_step_many's rules
# trajectory + writers, power warm-up on: tools/profile_gpu.sh r05 c3), then
# the whole GPU suite and the other configs' lines (r05b).
set -u
timeout -k 10 1000 bash tools/profile_gpu.sh r05 c3 > gpurun_out/profile_r05_c3.log 2>&1 || { tail -30 gpurun_out/profile_r05_c3.log; exit 1; }
tail -3 gpurun_out/profile_r05_c3.log
bash tools/gpu_calls/gpu_call_r05b.sh
