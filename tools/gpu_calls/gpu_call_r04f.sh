# Round 4, sixth call: where a 256-env SyncVectorEnv step's time goes
# (tools/vector_env_profile.py), then rocprofv3 kernel trace + PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ issue mix) of the round-4 build's c3
# (headline), c2 (k_step_group<1>) and c4 lines, the driver's bench command
# each (tools/profile_gpu.sh; tools/traffic.py condenses them locally).
set -u
mkdir -p gpurun_out/r04f
timeout -k 10 240 python -u tools/vector_env_profile.py --steps 30 > gpurun_out/r04f/vector_env_profile.txt 2>&1 || { tail -20 gpurun_out/r04f/vector_env_profile.txt; exit 1; }
grep "===" gpurun_out/r04f/vector_env_profile.txt
bash tools/profile_gpu.sh r04 c3 && bash tools/profile_gpu.sh r04 c2 && bash tools/profile_gpu.sh r04 c4
