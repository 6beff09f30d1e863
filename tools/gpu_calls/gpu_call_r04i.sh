# Round 4, ninth call: round-4 profiles of the other bench configs whose
# kernels changed this round (packed episode word): c3i (InformationState
# tensor, 2^18 lanes), c4t (6-player trajectory), c2t (2-player trajectory).
set -u
bash tools/profile_gpu.sh r04 c3i && bash tools/profile_gpu.sh r04 c4t && bash tools/profile_gpu.sh r04 c2t
