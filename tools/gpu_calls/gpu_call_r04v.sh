# Round 4, twenty-second call: where the split InformationStateTensor writer
# differs from the fused one (B = 1000, one and three steps), against the oracle.
set -u
D=gpurun_out/r04v
mkdir -p $D
timeout -k 10 120 python -u tools/info_split_diag.py 1000 3 > $D/diag.txt 2>&1 || { tail -20 $D/diag.txt; exit 1; }
cat $D/diag.txt
# (second run of this call: the prefix words written one row per thread as
# 32-bit values) then the equality tests and the c3i A/B if they hold
bash tools/gpu_calls/gpu_call_r04u.sh
