set -u
mkdir -p gpurun_out/r02k
bash tools/gpu_call_suite.sh r02k || exit $?
bash tools/boxinfo.sh > gpurun_out/r02k/box.txt 2>&1
for cfg in "c3:--obs 1" "c2:--batch 65536 --obs 0" "c2r:--batch 65536 --obs 0 --fused 20" "b20:--obs 0"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 400 bash tools/ab_builds.sh 3 build/libcoup_v1.so build/libcoup_v2.so -- $args > gpurun_out/r02k/ab_rules_$name.txt 2>&1 || exit $?
  echo "== $name"; cat gpurun_out/r02k/ab_rules_$name.txt
done
