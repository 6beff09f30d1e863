set -u
mkdir -p gpurun_out/r02l
timeout -k 10 400 python -u -m pytest tests/test_gpu_nplayer.py tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -k "regrouped or uniform_steps_match_spec or full_batch_sampled" > gpurun_out/r02l/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r02l/pytest.log
if grep -q "Timeout +++" gpurun_out/r02l/pytest.log; then exit 3; fi
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/boxinfo.sh > gpurun_out/r02l/box.txt 2>&1
timeout -k 10 400 bash tools/ab_builds.sh 3 build/libcoup_np_base.so build/libcoup_np_raw.so -- --players 6 --obs 0 > gpurun_out/r02l/ab_np_raw_c4.txt 2>&1 || exit $?
grep libcoup gpurun_out/r02l/ab_np_raw_c4.txt
timeout -k 10 400 bash tools/ab_builds.sh 3 build/libcoup_v1.so build/libcoup_v2.so -- --obs 0 --fused 20 > gpurun_out/r02l/ab_rules_b20r.txt 2>&1 || exit $?
grep libcoup gpurun_out/r02l/ab_rules_b20r.txt
exit $rc
