set -u
mkdir -p gpurun_out/r02j
timeout -k 10 400 python -u -m pytest tests/test_gpu_nplayer.py -x -q --timeout 150 --timeout-method thread -k "regrouped_step_equals or uniform_steps_match_spec" > gpurun_out/r02j/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r02j/pytest.log
if grep -q "Timeout +++" gpurun_out/r02j/pytest.log; then exit 3; fi
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/boxinfo.sh > gpurun_out/r02j/box.txt 2>&1
timeout -k 10 300 python -u tools/ab_step.py --players 6 --obs 0 --rounds 7 --steps 20 COUP_DEAL_DEFER=0 COUP_DEAL_DEFER=1 STATS=0,COUP_DEAL_DEFER=0 STATS=0,COUP_DEAL_DEFER=1 > gpurun_out/r02j/ab_c4_defer.jsonl 2>gpurun_out/r02j/ab.err || exit $?
cat gpurun_out/r02j/ab_c4_defer.jsonl
exit $rc
