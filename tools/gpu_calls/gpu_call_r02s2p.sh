# Round 2, session 2: 6-player step with bins_below instead of the wave-0 scan (one barrier fewer) -- N-player suite, then
# alternating-process A/B of the previous build (ab/base.so) and this one (ab/new.so).
set -u
D=gpurun_out/r02s2p
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_nplayer.py tests/test_gpu_trajectory.py -x -v --timeout 150 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 600 bash tools/ab_builds.sh 5 ab/base.so ab/new.so -- --players 6 --obs 0 --steps 20 > $D/ab_c4_bins_below.log 2>&1 || { tail $D/ab_c4_decision_node.log; exit 1; }
cat $D/ab_c4_bins_below.log
