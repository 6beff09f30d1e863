# Round 6: is the r06 library itself off (smoke, the slice tests), or the every-lane checker?
set -u
. tools/gpu_calls/attempt.sh r06c
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1; echo "smoke rc=$?"; tail -3 $D/smoke.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > $D/parity.log 2>&1; echo "parity rc=$?"; tail -3 $D/parity.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_headline.py -k c3_headline > $D/headline.log 2>&1; echo "headline rc=$?"; tail -3 $D/headline.log
