# Round 3: is LLVM's SLP vectorizer the trigger of the section-12 defect in
# every shape?  (1) the run-time-branch step of commit 0ce2c98 with and
# without -fno-slp-vectorize under the test that caught it; (2) the k_slot
# reproducer built without SLP; (3) same-process-alternating A/B of the
# current library with and without SLP on the c3, c2 and c4 steps.
set -u
D=gpurun_out/r03s
mkdir -p $D
for v in rtb_slp rtb_noslp; do
  COUP_LIB_PATH=$PWD/build/slp/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_server.py -m gpu -q --timeout 200 --timeout-method thread -k lane_ops_equal > $D/pytest_$v.log 2>&1
  echo "$v rc=$? $(tail -1 $D/pytest_$v.log)"
done
timeout -k 10 120 build/slp/repro_noslp 200000 > $D/repro_noslp.txt 2> $D/repro_noslp.err || { echo "repro failed"; tail -5 $D/repro_noslp.err; exit 1; }
python3 -c "
import json
lines=[json.loads(l) for l in open('$D/repro_noslp.txt') if l.startswith('{')]
print({k: v['mismatch'] for k, v in lines[0]['slot_variants'].items()}, lines[-1]['uniform_inline_mismatch'], lines[-1]['uniform_call_mismatch'])"
L1=$PWD/open_spiel_coup_amd/libcoup_mi355x.so; L2=$PWD/build/slp/lib_noslp.so
timeout -k 10 400 bash tools/ab_builds.sh 4 $L1 $L2 > $D/ab_c3.txt 2>&1 || { tail -5 $D/ab_c3.txt; exit 1; }
cat $D/ab_c3.txt
timeout -k 10 400 bash tools/ab_builds.sh 4 $L1 $L2 -- --batch 65536 --obs 0 > $D/ab_c2.txt 2>&1 || { tail -5 $D/ab_c2.txt; exit 1; }
cat $D/ab_c2.txt
timeout -k 10 400 bash tools/ab_builds.sh 4 $L1 $L2 -- --players 6 --obs 0 > $D/ab_c4.txt 2>&1 || { tail -5 $D/ab_c4.txt; exit 1; }
cat $D/ab_c4.txt
