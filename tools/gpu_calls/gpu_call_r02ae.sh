# Branch-free policy draw (ab/select.so): parity under that build, A/B on c4 / c4r / c2r / c3.
set -u
mkdir -p gpurun_out/r02ae
COUP_LIB_PATH=ab/select.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_nplayer.py > gpurun_out/r02ae/parity_select.log 2>&1 || { tail -20 gpurun_out/r02ae/parity_select.log; exit 1; }
tail -1 gpurun_out/r02ae/parity_select.log
for args in "--players 6 --obs 0" "--players 6 --obs 0 --fused 20" "--players 2 --obs 0 --batch 65536 --fused 20" "--players 2 --obs 1"; do
  echo "## $args"
  timeout -k 10 400 bash tools/ab_builds.sh 3 open_spiel_coup_amd/libcoup_mi355x.so ab/select.so -- $args > gpurun_out/r02ae/ab.log 2>&1 || { tail gpurun_out/r02ae/ab.log; exit 1; }
  grep variant gpurun_out/r02ae/ab.log | cut -c1-110
done
