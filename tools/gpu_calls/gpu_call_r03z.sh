# Round 3, final tree: whole GPU suite, smoke(), the driver's default bench
# line, then -O2 against -O3 for the N-player trajectory / rollout kernels
# (tools/traj_ab.py in alternating processes: the product library, N-player
# file at -O2, against build/ab/lib_o3.so, both files at -O3, no SLP).
set -u
D=gpurun_out/r03z
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python -u bench.py > $D/bench_c3.json 2> $D/bench_c3.err || { tail -5 $D/bench_c3.err; exit 1; }
cut -c1-250 $D/bench_c3.json
for i in 1 2 3; do
  for lib in $PWD/open_spiel_coup_amd/libcoup_mi355x.so $PWD/build/ab/lib_o3.so; do
    COUP_LIB_PATH=$lib timeout -k 10 200 python -u tools/traj_ab.py --players 6 --steps 50 --rounds 2 > $D/traj_${i}_$(basename $lib).jsonl 2> $D/traj.err || { tail -5 $D/traj.err; exit 1; }
    echo "$(basename $lib) $(tr '\n' ' ' < $D/traj_${i}_$(basename $lib).jsonl | cut -c1-700)"
  done
done
