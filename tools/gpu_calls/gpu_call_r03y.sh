# Round 3: -O2 against -O3 for the N-player trajectory and rollout kernels
# (tools/traj_ab.py, alternating processes: the product library, N-player
# file at -O2, against build/slp/lib_noslp.so, both files at -O3).
set -u
D=gpurun_out/r03y
mkdir -p $D
for i in 1 2 3; do
  for lib in $PWD/open_spiel_coup_amd/libcoup_mi355x.so $PWD/build/ab/lib_o3.so; do
    COUP_LIB_PATH=$lib timeout -k 10 200 python -u tools/traj_ab.py --players 6 --steps 50 --rounds 2 > $D/traj_$i_$(basename $lib).jsonl 2> $D/traj.err || { tail -5 $D/traj.err; exit 1; }
    echo "$(basename $lib) $(tr '\n' ' ' < $D/traj_$i_$(basename $lib).jsonl | cut -c1-600)"
  done
done
