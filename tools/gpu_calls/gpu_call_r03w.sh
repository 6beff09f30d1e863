# Round 3: compiler scheduling variants of the (no-SLP) library -- A/B in
# alternating processes on one box for the c3, c4 and c2 steps.
set -u
D=gpurun_out/r03w
mkdir -p $D
L0=$PWD/open_spiel_coup_amd/libcoup_mi355x.so
LS="$L0 $PWD/build/flags/lib_maxilp.so $PWD/build/flags/lib_memclause.so $PWD/build/flags/lib_o2.so $PWD/build/flags/lib_occ.so"
timeout -k 10 500 bash tools/ab_builds.sh 3 $LS > $D/ab_c3.txt 2>&1 || { tail -5 $D/ab_c3.txt; exit 1; }
grep -v amdgpu.ids $D/ab_c3.txt
timeout -k 10 500 bash tools/ab_builds.sh 3 $LS -- --players 6 --obs 0 > $D/ab_c4.txt 2>&1 || { tail -5 $D/ab_c4.txt; exit 1; }
grep -v amdgpu.ids $D/ab_c4.txt
timeout -k 10 500 bash tools/ab_builds.sh 3 $LS -- --batch 65536 --obs 0 > $D/ab_c2.txt 2>&1 || { tail -5 $D/ab_c2.txt; exit 1; }
grep -v amdgpu.ids $D/ab_c2.txt
