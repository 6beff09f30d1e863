# Round 4: smoke() with the split writers forced on at its size.
set -u
D=gpurun_out/r04zc
mkdir -p $D
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -30 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
