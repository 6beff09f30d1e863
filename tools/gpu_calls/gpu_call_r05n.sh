# Round 5: the rules trajectory's chunk length (6 / 8 / 10 / 12 / 16 steps per
# launch; r05m: 16 measured 165 us per step against 134.5 at 8), then a
# kernel trace of chunk 8 against 16 to see which kernel slows.
set -u
D=gpurun_out/r05n
mkdir -p $D
timeout -k 10 400 python -u tools/pipe_ab.py > $D/pipe_ab.jsonl 2> $D/pipe_ab.err || { tail -20 $D/pipe_ab.err; exit 1; }
cat $D/pipe_ab.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/trace -o run -- python3 -u tools/pipe_ab.py --rounds 3 traj8:COUP_PIPE=1 traj16:COUP_TRAJ_CHUNK=16 > $D/traced.jsonl 2> $D/traced.err || { tail -20 $D/traced.err; exit 1; }
cat $D/traced.jsonl
