# Round 5: the split writers' store policy (measurement build, COUP_WRITER_POL:
# 0 nt shipped, 1 plain, 2 sc1, 3 sc1 nt buffer stores) -- equality, then
# same-process A/Bs: c3 in the driver's graph form, c3i eager steps.
set -u
D=gpurun_out/r05x
mkdir -p $D
export COUP_LIB_PATH=build/variants/libcoup_mi355x.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/ab_variants/test_ab_overlap.py tests/ab_variants/test_ab_split_shapes.py -k "policies" > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 400 python -u tools/pipe_ab.py nt:COUP_WRITER_POL=0 plain:COUP_WRITER_POL=1 sc1:COUP_WRITER_POL=2 sc1nt:COUP_WRITER_POL=3 > $D/pipe_ab.jsonl 2> $D/pipe_ab.err || { tail -20 $D/pipe_ab.err; exit 1; }
cut -c1-120 $D/pipe_ab.jsonl
timeout -k 10 600 python -u tools/ab_step.py --batch 262144 --obs 0 --info 1 --rounds 5 nt:COUP_WRITER_POL=0 plain:COUP_WRITER_POL=1 sc1:COUP_WRITER_POL=2 sc1nt:COUP_WRITER_POL=3 > $D/c3i_ab.jsonl 2> $D/c3i_ab.err || { tail -20 $D/c3i_ab.err; exit 1; }
cut -c1-160 $D/c3i_ab.jsonl
