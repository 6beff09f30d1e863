# Round 2, session 2: c3 step in blocks of 64 / 128 / 256 / 512 threads (COUP_OBS_MODE 10 / 11 / 9 / 12) --
# obs-writer parity, then same-process A/B with the store ceiling.
set -u
D=gpurun_out/r02s2n
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 150 --timeout-method thread -k obs_writers > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 400 python -u tools/ab_step.py --rounds 7 --steps 20 COUP_OBS_MODE=9 COUP_OBS_MODE=10 COUP_OBS_MODE=11 COUP_OBS_MODE=12 CEIL=1 > $D/ab_c3_block.jsonl 2>$D/ab.err || { tail $D/ab.err; exit 1; }
cat $D/ab_c3_block.jsonl
