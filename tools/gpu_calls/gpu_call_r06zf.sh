# Round 6, end of session: the final tree on the whole GPU suite, smoke(),
# the driver's default line; then the 6-player trajectory's regrouping block
# (COUP_NP_SORT_THREADS=512 / 256, measurement build) against the shipped
# 1024, and c3 with one 20-step rules launch of 16-byte records (320 MB).
set -u
. tools/gpu_calls/attempt.sh r06zf
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_default.json 2> $D/bench_default.err || { tail -20 $D/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_default.json')); r=d['roofline']; print('c3', d['value'], r['frac'], r['kernel_ms'], r['kernel'] == r['kernel_launched'])"
P=open_spiel_coup_amd/libcoup_mi355x.so
V=build/variants/libcoup_mi355x.so
timeout -k 10 500 python -u tools/bench_ab.py --rounds 3 $P $V:COUP_NP_SORT_THREADS=512 $V:COUP_NP_SORT_THREADS=256 -- --config c4 --steps 20 --warmup 5 > $D/ab_c4.jsonl 2> $D/ab_c4.err || { tail -20 $D/ab_c4.err; exit 1; }
grep median $D/ab_c4.jsonl
timeout -k 10 500 python -u tools/bench_ab.py --rounds 3 $P $P:COUP_TRAJ_CHUNK=20 -- --config c3 --steps 20 --warmup 5 > $D/ab_c3_chunk20.jsonl 2> $D/ab_c3_chunk20.err || { tail -20 $D/ab_c3_chunk20.err; exit 1; }
grep median $D/ab_c3_chunk20.jsonl
