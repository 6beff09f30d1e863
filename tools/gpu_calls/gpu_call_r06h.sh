# Round 6: the c3 writer's blocks per CU (COUP_WRITER_DYN_LDS caps them with
# dynamic LDS: 40 KB -> 4, 48 KB -> 3, 72 KB -> 2 per CU), same-process A/B in the
# driver's graph form (measurement build).
set -u
. tools/gpu_calls/attempt.sh r06h
export COUP_LIB_PATH=build/variants/libcoup_mi355x.so
timeout -k 10 400 python -u tools/pipe_ab.py --rounds 9 rows:COUP_PIPE=1 lds40k:COUP_WRITER_DYN_LDS=40960 \
  lds48k:COUP_WRITER_DYN_LDS=49152 lds72k:COUP_WRITER_DYN_LDS=73728 > $D/ab.jsonl 2> $D/ab.err || { tail -20 $D/ab.err; exit 1; }
python3 -c "
import json
for l in open('$D/ab.jsonl'):
    d=json.loads(l); print(d['variant'], d['median_us'], d['min_us'], d['frac_of_spec'])"
