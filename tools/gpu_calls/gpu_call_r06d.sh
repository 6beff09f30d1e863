# Round 6: the nibble + table observation writer (COUP_WRITER_FORM, measurement
# build): equality with stepping, then the same-process A/B in the driver's graph
# form against the shipped rows writer.
set -u
. tools/gpu_calls/attempt.sh r06d
export COUP_LIB_PATH=build/variants/libcoup_mi355x.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/ab_variants/test_ab_overlap.py -k nibble > $D/nib_eq.log 2>&1 || { tail -30 $D/nib_eq.log; exit 1; }
tail -1 $D/nib_eq.log
timeout -k 10 400 python -u tools/pipe_ab.py --rounds 9 rows:COUP_PIPE=1 nib512x2:COUP_WRITER_FORM=1 \
  nib512x4:COUP_WRITER_FORM=2 nib1024x2:COUP_WRITER_FORM=3 nib256x4:COUP_WRITER_FORM=4 > $D/ab.jsonl 2> $D/ab.err || { tail -20 $D/ab.err; exit 1; }
python3 -c "
import json
for l in open('$D/ab.jsonl'):
    d=json.loads(l); print(d['variant'], d['median_us'], d['min_us'], d['frac_of_spec'])"
