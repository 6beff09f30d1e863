# Round 6: the split writers' store rate against the size of the buffer they
# fill (c3i's InformationStateTensor writer runs ~12% below
# c3's observation writer on the same store pattern).  If the 256 MB Infinity
# Cache absorbs the tail of each step's stores, a writer's rate falls with
# its buffer: c3i at 2^15 .. 2^18 lanes (0.65 .. 5.2 GB per step), c3 at 2^19 ..
# 2^21 lanes (0.41 .. 1.64 GB).  Driver-form lines, one process each.
set -u
. tools/gpu_calls/attempt.sh r06m
for b in 32768 65536 131072 262144; do
  timeout -k 10 200 python -u bench.py --config c3i --batch $b --steps 20 --warmup 5 --no-cpu-baseline > $D/c3i_$b.json 2> $D/c3i_$b.err || { tail -20 $D/c3i_$b.err; exit 1; }
done
for b in 524288 1048576 2097152; do
  timeout -k 10 200 python -u bench.py --config c3 --batch $b --steps 20 --warmup 5 --no-cpu-baseline > $D/c3_$b.json 2> $D/c3_$b.err || { tail -20 $D/c3_$b.err; exit 1; }
done
python3 - "$D" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/c3*.json")):
    d = json.load(open(f)); r = d["roofline"]
    print(f.split("/")[-1], round(d["ms_per_step"] * 1e3, 1), "us/step", "frac", round(r["frac"], 3),
          "GB/s", round(r["achieved"], 0))
PY
