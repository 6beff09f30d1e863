# Round 3: the section-12 code-generation hazard, bisected over the IR
# passes.  build/bisect.tar.gz holds tools/slot_bisect_build.sh's reproducers
# built with -mllvm -opt-bisect-limit=N at the IR-pass boundaries of the
# k_min<0> kernel (profiles/r03/codegen/k_min0_passes.txt; -1 = no limit).
# Each runs 20,000 cases; its k_slot-copy mismatch counts go to one line each.
set -u
D=gpurun_out/r03q
mkdir -p $D /tmp/bis
tar xzf build/bisect.tar.gz -C /tmp/bis
for n in -1 32640 29011 28814 27068 27051 24026 24017 24005 23987 23971 3258 2926 1429; do
  timeout -k 10 120 /tmp/bis/repro_$n 20000 > $D/bisect_$n.txt 2> $D/bisect_$n.err || { echo "limit $n failed rc=$?"; tail -5 $D/bisect_$n.err; exit 1; }
  echo "limit $n: $(head -c 300 $D/bisect_$n.txt | tr -d '\n')"
done
# the facade latency table after the one-call apply_action / child path and
# the slot op's joined record + history loads
timeout -k 10 400 python -u tools/facade_latency.py --rounds 5 > $D/facade_latency.json 2> $D/facade.err || { tail -20 $D/facade.err; exit 1; }
python -c "import json; d=json.load(open('$D/facade_latency.json')); [print(k, v) for k, v in d['rows_us'].items()]"
