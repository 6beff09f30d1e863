# Round 3: the section-12 hazard, second bisect round: one reproducer per
# optional IR pass between the last passing and the first failing limit of
# round 1 (k_min<0>: 29507..29522 in profiles/r03/codegen/k_min0_passes.txt).
set -u
D=gpurun_out/r03r
mkdir -p $D /tmp/bis
tar xzf build/bisect.tar.gz -C /tmp/bis
for n in ${BISECT_LIMITS:-$(seq 29507 29522)}; do
  timeout -k 10 120 /tmp/bis/repro_$n 20000 > $D/bisect_$n.txt 2> $D/bisect_$n.err || { echo "limit $n failed rc=$?"; tail -5 $D/bisect_$n.err; exit 1; }
  echo "limit $n: $(grep -o '"min0_load_apply_store":{"mismatch":[0-9]*' $D/bisect_$n.txt)"
done
