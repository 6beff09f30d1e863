# Round 5, VERDICT r4 item 1: which llc stage brings the uint2-prefix defect.
# The reproducer's own kernels three times (is the mismatch count the same
# run to run?), then k_sweep_uint2<512, 2> / k_sweep_rows<512, 2> from the
# device IR through llc -O0, -O3, GlobalISel, an s_nop before every
# instruction, every s_waitcnt forced to zero, and every opt-bisect limit
# over llc's 135 optional passes (tools/info_modules.sh); k_min<0>'s SLP IR
# of round 4 with the same two switches.
set -u
D=gpurun_out/r05o
mkdir -p $D
for i in 1 2 3; do
  timeout -k 10 120 build/info_prefix_repro 20000 > $D/repro_$i.jsonl 2>&1 || { cat $D/repro_$i.jsonl; exit 1; }
  grep uint2 $D/repro_$i.jsonl | cut -c1-140
done
timeout -k 10 600 build/info_prefix_repro 20000 build/infomod/O0.co build/infomod/O3.co build/infomod/O3gisel.co \
  build/infomod/O3snop4.co build/infomod/O3waitzero.co build/infomod/O0snop4.co > $D/modules_switches.jsonl 2>&1 || { tail -5 $D/modules_switches.jsonl; exit 1; }
cut -c1-150 $D/modules_switches.jsonl
timeout -k 10 300 build/w3phi/w3_module_check 20000 build/w3phi/kmin_none_O3.co build/w3phi/kmin_slp_O3snop4.co build/w3phi/kmin_slp_O3waitzero.co build/w3phi/kmin_all_O3.co > $D/kmin_switches.json 2>&1 || { tail -5 $D/kmin_switches.json; exit 1; }
python3 -c "
import json; d=json.load(open('$D/kmin_switches.json'))
for k,v in d['modules'].items(): print(k, v['mismatch'], v['by_word'])"
timeout -k 10 900 build/info_prefix_repro 20000 $(ls build/infomod/bisect_*.co) > $D/modules_bisect.jsonl 2>&1 || { tail -5 $D/modules_bisect.jsonl; exit 1; }
python3 -c "
import json
rows=[json.loads(l) for l in open('$D/modules_bisect.jsonl')]
print(' '.join('%s:%d' % (r['kernel'].split('bisect_')[1].replace('.co ',''), r['mismatching_lanes']) for r in rows))"
