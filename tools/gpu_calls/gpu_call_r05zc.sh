# Round 5, the uint2-prefix fault: does it need several blocks per CU?  The
# failing code objects (llc -O3, opt-bisect limit 96) launched with 0, 32 KB,
# 80 KB and 150 KB of extra dynamic LDS per block (8+, ~4, ~2, 1 block per
# CU), three times each.
set -u
D=gpurun_out/r05zc
mkdir -p $D
for dyn in 0 32768 81920 153600; do
  for i in 1 2 3; do
    INFO_REPRO_DYN_LDS=$dyn timeout -k 10 300 build/info_prefix_repro 20000 build/infomod/O3.co build/infomod/bisect_096.co > $D/dyn${dyn}_$i.jsonl 2>&1 || { tail -5 $D/dyn${dyn}_$i.jsonl; exit 1; }
  done
  python3 -c "
import json,glob
rows=[json.loads(l) for f in sorted(glob.glob('$D/dyn${dyn}_*.jsonl')) for l in open(f)]
print('dyn $dyn', ' '.join('%s:%d' % (r['kernel'].split('/')[-1], r['mismatching_lanes']) for r in rows))"
done
