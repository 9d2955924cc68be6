cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/specsweep; mkdir -p $O
for v in 16 8 32 64 16; do
  OWGS_RES_SPEC=$v timeout -k 10 200 python tools/shim_leg.py --drains 64,512 > $O/shim_$v.json 2> $O/shim_$v.err || { tail -5 $O/shim_$v.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/shim_$v.json'))
for l in d['legs']:
    if l['mode']=='fused' and l['drain']<=512:
        r=l['resident']; s=r['served']
        print('$v', l['drain'], l['p50_us'], round(l['decisions_per_s']/1e6,2), 'alone', round(r['decided_alone']/s,1), round(r['alone_cycles']/s), 'spec', round(r['speculation_cycles']/s), 'val', round(r['validation_cycles']/s), 'pub', round(r['publish_cycles']/s))
" | tee -a $O/sweep.txt
done
