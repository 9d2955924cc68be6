#!/bin/bash
# Same-box A/B of the shim leg: the in-tree library against openwhisk_amd/variants/libowgs_$AB_BASE.so, alternating
# (new, base, new, base), then the resident engine's tests on the in-tree library.  Outputs under gpurun_out/ab.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab; mkdir -p $O; export TMPDIR=/tmp
B=openwhisk_amd/variants/libowgs_${AB_BASE:-base}.so
for i in 1 2; do
  for lib in openwhisk_amd/libowgs.so $B; do
    n=$(basename $lib .so)_$i
    OWGS_LIB=$lib timeout -k 10 200 python tools/shim_leg.py --drains 64,512 > $O/shim_$n.json 2> $O/shim_$n.err || { tail -5 $O/shim_$n.err; exit 1; }
    python3 -c "
import json
d=json.load(open('$O/shim_$n.json'))
for l in d['legs']:
    if l['mode']=='fused' and l['drain']<=512:
        r=l['resident']; s=r['served']
        print('$n', l['drain'], l['p50_us'], round(l['decisions_per_s']/1e6,2), 'pub', round(r['publish_cycles']/s), 'conc', round(r['conc_walk_cycles']/s), 'alone', round(r['alone_cycles']/s))
" | tee -a $O/ab.txt
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_shim_sequence.py -x -v --timeout 200 --timeout-method thread > $O/pytest_res.log 2>&1
rc=$?; tail -2 $O/pytest_res.log; exit $rc
