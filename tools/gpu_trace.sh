#!/bin/bash
# Barrier timelines of -DOWGS_TRACE engines (variants/libowgs_${TRACE_VARIANTS:-trace}.so) on $TRACE_CFG, analysed by
# trace_timeline.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/trace; mkdir -p $O; export TMPDIR=/tmp
for v in ${TRACE_VARIANTS:-trace}; do
for c in ${TRACE_CFG:-headline}; do
  f=$O/${v}_${c//[:\/]/_}
  OWGS_LIB=openwhisk_amd/variants/libowgs_$v.so OWGS_TRACE_FILE=$f.bin REPS=1 timeout -k 10 300 python tools/prof_phases.py $c > $O/run.log 2>&1 || { tail $O/run.log; exit 1; }
  echo "== $v $c"; grep -v amdgpu $O/run.log | head -1 | sed 's/.*{/{/'; python tools/trace_timeline.py $f.bin | tee $f.txt
  rm -f $f.bin
done
done
