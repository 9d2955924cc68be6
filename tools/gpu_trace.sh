#!/bin/bash
# Barrier timeline of a -DOWGS_TRACE engine (variants/libowgs_trace.so) on $TRACE_CFG, analysed by trace_timeline.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/trace; mkdir -p $O; export TMPDIR=/tmp
for c in ${TRACE_CFG:-headline}; do
  OWGS_LIB=openwhisk_amd/variants/libowgs_trace.so OWGS_TRACE_FILE=$O/${c//[:\/]/_}.bin REPS=1 timeout -k 10 300 python tools/prof_phases.py $c > $O/run.log 2>&1 || { tail $O/run.log; exit 1; }
  echo "== $c"; python tools/trace_timeline.py $O/${c//[:\/]/_}.bin | tee $O/${c//[:\/]/_}.txt
  rm -f $O/${c//[:\/]/_}.bin
done
