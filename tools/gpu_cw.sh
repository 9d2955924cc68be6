#!/bin/bash
# chunk-width sweep (OWGS_CW) of the in-tree engine and the lane-geometry variants in openwhisk_amd/diag2/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for cw in ${CWS:-128 192 256 336}; do
  echo "== cw $cw"; OWGS_CW=$cw REPS=2 timeout -k 10 300 python tools/prof_phases.py ${PHASES:-c2 c4 headline:0/8 headline:0/4} 2>&1 | grep "ms (min" | cut -c1-120 || exit 1
done
for so in openwhisk_amd/diag2/*.so; do
  for cw in ${CWS2:-336 448}; do
    echo "== $so cw $cw"; OWGS_LIB=$so OWGS_CW=$cw REPS=2 timeout -k 10 300 python tools/prof_phases.py ${PHASES2:-headline} 2>&1 | grep "ms (min" | cut -c1-120 || exit 1
  done
done
