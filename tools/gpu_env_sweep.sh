#!/bin/bash
# rates of the regular build under env settings: SWEEP="OWGS_CW=160 OWGS_DEAL=1 ..." (one setting per run)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sweep; mkdir -p $O
C=${CFGS:-c2 c4 headline:0/8}
for e in $SWEEP; do
  echo "== $e"
  env $e REPS=${REPS:-3} timeout -k 10 200 python -u tools/prof_phases.py $C > $O/rates_$e.log 2>&1 || exit 1
  grep -v amdgpu.ids $O/rates_$e.log | grep -v cycles/activation | cut -c1-100
done
