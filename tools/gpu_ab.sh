#!/bin/bash
# A/B on one box: a parity subset ($TESTK) with the in-tree engine, then replay timings (tools/prof_phases.py) of
# openwhisk_amd/variants/libowgs_*.so and the in-tree libowgs.so on the same workloads ($PHASES).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab; mkdir -p $O; export TMPDIR=/tmp
if [ -n "${TESTK}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTK}" > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |Error|mismatch" $O/pytest.log | head -20; exit $rc; }
fi
for so in $(ls openwhisk_amd/variants/*.so 2>/dev/null) openwhisk_amd/libowgs.so; do
  echo "== $so"
  OWGS_LIB=$so REPS=${REPS:-3} timeout -k 10 400 python tools/prof_phases.py ${PHASES:-headline c2 c3 c4 headline:0/8} > $O/t.log 2>&1
  rc=$?; grep -v amdgpu.ids $O/t.log | cut -c1-260; [ $rc -eq 0 ] || exit $rc
done
