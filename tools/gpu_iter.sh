#!/bin/bash
# Quick iteration on the GPU: parity subset, then per-phase timings (profile build) and variant timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/iter; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "${TESTK:-stream_parity or c5 or cluster_shard or multi_shard or shim}" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |Error" $O/pytest.log | head -20; exit $rc; }
OWGS_LIB=openwhisk_amd/libowgs_prof.so REPS=2 timeout -k 10 400 python tools/prof_phases.py ${PHASES:-headline c2 c4 headline:0/8} > $O/phases.log 2>&1
rc=$?; cut -c1-330 $O/phases.log; [ $rc -eq 0 ] || exit $rc
for so in $(ls openwhisk_amd/variants/*.so 2>/dev/null) openwhisk_amd/libowgs.so; do
  echo "== $so"; OWGS_LIB=$so REPS=3 timeout -k 10 300 python tools/prof_phases.py ${VPHASES:-headline headline:0/8} 2>&1 | grep -v amdgpu.ids | cut -c1-200 || exit 1
done
