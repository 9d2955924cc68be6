#!/bin/bash
# Variant check on the GPU: parity subset with each variant library ($VARS, names under openwhisk_amd/variants),
# then timings of $VPHASES for each variant and the default library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/var; mkdir -p $O; export TMPDIR=/tmp
for v in ${VARS}; do
  OWGS_LIB=openwhisk_amd/variants/libowgs_$v.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "${TESTK:-stream_parity or c5 or multi_shard}" > $O/pytest_$v.log 2>&1
  rc=$?; echo "== $v parity"; tail -2 $O/pytest_$v.log; [ $rc -eq 0 ] || { grep -E "^E " $O/pytest_$v.log | head -10; exit $rc; }
done
for v in ${VARS} ${BASE:-r01}; do
  so=openwhisk_amd/variants/libowgs_$v.so
  echo "== $v"; OWGS_LIB=$so REPS=3 timeout -k 10 300 python tools/prof_phases.py ${VPHASES:-headline headline:0/8} 2>&1 | grep -v amdgpu.ids | grep -v cycles/act | cut -c1-150 || exit 1
done
echo "== default"; REPS=3 timeout -k 10 300 python tools/prof_phases.py ${VPHASES:-headline headline:0/8} 2>&1 | grep -v amdgpu.ids | grep -v cycles/act | cut -c1-150
