#!/bin/bash
# Round-4 A/B: rates of the regular build, then of VARIANTS (openwhisk_amd/variants/libowgs_<v>.so), parity subset
# first for each variant; outputs under gpurun_out/r04/$TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04/${TAG:-ab}; mkdir -p $O; export TMPDIR=/tmp
C=${CFGS:-headline c2 c4 headline:0/8}
K="stream_parity or full_size or shard or golden or release or large_pool or span"
REPS=${REPS:-3} timeout -k 10 300 python -u tools/prof_phases.py $C > $O/rates.log 2>&1 || { tail $O/rates.log; exit 1; }
grep -v amdgpu.ids $O/rates.log | grep -v cycles/activation | cut -c1-110
for v in $VARIANTS; do
  echo "== $v"
  OWGS_LIB=openwhisk_amd/variants/libowgs_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -k "$K" > $O/pytest_$v.log 2>&1
  rc=$?; tail -1 $O/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
  OWGS_LIB=openwhisk_amd/variants/libowgs_$v.so REPS=${REPS:-3} timeout -k 10 300 python -u tools/prof_phases.py $C > $O/rates_$v.log 2>&1 || exit 1
  grep -v amdgpu.ids $O/rates_$v.log | grep -v cycles/activation | cut -c1-110
done
echo "gpu_r04b done"
