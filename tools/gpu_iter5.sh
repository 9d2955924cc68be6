#!/bin/bash
# iteration: rates of the regular build; VARIANTS: parity subset + rates; RATEONLY: rates only (wide-geometry configs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/it5; mkdir -p $O; export TMPDIR=/tmp
C=${CFGS:-headline c2 c4 headline:0/8}
REPS=${REPS:-3} timeout -k 10 300 python -u tools/prof_phases.py $C > $O/rates.log 2>&1 || { tail $O/rates.log; exit 1; }
grep -v amdgpu.ids $O/rates.log | grep -v cycles/activation | cut -c1-110
for v in $VARIANTS; do
  echo "== $v"
  OWGS_LIB=openwhisk_amd/variants/libowgs_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -k "stream_parity or full_size or shard or specialisation" > $O/pytest_$v.log 2>&1
  rc=$?; tail -1 $O/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
  OWGS_LIB=openwhisk_amd/variants/libowgs_$v.so REPS=${REPS:-3} timeout -k 10 300 python -u tools/prof_phases.py $C > $O/rates_$v.log 2>&1 || exit 1
  grep -v amdgpu.ids $O/rates_$v.log | grep -v cycles/activation | cut -c1-110
done
for v in $RATEONLY; do
  echo "== $v (rates only)"
  OWGS_LIB=openwhisk_amd/variants/libowgs_$v.so REPS=${REPS:-3} timeout -k 10 200 python -u tools/prof_phases.py $C > $O/rates_$v.log 2>&1 || exit 1
  grep -v amdgpu.ids $O/rates_$v.log | grep -v cycles/activation | cut -c1-110
done
if [ -n "$PCFGS" ]; then
  OWGS_LIB=openwhisk_amd/libowgs_prof.so REPS=2 timeout -k 10 300 python -u tools/prof_phases.py $PCFGS > $O/phases.log 2>&1 || exit 1
  cut -c1-2000 $O/phases.log | grep -v amdgpu.ids
fi
echo "iter5 done"
