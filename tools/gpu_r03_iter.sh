#!/bin/bash
# round-3 iteration: full -m gpu suite and per-config rates of the regular build; then, for each VARIANTS name, the
# stream-parity tests and rates of openwhisk_amd/variants/libowgs_NAME.so; PROF=path: a profile build's phase cycles
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
C=${CFGS:-headline c2 c4 c5:0/8}
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 250 python -u tools/prof_phases.py $C > gpurun_out/rates.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/rates.log | grep -v cycles/activation | cut -c1-150
for v in $VARIANTS; do
  echo "== $v"
  OWGS_LIB=openwhisk_amd/variants/libowgs_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -k "stream_parity or full_size or shard" > gpurun_out/pytest_$v.log 2>&1
  rc=$?; tail -1 gpurun_out/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
  OWGS_LIB=openwhisk_amd/variants/libowgs_$v.so timeout -k 10 250 python -u tools/prof_phases.py $C > gpurun_out/rates_$v.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/rates_$v.log | grep -v cycles/activation | cut -c1-150
done
if [ -n "$PROF" ]; then
  OWGS_LIB=$PROF REPS=2 timeout -k 10 250 python -u tools/prof_phases.py $C > gpurun_out/prof.log 2>&1 || exit $?
fi
