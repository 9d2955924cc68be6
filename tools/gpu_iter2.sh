#!/bin/bash
# iteration: stream-parity tests of the regular build, its per-config rates, then optional barrier traces
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/it2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "stream_parity or full_size or shard or golden" > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=${REPS:-3} timeout -k 10 300 python -u tools/prof_phases.py ${CFGS:-headline c2 c3 c4 headline:0/8} > $O/rates.log 2>&1 || { tail $O/rates.log; exit 1; }
grep -v amdgpu.ids $O/rates.log | grep -v cycles/activation | cut -c1-150
if [ -n "$TRACE" ]; then TRACE_CFG="$TRACE" timeout -k 10 400 bash tools/gpu_trace.sh || exit 1; fi
echo "iter2 done"
