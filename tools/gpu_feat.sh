#!/bin/bash
# Engine specialisations (OWGS_F_*): the full -m gpu suite on the regular build, then per-config rates with the
# specialised engines (default) against the general engine for every launch (OWGS_FEAT_ALL=1, same binary), then the
# instruction-cache counters of both on configs[1].  Each step under its own limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/feat; O=gpurun_out/feat; export TMPDIR=/tmp
C=${CFGS:-headline c2 c4 headline:0/8}
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
REPS=3 timeout -k 10 300 python -u tools/prof_phases.py $C > $O/rates_spec.log 2>&1 || { tail $O/rates_spec.log; exit 1; }
grep -v amdgpu.ids $O/rates_spec.log | grep -v cycles/activation | cut -c1-150
OWGS_FEAT_ALL=1 REPS=3 timeout -k 10 300 python -u tools/prof_phases.py $C > $O/rates_all.log 2>&1 || { tail $O/rates_all.log; exit 1; }
echo "== general engine (OWGS_FEAT_ALL=1)"
grep -v amdgpu.ids $O/rates_all.log | grep -v cycles/activation | cut -c1-150
if [ -z "$SKIP_ICACHE" ]; then
  ARGS="--config c2" timeout -k 10 300 bash tools/gpu_icache.sh > $O/icache_c2_spec.txt 2>&1; cat $O/icache_c2_spec.txt | cut -c1-400
  OWGS_FEAT_ALL=1 ARGS="--config c2" timeout -k 10 300 bash tools/gpu_icache.sh > $O/icache_c2_all.txt 2>&1; cat $O/icache_c2_all.txt | cut -c1-400
fi
echo "gpu_feat done"
