#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel-trace.  Every GPU step has its own time limit and the
# script stops at the first step that faults, aborts, segfaults or times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() {  # $1 = rc, $2 = step
  case "$1" in
    0|1) return 0 ;;
    *) echo "STEP $2 ended with rc=$1 -- stopping"; exit "$1" ;;
  esac
}
STEPS="${STEPS:-tests smoke bench prof}"
for s in $STEPS; do
  case "$s" in
    tests)
      timeout -k 10 ${T_TESTS:-600} python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; tail -25 gpurun_out/pytest_gpu.log; stop_on_fault $rc tests ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; tail -5 gpurun_out/smoke.log; stop_on_fault $rc smoke ;;
    bench)
      timeout -k 10 ${T_BENCH:-600} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
      rc=$?; tail -5 gpurun_out/bench.log; stop_on_fault $rc bench ;;
    prof)
      rm -rf gpurun_out/prof
      timeout -k 10 ${T_PROF:-600} rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
        python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
      rc=$?; tail -3 gpurun_out/prof.log; find gpurun_out/prof -name "*stats*" | head; stop_on_fault $rc prof ;;
  esac
done
echo "gpu_check done"
