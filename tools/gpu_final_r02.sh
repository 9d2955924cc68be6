#!/bin/bash
# Round-2 evidence session, part 1 (the build that ships): full GPU suite, smoke, HBM traffic per bench workload
# (pmc_traffic.json for N = 1, 2, 4, 8 split shards), SQ counters, per-phase cycles.  Part 2 (bench lines, kernel
# trace) runs after pmc_traffic.json is in the tree: tools/gpu_r02.sh STEPS="bench prof cfgs".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final; mkdir -p $O; export TMPDIR=/tmp
stop() { echo "STEP $1 rc=$2 -- stopping"; exit "$2"; }
for s in ${STEPS:-tests smoke pmc sq phases}; do
  case "$s" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
      rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || stop tests $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
      rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || stop smoke $rc ;;
    pmc)
      for c in "" "--cluster-size 2" "--cluster-size 4" "--cluster-size 8"; do
        timeout -k 10 600 python3 tools/pmc_traffic.py $c > $O/pmc_traffic$(echo $c | tr -d ' -').log 2>&1
        rc=$?; cut -c1-300 $O/pmc_traffic$(echo $c | tr -d ' -').log; [ $rc -eq 0 ] || stop "pmc $c" $rc
      done ;;
    sq)
      timeout -k 10 900 bash tools/pmc_run.sh --config headline > $O/sq.log 2>&1
      rc=$?; tail -4 $O/sq.log; [ $rc -eq 0 ] || stop sq $rc ;;
    phases)
      OWGS_LIB=openwhisk_amd/libowgs_prof.so REPS=2 timeout -k 10 600 python tools/prof_phases.py headline c2 c3 c4 headline:0/2 headline:0/4 headline:0/8 > $O/phases.log 2>&1
      rc=$?; cut -c1-200 $O/phases.log; [ $rc -eq 0 ] || stop phases $rc ;;
  esac
done
echo "gpu_final_r02 done"
