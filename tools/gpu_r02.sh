#!/bin/bash
# Round-2 GPU session: steps chosen by $STEPS (default: tests bench cfgs phases), each under its own time limit; the
# script stops at the first step that faults, aborts, segfaults or times out.  Outputs under gpurun_out/r02/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02
mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STEP $1 rc=$2 -- stopping"; exit "$2"; }
for s in ${STEPS:-tests bench cfgs phases}; do
  case "$s" in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1
      rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -eq 0 ] || stop tests $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
      rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || stop smoke $rc ;;
    bench)
      timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err
      rc=$?; cut -c1-600 $O/bench.json; [ $rc -eq 0 ] || { tail -20 $O/bench.err; stop bench $rc; } ;;
    cfgs)  # one bench line per config (own cpu baseline): configs[1..3] and configs[4] shards at clusterSize 2, 4, 8
      for c in "--config c2" "--config c3" "--config c4" "--cluster-size 2" "--cluster-size 4" "--cluster-size 8"; do
        timeout -k 10 400 python bench.py $c --steps 5 --warmup 1 --no-h2d ${CFG_ARGS:-} >> $O/cfgs.jsonl 2>> $O/cfgs.err
        rc=$?; tail -1 $O/cfgs.jsonl | cut -c1-300; [ $rc -eq 0 ] || { tail -20 $O/cfgs.err; stop "cfg $c" $rc; }
      done ;;
    phases)
      OWGS_LIB=openwhisk_amd/libowgs_prof.so REPS=2 timeout -k 10 400 python tools/prof_phases.py ${PHASES:-headline c2 c4 headline:0/8} > $O/phases.log 2>&1
      rc=$?; cat $O/phases.log | cut -c1-400; [ $rc -eq 0 ] || stop phases $rc ;;
    prof)
      rm -rf $O/prof
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
        python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check --no-h2d ${BENCH_ARGS:-} > $O/prof.log 2>&1
      rc=$?; tail -2 $O/prof.log | cut -c1-300; [ $rc -eq 0 ] || stop prof $rc ;;
    pmc)
      timeout -k 10 600 python3 tools/pmc_traffic.py ${BENCH_ARGS:-} > $O/pmc.log 2>&1
      rc=$?; tail -2 $O/pmc.log | cut -c1-400; [ $rc -eq 0 ] || stop pmc $rc ;;
    pmccfg)  # HBM traffic entries for the per-config bench lines (configs[1..3])
      for c in c2 c3 c4; do
        timeout -k 10 600 python3 tools/pmc_traffic.py --config $c > $O/pmc_$c.log 2>&1
        rc=$?; tail -1 $O/pmc_$c.log | cut -c1-200; [ $rc -eq 0 ] || stop "pmc $c" $rc
      done ;;
  esac
done
echo "gpu_r02 done"
