#!/bin/bash
# Round-4 evidence for the shipped build.  $PART selects the call (each fits one gpurun limit):
#   A: full GPU suite, smoke, HBM traffic (pmc_traffic.json) for every bench key, SQ counters
#   B: bench line (default args), kernel trace of the bench, per-config lines, the shim-path leg and its kernel trace,
#      the resident engine's stream mode on every config
# Each step runs under its own time limit; the script stops at the first step that fails.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04f; mkdir -p $O; export TMPDIR=/tmp
stop() { echo "STEP $1 rc=$2 -- stopping"; exit "$2"; }
if [ "$PART" = A ]; then STEPS=${STEPS:-"tests smoke pmc sq"}; else STEPS=${STEPS:-"bench prof cfgs shim shimprof streammode"}; fi
for s in $STEPS; do
  case "$s" in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
      rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || stop tests $rc ;;
    ab)  # rates of the shipped build against $AB_BASE (a variant library of the previous build), same box
      for lib in openwhisk_amd/libowgs.so openwhisk_amd/variants/libowgs_${AB_BASE:-base}.so; do
        [ -f "$lib" ] || continue
        echo "-- $lib"
        OWGS_LIB=$lib REPS=3 timeout -k 10 300 python -u tools/prof_phases.py c2 c4 headline:0/8 headline > $O/ab.log 2>&1
        rc=$?; grep -v amdgpu.ids $O/ab.log | grep -v cycles/activation | cut -c1-100; [ $rc -eq 0 ] || stop ab $rc
        cp $O/ab.log "$O/ab_$(basename $lib .so).log"
      done ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
      rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || stop smoke $rc ;;
    pmc)
      for c in "" "--cluster-size 2" "--cluster-size 4" "--cluster-size 8" "--config c2" "--config c2_64k" "--config c3" "--config c4"; do
        f=$O/pmc_traffic$(echo $c | tr -d ' -').log
        timeout -k 10 400 python3 tools/pmc_traffic.py $c > $f 2>&1
        rc=$?; tail -1 $f | cut -c1-200; [ $rc -eq 0 ] || stop "pmc $c" $rc
      done
      cp pmc_traffic.json $O/pmc_traffic.json ;;
    sq)
      timeout -k 10 600 bash tools/pmc_run.sh --config headline > $O/sq.log 2>&1
      rc=$?; tail -3 $O/sq.log; [ $rc -eq 0 ] || stop sq $rc
      cp gpurun_out/pmc/summary.txt $O/sq_pmc.txt ;;
    bench)
      timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
      rc=$?; cut -c1-300 $O/bench.json; [ $rc -eq 0 ] || { tail -20 $O/bench.err; stop bench $rc; } ;;
    prof)
      rm -rf $O/prof
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
        python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check --no-h2d --no-shim-path > $O/prof.log 2>&1
      rc=$?; tail -1 $O/prof.log | cut -c1-200; [ $rc -eq 0 ] || stop prof $rc ;;
    cfgs)  # one bench line per config (own cpu baseline): configs[1..3] and configs[4] shards at clusterSize 2, 4, 8
      rm -f $O/cfgs.jsonl
      for c in "--config c2" "--config c2_64k" "--config c3" "--config c4" "--cluster-size 2" "--cluster-size 4" "--cluster-size 8"; do
        timeout -k 10 400 python bench.py $c --steps 5 --warmup 1 --no-h2d --no-shim-path >> $O/cfgs.jsonl 2>> $O/cfgs.err
        rc=$?; tail -1 $O/cfgs.jsonl | cut -c1-160; [ $rc -eq 0 ] || { tail -20 $O/cfgs.err; stop "cfg $c" $rc; }
      done ;;
    churn)  # configs[4] cadence on one GPU: health all-gathered and applied before every batch
      rm -f $O/churn.jsonl
      for c in "" "--cluster-size 8"; do
        timeout -k 10 400 python bench.py --health-churn $c --steps 3 --warmup 1 --no-shim-path --no-cpu-baseline >> $O/churn.jsonl 2>> $O/churn.err
        rc=$?; tail -1 $O/churn.jsonl | cut -c1-160; [ $rc -eq 0 ] || { tail -20 $O/churn.err; stop "churn $c" $rc; }
      done ;;
    shim)  # the bench's shim-path leg alone at drains 64 and 512 (resident engine counters, host timing)
      timeout -k 10 300 python tools/shim_leg.py --drains 64,512 > $O/shim.json 2> $O/shim.err
      rc=$?; cut -c1-300 $O/shim.json; [ $rc -eq 0 ] || { tail -5 $O/shim.err; stop shim $rc; } ;;
    streammode)  # the resident engine's stream mode on every config (OWGS_SPEC_REPLAY=1), same box as cfgs
      rm -f $O/stream_cfgs.jsonl
      for c in "--config c2" "--config c3" "--config c4" "--cluster-size 8" ""; do
        OWGS_SPEC_REPLAY=1 timeout -k 10 400 python bench.py $c --steps 3 --warmup 1 --no-h2d --no-shim-path --no-cpu-baseline >> $O/stream_cfgs.jsonl 2>> $O/stream_cfgs.err
        rc=$?; tail -1 $O/stream_cfgs.jsonl | cut -c1-160; [ $rc -eq 0 ] || { tail -20 $O/stream_cfgs.err; stop "stream $c" $rc; }
      done ;;
    shimprof)  # kernel trace of the shim path (owgs_process_batch at drain 512)
      rm -rf $O/shimprof
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/shimprof -o run --output-format csv -- \
        python3 tools/shim_leg.py --drains 512 > $O/shimprof.log 2>&1
      rc=$?; tail -1 $O/shimprof.log | cut -c1-200; [ $rc -eq 0 ] || stop shimprof $rc ;;
    phases)
      OWGS_LIB=openwhisk_amd/libowgs_prof.so REPS=2 timeout -k 10 400 python tools/prof_phases.py headline c2 c4 headline:0/8 > $O/phases.log 2>&1
      rc=$?; cut -c1-160 $O/phases.log; [ $rc -eq 0 ] || stop phases $rc ;;
  esac
done
echo "gpu_final_r04 PART=$PART done"
