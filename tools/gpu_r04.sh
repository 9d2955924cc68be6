#!/bin/bash
# Round-4 GPU steps.  STEPS selects them (space separated); each step runs under its own time limit and the script
# stops at the first step that fails.  Outputs under gpurun_out/r04/$TAG.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04/${TAG:-a}; mkdir -p $O; export TMPDIR=/tmp
stop() { echo "STEP $1 rc=$2 -- stopping"; exit "$2"; }
for s in ${STEPS:-tests smoke}; do
  case "$s" in
    handoff)  # cross-CU hand-off latency
      timeout -k 10 60 ./tools/micro/handoff > $O/handoff.json 2>&1
      rc=$?; cat $O/handoff.json; [ $rc -eq 0 ] || stop handoff $rc ;;
    launchlat)  # fixed costs of a shim call: launches, copies, zero-copy, resident-kernel doorbell
      timeout -k 10 90 ./tools/micro/launch_lat > $O/launch_lat.json 2>&1
      rc=$?; cat $O/launch_lat.json; [ $rc -eq 0 ] || stop launchlat $rc ;;
    restests)  # the resident engine's tests alone (fast feedback)
      timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_shim_sequence.py -x -v --timeout 200 --timeout-method thread > $O/pytest_res.log 2>&1
      rc=$?; tail -3 $O/pytest_res.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error|assert" $O/pytest_res.log | head -30; stop restests $rc; } ;;
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
      rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; stop tests $rc; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
      rc=$?; tail -3 $O/smoke.log; [ $rc -eq 0 ] || stop smoke $rc ;;
    shim)  # the bench's shim-path leg (calls vs fused) at drains 64 / 512
      timeout -k 10 300 python tools/shim_leg.py --drains 64,512 > $O/shim.json 2> $O/shim.err
      rc=$?; cut -c1-1500 $O/shim.json; [ $rc -eq 0 ] || { tail -5 $O/shim.err; stop shim $rc; } ;;
    resrate)  # sequential resident engine vs the launch chain on whole streams in 1500-job drains (decisions/s)
      rm -f $O/resrate.jsonl
      for c in ${RES_CFGS:-headline c2 c4 headline:0/8}; do
        OWGS_RES_MAX=2048 timeout -k 10 300 python tools/shim_leg.py --config $c --drains 1500 --budget 150000 --modes fused >> $O/resrate.jsonl 2>> $O/resrate.err
        rc=$?; [ $rc -eq 0 ] || { tail -5 $O/resrate.err; stop resrate $rc; }
        OWGS_RESIDENT=0 timeout -k 10 300 python tools/shim_leg.py --config $c --drains 1500 --budget 150000 --modes fused >> $O/resrate.jsonl 2>> $O/resrate.err
        rc=$?; [ $rc -eq 0 ] || { tail -5 $O/resrate.err; stop resrate $rc; }
      done
      cut -c1-600 $O/resrate.jsonl ;;
    shimphases)  # per-call engine cycles at small drains (profile build)
      OWGS_LIB=openwhisk_amd/libowgs_prof.so CALLS=300 timeout -k 10 300 python tools/shim_phases.py 64,512 > $O/shimphases.jsonl 2> $O/shimphases.err
      rc=$?; cat $O/shimphases.jsonl; [ $rc -eq 0 ] || { tail -5 $O/shimphases.err; stop shimphases $rc; } ;;
    shimtrace)  # kernel trace of the shim path at drain 64 (launches per call)
      rm -rf $O/shimtrace
      CALLS=300 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/shimtrace -o run --output-format csv -- \
        python3 tools/shim_phases.py 64 > $O/shimtrace.log 2>&1
      rc=$?; tail -1 $O/shimtrace.log | cut -c1-300; [ $rc -eq 0 ] || stop shimtrace $rc ;;
    bench)
      timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
      rc=$?; cut -c1-400 $O/bench.json; [ $rc -eq 0 ] || { tail -20 $O/bench.err; stop bench $rc; } ;;
    dbgres)  # permits after every resident call, per config (tools/debug_resident.py)
      for c in ${DBG_CFGS:-headline c4 hot}; do
        timeout -k 10 200 python -u tools/debug_resident.py $c >> $O/dbgres.log 2>&1; rc=$?
        tail -12 $O/dbgres.log | cut -c1-400; [ $rc -eq 0 ] || [ $rc -eq 1 ] || stop dbgres $rc
      done ;;
    spectests)  # the parity suite (full-size streams included) with the replay path as the environment sets it
      timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_resident.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_parity.log 2>&1
      rc=$?; tail -2 $O/pytest_parity.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error|assert" $O/pytest_parity.log | head -30; stop spectests $rc; } ;;
    vtests)  # the resident engine's tests under each variant library in $V (openwhisk_amd/variants/libowgs_<v>.so)
      for v in $V; do
        OWGS_LIB=openwhisk_amd/variants/libowgs_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_shim_sequence.py -x -v --timeout 120 --timeout-method thread > $O/pytest_v_$v.log 2>&1
        rc=$?; echo "== $v"; tail -2 $O/pytest_v_$v.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error|assert" $O/pytest_v_$v.log | head -30; stop vtests $rc; }
      done ;;
    vshim)  # the shim leg under each variant library in $V
      for v in $V; do
        OWGS_LIB=openwhisk_amd/variants/libowgs_$v.so timeout -k 10 300 python tools/shim_leg.py --drains 64,512 > $O/shim_v_$v.json 2> $O/shim_v_$v.err
        rc=$?; echo "== $v"; cut -c1-1500 $O/shim_v_$v.json; [ $rc -eq 0 ] || { tail -5 $O/shim_v_$v.err; stop vshim $rc; }
      done ;;
    benchprof)  # kernel stats of the default bench command (profiles/r04_kernel_stats.csv)
      rm -rf $O/benchprof
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/benchprof -o run --output-format csv -- \
        python3 bench.py --no-shim-path > $O/benchprof.log 2>&1
      rc=$?; tail -1 $O/benchprof.log | cut -c1-300; [ $rc -eq 0 ] || stop benchprof $rc ;;
    phases)
      OWGS_LIB=openwhisk_amd/libowgs_prof.so REPS=2 timeout -k 10 400 python tools/prof_phases.py ${PHASE_CFGS:-headline c2 c4 headline:0/8} > $O/phases.log 2>&1
      rc=$?; cut -c1-200 $O/phases.log; [ $rc -eq 0 ] || stop phases $rc ;;
    cfgs)
      rm -f $O/cfgs.jsonl
      for c in "--config c2" "--config c3" "--config c4" "--cluster-size 8"; do
        timeout -k 10 400 python bench.py $c --steps 5 --warmup 1 --no-h2d --no-shim-path >> $O/cfgs.jsonl 2>> $O/cfgs.err
        rc=$?; tail -1 $O/cfgs.jsonl | cut -c1-160; [ $rc -eq 0 ] || { tail -20 $O/cfgs.err; stop "cfg $c" $rc; }
      done ;;
  esac
done
echo "gpu_r04 STEPS='${STEPS:-tests smoke}' done"
