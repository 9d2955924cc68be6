#!/bin/bash
# Round-6 GPU steps, selected by $STEPS (space separated); outputs under gpurun_out/r06/$TAG.  Each step runs under its
# own time limit and the script stops at the first step that fails (no GPU step after a failure).
#   tests      full GPU suite                       restests  the resident / shim suites only
#   smoke      __graft_entry__.smoke()              bench     bench line (default args)
#   prof       kernel trace of the bench            cfgs      one bench line per config
#   pmc        HBM traffic per bench key            sq        SQ counters of the headline engine
#   shim       the shim leg (drains 64, 512, 4096)  abshim    same-box A/B of the shim leg vs variants/libowgs_$AB_BASE.so
#   abcfg      same-box A/B of per-config engine rates vs variants/libowgs_$AB_BASE.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06/${TAG:-a}; mkdir -p $O; export TMPDIR=/tmp
stop() { echo "STEP $1 rc=$2 -- stopping"; exit "$2"; }
for s in ${STEPS:-tests}; do
  case "$s" in
    tests)
      timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
      rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -20; stop tests $rc; } ;;
    restests)
      timeout -k 10 500 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_shim_sequence.py -x -v --timeout 200 --timeout-method thread > $O/pytest_res.log 2>&1
      rc=$?; tail -2 $O/pytest_res.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_res.log | head -20; stop restests $rc; } ;;
    sel)  # the tests named by $TESTSEL
      timeout -k 10 600 python -u -m pytest $TESTSEL ${KSEL:+-k "$KSEL"} -x -v --timeout 200 --timeout-method thread > $O/pytest_sel.log 2>&1
      rc=$?; tail -2 $O/pytest_sel.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_sel.log | head -20; stop sel $rc; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
      rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || stop smoke $rc ;;
    bench)
      timeout -k 10 400 python bench.py ${BENCHARGS} > $O/bench.json 2> $O/bench.err
      rc=$?; cut -c1-400 $O/bench.json; [ $rc -eq 0 ] || { tail -20 $O/bench.err; stop bench $rc; } ;;
    prof)
      rm -rf $O/prof
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
        python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check --no-h2d --no-shim-path > $O/prof.log 2>&1
      rc=$?; tail -1 $O/prof.log | cut -c1-200; [ $rc -eq 0 ] || stop prof $rc ;;
    cfgs)
      rm -f $O/cfgs.jsonl
      for c in "--config c2" "--config c2_64k" "--config c3" "--config c4" "--cluster-size 2" "--cluster-size 4" "--cluster-size 8"; do
        timeout -k 10 400 python bench.py $c --steps 5 --warmup 1 --no-h2d --no-shim-path >> $O/cfgs.jsonl 2>> $O/cfgs.err
        rc=$?; tail -1 $O/cfgs.jsonl | cut -c1-160; [ $rc -eq 0 ] || { tail -20 $O/cfgs.err; stop "cfg $c" $rc; }
      done ;;
    pmc)
      IFS=',' read -ra CF <<< "${PMCCFGS:-,--cluster-size 8,--config c2,--config c4}"  # (comma-separated; empty = headline)
      for c in "${CF[@]}"; do
        f=$O/pmc_traffic$(echo $c | tr -d ' -').log
        timeout -k 10 400 python3 tools/pmc_traffic.py ${c} > $f 2>&1
        rc=$?; tail -1 $f | cut -c1-200; [ $rc -eq 0 ] || stop "pmc $c" $rc
      done
      cp pmc_traffic.json $O/pmc_traffic.json ;;
    sq)
      timeout -k 10 600 bash tools/pmc_run.sh --config headline > $O/sq.log 2>&1
      rc=$?; tail -3 $O/sq.log; [ $rc -eq 0 ] || stop sq $rc
      cp gpurun_out/pmc/summary.txt $O/sq_pmc.txt ;;
    shim)
      timeout -k 10 300 python tools/shim_leg.py --drains ${DRAINS:-64,512,4096} > $O/shim.json 2> $O/shim.err
      rc=$?; cut -c1-300 $O/shim.json; [ $rc -eq 0 ] || { tail -5 $O/shim.err; stop shim $rc; } ;;
    abshim)  # alternating runs on one box: in-tree library, then the base variant, twice
      B=openwhisk_amd/variants/libowgs_${AB_BASE:-r04}.so
      for i in 1 2; do
        for lib in openwhisk_amd/libowgs.so $B; do
          n=$(basename $lib .so)_$i
          OWGS_LIB=$lib timeout -k 10 200 python tools/shim_leg.py --drains ${DRAINS:-64,512} --modes fused > $O/shim_$n.json 2> $O/shim_$n.err || { tail -5 $O/shim_$n.err; stop abshim 1; }
          python3 -c "
import json
d=json.load(open('$O/shim_$n.json'))
for l in d['legs']:
    r=l.get('resident') or {}; s=max(1, r.get('served', 0))
    if l['mode'] == 'fused-reset':
        print('$n', l['mode'], 'resident', l['resident_fraction_after'], 'p50 before/after', round(l['p50_us_before'],1), round(l['p50_us_after'],1), 'p99', round(l['p99_us_after'],1), 'exact', l['bit_exact']); continue
    print('$n', l['mode'], l['drain'], 'p50', round(l['p50_us'],1), 'p99', round(l.get('p99_us'),1), round(l['decisions_per_s']/1e6,2), 'M/s pub', round(r.get('publish_cycles',0)/s), 'alone', round(r.get('alone_cycles',0)/s), 'launches', r.get('launches'), 'chained', r.get('chained'))
" | tee -a $O/abshim.txt
        done
      done ;;
    abenv)  # alternating runs of the shim leg with $ABENV set to 1 and to 0 (same library)
      for i in 1 2; do
        for v in ${ABVALS:-1 0}; do
          n=${ABENV}_${v}_$i
          env ${ABFIX} ${ABENV}=$v timeout -k 10 200 python tools/shim_leg.py --drains ${DRAINS:-64,512} --modes fused > $O/shim_$n.json 2> $O/shim_$n.err || { tail -5 $O/shim_$n.err; stop abenv 1; }
          python3 -c "
import json
d=json.load(open('$O/shim_$n.json'))
for l in d['legs']:
    r=l.get('resident') or {}; s=max(1, r.get('served', 0))
    if l['mode'] == 'fused-reset':
        print('$n', l['mode'], 'resident', l['resident_fraction_after'], 'p50 before/after', round(l['p50_us_before'],1), round(l['p50_us_after'],1), 'exact', l['bit_exact']); continue
    x = ''
    if l['mode'] == 'fused-mixed':
        x = 'after_chain %.1f steady %.1f gt1024 %.1f' % (l['p50_us_le1024_after_chain'], l['p50_us_le1024_steady'], l['p50_us_gt1024'])
    print('$n', l['mode'], l['drain'], 'p50', round(l['p50_us'],1), 'p99', round(l.get('p99_us'),1), round(l['decisions_per_s']/1e6,2), 'M/s pub', round(r.get('publish_cycles',0)/s), 'alone', round(r.get('alone_cycles',0)/s), 'exact', l['bit_exact'], x)
" | tee -a $O/abenv.txt
        done
      done ;;
    abcfg)  # engine rates per config, in-tree library vs the base variant, alternating
      B=openwhisk_amd/variants/libowgs_${AB_BASE:-r04}.so
      for i in 1 2; do
        for lib in openwhisk_amd/libowgs.so $B; do
          echo "-- $lib" >> $O/abcfg.txt
          OWGS_LIB=$lib REPS=3 timeout -k 10 300 python -u tools/prof_phases.py ${ABCFGS:-c2 c4 headline:0/8 headline} > $O/abcfg_$i.log 2>&1
          rc=$?; grep -v amdgpu.ids $O/abcfg_$i.log | grep -v cycles/activation | cut -c1-120 | tee -a $O/abcfg.txt; [ $rc -eq 0 ] || stop abcfg $rc
        done
      done ;;
    churn)  # configs[4] cadence on one GPU (health exchanged and applied before every batch) vs one launch per step
      rm -f $O/churn.jsonl
      for c in "" "--cluster-size 8"; do
        for h in "" "--health-churn" "--health-churn --health-group 1"; do
          timeout -k 10 400 python bench.py $h $c --steps 5 --warmup 1 --no-shim-path --no-cpu-baseline --no-h2d >> $O/churn.jsonl 2>> $O/churn.err
          rc=$?; tail -1 $O/churn.jsonl | cut -c1-200; [ $rc -eq 0 ] || { tail -20 $O/churn.err; stop "churn $h $c" $rc; }
        done
      done ;;
    churnprof)  # kernel trace of the per-batch cadence (gaps between a span's launches)
      rm -rf $O/churnprof
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/churnprof -o run --output-format csv -- \
        python3 bench.py --health-churn ${CHURNARGS} --steps 3 --warmup 1 --no-cpu-baseline --no-check --no-h2d --no-shim-path > $O/churnprof.log 2>&1
      rc=$?; tail -1 $O/churnprof.log | cut -c1-200; [ $rc -eq 0 ] || stop churnprof $rc ;;
    spanhost)  # host microseconds per call of the per-batch cadence (calls that wait for the GPU)
      for n in 1 8; do
        timeout -k 10 300 python tools/span_host_timing.py $n >> $O/spanhost.jsonl 2>> $O/spanhost.err
        rc=$?; tail -1 $O/spanhost.jsonl | cut -c1-600; [ $rc -eq 0 ] || { tail -5 $O/spanhost.err; stop spanhost $rc; }
      done ;;
    p99)  # per-call counters of the 512-job shim leg: the slowest 1 % against the median
      timeout -k 10 300 python tools/shim_p99.py > $O/p99.json 2> $O/p99.err
      rc=$?; cut -c1-600 $O/p99.json; [ $rc -eq 0 ] || { tail -5 $O/p99.err; stop p99 $rc; } ;;
    large)  # large-state engine rate (pools beyond the on-chip image) against the one-core oracle
      timeout -k 10 400 python -u tools/time_large.py ${LARGEN:-40000 25000} > $O/large.jsonl 2> $O/large.err
      rc=$?; cut -c1-400 $O/large.jsonl; [ $rc -eq 0 ] || { tail -5 $O/large.err; stop large $rc; } ;;
    rccl)  # the per-batch cadence with the health all-gather through a one-rank RCCL group (--rccl) against the local
           # copy, alternating, headline and the configs[4] shard of 8
      for i in 1 2; do
        for c in "" "--cluster-size 8"; do
          for x in "--rccl" ""; do
            timeout -k 10 400 python bench.py --health-churn $x $c --steps 5 --warmup 1 --no-shim-path --no-cpu-baseline --no-h2d >> $O/rccl.jsonl 2>> $O/rccl.err
            rc=$?; tail -1 $O/rccl.jsonl | cut -c1-200; [ $rc -eq 0 ] || { tail -20 $O/rccl.err; stop "rccl $x $c" $rc; }
          done
        done
      done ;;
    rcclprof)  # kernel trace of the RCCL cadence: do the all-gather kernels overlap the group's engine launch?
      rm -rf $O/rcclprof
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rcclprof -o run --output-format csv -- \
        python3 bench.py --health-churn --rccl ${CHURNARGS} --steps 3 --warmup 1 --no-cpu-baseline --no-check --no-h2d --no-shim-path > $O/rcclprof.log 2>&1
      rc=$?; tail -1 $O/rcclprof.log | cut -c1-200; [ $rc -eq 0 ] || stop rcclprof $rc ;;
    capparity)  # the parity file with the memory-class engines forced on wherever the classes fit (OWGS_CAPC=1)
      OWGS_CAPC=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread > $O/pytest_cap.log 2>&1
      rc=$?; tail -2 $O/pytest_cap.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_cap.log | head -20; stop capparity $rc; } ;;
    capab)  # engine rates per config with the memory-class counts off / on (OWGS_CAPC), alternating, same library
      for i in 1 2; do
        for v in ${CAPVALS:-0 1}; do
          echo "-- OWGS_CAPC=$v run $i" >> $O/capab.txt
          OWGS_CAPC=$v REPS=3 timeout -k 10 400 python -u tools/prof_phases.py ${ABCFGS:-c3 headline:0/8 headline:0/4 headline:0/2 headline c2 c4} > $O/capab_${v}_$i.log 2>&1
          rc=$?; grep -v amdgpu.ids $O/capab_${v}_$i.log | grep -v cycles/activation | cut -c1-150 | tee -a $O/capab.txt; [ $rc -eq 0 ] || stop capab $rc
        done
      done ;;
    shimtrace)  # kernel + copy trace of the shim leg's fused calls at one drain size (where a chained call's time goes)
      rm -rf $O/shimtrace
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/shimtrace -o run --output-format csv -- \
        python3 tools/shim_leg.py --drains ${DRAINS:-4096} --modes fused > $O/shimtrace.json 2> $O/shimtrace.err
      rc=$?; cut -c1-300 $O/shimtrace.json; [ $rc -eq 0 ] || { tail -5 $O/shimtrace.err; stop shimtrace $rc; } ;;
    largeall)  # the large-state engine's rate at 40,000 invokers with 0 / 20 / 50 % concurrent actions, and 25,000
      for cc in 0 0.2 0.5; do
        CONC=$cc timeout -k 10 400 python -u tools/time_large.py 40000 >> $O/large.jsonl 2>> $O/large.err
        rc=$?; tail -1 $O/large.jsonl | cut -c1-300; [ $rc -eq 0 ] || { tail -5 $O/large.err; stop largeall $rc; }
      done
      timeout -k 10 400 python -u tools/time_large.py 25000 >> $O/large.jsonl 2>> $O/large.err
      rc=$?; tail -1 $O/large.jsonl | cut -c1-300; [ $rc -eq 0 ] || { tail -5 $O/large.err; stop largeall $rc; } ;;
    rcclq8)  # the same trace with 8 hardware queues per process (GPU_MAX_HW_QUEUES, the box's default is 4): does the
             # collective then overlap the engine instead of queueing behind it?
      rm -rf $O/rcclq8
      GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rcclq8 -o run --output-format csv -- \
        python3 bench.py --health-churn --rccl ${CHURNARGS} --steps 3 --warmup 1 --no-cpu-baseline --no-check --no-h2d --no-shim-path > $O/rcclq8.log 2>&1
      rc=$?; tail -1 $O/rcclq8.log | cut -c1-200; [ $rc -eq 0 ] || stop rcclq8 $rc ;;
    rcclline)  # with --rccl the bench's stdout must still be its one JSON line (RCCL's banner goes to stderr)
      timeout -k 10 300 python bench.py --health-churn --rccl --steps 2 --warmup 1 --no-cpu-baseline --no-shim-path --no-h2d > $O/rcclline.out 2> $O/rcclline.err
      rc=$?; [ $rc -eq 0 ] || { tail -5 $O/rcclline.err; stop rcclline $rc; }
      python3 -c "
import json,sys
lines=open('$O/rcclline.out').read().splitlines()
assert len(lines)==1, lines[:3]
d=json.loads(lines[0]); print('one JSON line:', d['config']['health_exchange'], round(d['value']/1e6,2), 'M/s exact', d['bit_exact'])" || stop rcclline 1 ;;
    diag)  # per-phase cycles (profile build), re-decision costs (-DOWGS_EXT_PROF) and stop reasons of the engine
      OWGS_LIB=openwhisk_amd/libowgs_prof.so REPS=2 timeout -k 10 300 python -u tools/prof_phases.py ${DIAGCFGS:-headline c2 c4 headline:0/8} > $O/phases.out 2>&1
      rc=$?; tail -2 $O/phases.out | cut -c1-300; [ $rc -eq 0 ] || stop diag-phases $rc
      OWGS_LIB=openwhisk_amd/variants/libowgs_extprof.so REPS=1 timeout -k 10 300 python -u tools/prof_phases.py ${DIAGCFGS:-headline c2 c4 headline:0/8} > $O/extprof.out 2>&1
      rc=$?; tail -1 $O/extprof.out | cut -c1-300; [ $rc -eq 0 ] || stop diag-extprof $rc
      OWGS_LIB=openwhisk_amd/variants/libowgs_why.so timeout -k 10 300 python -u tools/stop_reasons.py ${DIAGCFGS:-headline c2 c4 headline:0/8} > $O/why.out 2>&1
      rc=$?; tail -1 $O/why.out | cut -c1-300; [ $rc -eq 0 ] || stop diag-why $rc ;;
    resbd)  # the resident engine's per-call counters at drains 64 / 512 (in-tree library, then $AB_BASE if given)
      for lib in openwhisk_amd/libowgs.so ${AB_BASE:+openwhisk_amd/variants/libowgs_${AB_BASE}.so}; do
        n=$(basename $lib .so)
        OWGS_LIB=$lib timeout -k 10 300 python -u tools/res_breakdown.py ${DRAINS:-64,512} > $O/resbd_$n.json 2> $O/resbd_$n.err
        rc=$?; cut -c1-300 $O/resbd_$n.json; [ $rc -eq 0 ] || { tail -5 $O/resbd_$n.err; stop resbd $rc; }
      done ;;
    chainphases)  # per-phase engine cycles of the chained calls (profile build) at drain $DRAINS (default 4096)
      OWGS_LIB=openwhisk_amd/libowgs_prof.so CALLS=${CALLS:-120} timeout -k 10 300 python -u tools/shim_phases.py ${DRAINS:-4096} > $O/chainphases.json 2> $O/chainphases.err
      rc=$?; cut -c1-600 $O/chainphases.json; [ $rc -eq 0 ] || { tail -5 $O/chainphases.err; stop chainphases $rc; } ;;
    cwsweep)  # chunk width sweep (OWGS_CW) of one config's engine rate, each width twice, alternating
      for i in 1 2; do
        for w in ${CWS:-128 160 192 224 256}; do
          OWGS_CW=$w REPS=3 timeout -k 10 300 python -u tools/prof_phases.py ${CWCFG:-c2} > $O/cw_${w}_$i.log 2>&1
          rc=$?; echo "cw $w: $(grep -v amdgpu.ids $O/cw_${w}_$i.log | grep -v cycles/activation | cut -c1-110)" | tee -a $O/cwsweep.txt; [ $rc -eq 0 ] || stop cwsweep $rc
        done
      done ;;
    ablarge)  # the large-state engine's 25,000-invoker (release-heavy) rate, in-tree library vs the base variant, alternating
      B=openwhisk_amd/variants/libowgs_${AB_BASE:-r04}.so
      for i in 1 2; do
        for lib in openwhisk_amd/libowgs.so $B; do
          OWGS_LIB=$lib timeout -k 10 400 python -u tools/time_large.py ${LARGEN:-25000} > $O/ablarge_$(basename $lib .so)_$i.jsonl 2>> $O/ablarge.err
          rc=$?; echo "$(basename $lib .so) $i $(cut -c1-260 $O/ablarge_$(basename $lib .so)_$i.jsonl)" | tee -a $O/ablarge.txt; [ $rc -eq 0 ] || { tail -5 $O/ablarge.err; stop ablarge $rc; }
        done
      done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "ALL STEPS OK"
