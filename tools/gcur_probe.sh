#!/bin/bash
# Round-4 diagnostic for c4's extra HBM writes: the shipped library against the OWGS_EXP_NOGCUR variant (no walk-cursor
# stores, tools/build_variant.sh nogcur -DOWGS_EXP_NOGCUR): bench rate + bit-exactness, WRITE_SIZE and store
# wave-instructions of the engine dispatch, per config.  Outputs under gpurun_out/gcur.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/gcur; mkdir -p $O; export TMPDIR=/tmp
for lib in openwhisk_amd/libowgs.so openwhisk_amd/variants/libowgs_nogcur.so; do
  n=$(basename $lib .so)
  for c in c4 headline; do
    OWGS_LIB=$lib timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-h2d --no-shim-path --no-cpu-baseline > $O/bench_${n}_$c.json 2> $O/bench_${n}_$c.err
    rc=$?; cut -c1-200 $O/bench_${n}_$c.json; [ $rc -eq 0 ] || { tail -5 $O/bench_${n}_$c.err; exit $rc; }
    OWGS_LIB=$lib timeout -k 10 300 python3 -c "
import sys, json; sys.path.insert(0, 'tools'); import pmc_traffic as P
w = P.run_pass('WRITE_SIZE', ['--config', '$c'], '$O/w_${n}_$c')
q = P.run_pass('SQ_INSTS_VMEM_WR SQ_WAVES', ['--config', '$c'], '$O/q_${n}_$c')
print(json.dumps({'lib': '$n', 'config': '$c', 'write_kib': w, 'vmem_wr': q['SQ_INSTS_VMEM_WR']}))" >> $O/pmc.jsonl 2> $O/pmc_${n}_$c.err
    rc=$?; tail -1 $O/pmc.jsonl; [ $rc -eq 0 ] || { tail -5 $O/pmc_${n}_$c.err; exit $rc; }
  done
done
echo gcur_probe done
