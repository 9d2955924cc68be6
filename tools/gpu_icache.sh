#!/bin/bash
# instruction-cache counters of the engine (one rocprofv3 --pmc pass per counter group): are instruction fetches a cost?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/icache; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1
grep -o "SQC_[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_LEVEL[A-Z_]*" $O/avail.txt | sort -u | tr '\n' ' '; echo
i=0
for set in "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $O/p$i -o run --output-format csv -- python3 tools/pmc_engine.py ${ARGS:-} > $O/p$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pass $i rc=$rc"; tail -3 $O/p$i.log; continue; }
  python3 - "$O/p$i" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "engine" in r.get("Kernel_Name", ""):
            agg[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
if agg:
    print(sys.argv[1], {k: f"{v:.4g}" for k, v in agg[max(agg)].items()})
PY
done
