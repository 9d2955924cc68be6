#!/bin/bash
# SQ counter passes for the engine kernel (each pass its own rocprofv3 run; no tracing domains besides kernel dispatch)
#   bash tools/pmc_run.sh [bench args, e.g. --config headline]   -> gpurun_out/pmc/summary.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 tools/pmc_engine.py "$@" > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i rc=$rc"; tail -5 gpurun_out/pmc/p$i.log; exit $rc; fi
done
python3 - <<'PY' | tee gpurun_out/pmc/summary.txt
import csv, glob, collections
agg = collections.defaultdict(dict)
for f in sorted(glob.glob("gpurun_out/pmc/p*/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        if "engine" not in k:
            continue
        agg[(f.split("/")[2], row.get("Dispatch_Id"))][row["Counter_Name"]] = float(row["Counter_Value"])
for (p, d), v in sorted(agg.items()):
    print(p, d, {k: f"{x:.4g}" for k, x in v.items()})
# the last dispatch of each pass is the measured replay (the first warms up)
last = {}
for (p, d), v in sorted(agg.items(), key=lambda kv: (kv[0][0], int(kv[0][1] or 0))):
    last[p] = v
tot = {k: x for v in last.values() for k, x in v.items()}
if tot.get("SQ_WAVE_CYCLES"):
    print("parked (SQ_WAIT_ANY / SQ_WAVE_CYCLES): %.3f" % (tot["SQ_WAIT_ANY"] / tot["SQ_WAVE_CYCLES"]))
    print("issuing (SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES): %.3f" % (tot["SQ_ACTIVE_INST_ANY"] / tot["SQ_WAVE_CYCLES"]))
if tot.get("SQ_INSTS_LDS"):
    print("LDS bank-conflict cycles per LDS instruction: %.3f" % (tot["SQ_LDS_BANK_CONFLICT"] / tot["SQ_INSTS_LDS"]))
PY
