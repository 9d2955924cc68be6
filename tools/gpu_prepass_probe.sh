#!/bin/bash
# pre-pass latency of small publish batches per batch size and dealing mode (tools/prepass_probe.py, kernel trace)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ppp; mkdir -p $O; export TMPDIR=/tmp
for n in ${SIZES:-16 64 300 448}; do
for d in ${DEALS:-1}; do
  rm -rf $O/d${d}_$n
  OWGS_DEAL=$d timeout -k 10 200 rocprofv3 --kernel-trace -d $O/d${d}_$n -o run --output-format csv -- python3 tools/prepass_probe.py $n 200 > $O/d${d}_$n.log 2>&1 || { tail $O/d${d}_$n.log; exit 1; }
  python3 - "$O/d${d}_$n" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "owgs_" in r["Kernel_Name"]:
        d[r["Kernel_Name"][5:20]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
print(sys.argv[1], {k: (len(v), round(sorted(v)[len(v) // 2], 1)) for k, v in d.items() if len(v) > 10})
PY
done
done
