cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && rm -rf gpurun_out/pmc_msgs && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/pmc_msgs -o p1 --output-format csv -- python3 tools/time_msgs.py > gpurun_out/pmc_msgs.log 2>&1; \
python3 - <<'PY'
import csv, glob, collections
for f in glob.glob("gpurun_out/pmc_msgs/**/*counter_collection.csv", recursive=True):
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:40]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); 
    for k, d in agg.items():
        if "msg_write" in k or "msg_size" in k:
            print(k, {c: f"{v:.4g}" for c, v in d.items()})
PY
