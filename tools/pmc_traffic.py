#!/usr/bin/env python3
"""HBM traffic of the engine kernel from rocprofv3 --pmc passes, recorded per build for bench.py's roofline.traffic.

Run on the GPU box (this process never touches the GPU; every pass is a child `rocprofv3 --pmc ... -- python3
tools/pmc_engine.py <bench args>`): FETCH_SIZE and WRITE_SIZE in separate passes (they need 3 + 2 TCC counters, 4
fit in one pass).  Per MI355X_MICROARCH.md (HBM / rocprofv3): on gfx950 FETCH_SIZE reports half the bytes of wide
16 B/lane streaming reads (the engine's LDS-DMA dwordx4 record stream), so the bytes are 2 x FETCH_SIZE + WRITE_SIZE
(an upper bound: the engine's 4-byte reads are counted in full); both raw counters are kept.  The entry is keyed by
the bench workload and the sha256 of openwhisk_amd/libowgs.so; bench.py reports it only for the same library.

    python3 tools/pmc_traffic.py [bench args, e.g. --config headline]
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def run_pass(counter: str, argv, out_dir: str):
    """one rocprofv3 --pmc pass; counter = one name (returns its values per engine dispatch) or several separated by
    spaces (returns {name: values})"""
    names = counter.split()
    shutil.rmtree(out_dir, ignore_errors=True)
    cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc"] + names + ["-d", out_dir, "-o", "run",
           "--output-format", "csv", "--", sys.executable, os.path.join(ROOT, "tools", "pmc_engine.py")] + argv
    with open(out_dir + ".log", "w") as log:
        rc = subprocess.call(cmd, stdout=log, stderr=subprocess.STDOUT, env=dict(os.environ, TMPDIR="/tmp"))
    if rc != 0:
        raise SystemExit(f"pmc pass {counter} rc={rc} (log {out_dir}.log)")
    vals = {n: [] for n in names}
    for f in sorted(glob.glob(os.path.join(out_dir, "**", "*counter_collection.csv"), recursive=True)):
        for row in csv.DictReader(open(f)):
            if "engine" in row.get("Kernel_Name", "") and row["Counter_Name"] in vals:
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    if not all(vals.values()):
        raise SystemExit(f"no engine dispatch in pass {counter}")
    return vals[names[0]] if len(names) == 1 else vals


ISSUE_PASSES = ("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY",
                "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR")


def issue_entry(argv, base: str, n_decisions: int) -> dict:
    """What bounds the engine instead of HBM: wave-instructions per decision and the fraction of wave cycles that
    issue an instruction (SQ counters of the measured dispatch, two passes)."""
    v = {}
    for i, counters in enumerate(ISSUE_PASSES):
        for k, x in run_pass(counters, argv, os.path.join(base, f"sq{i}")).items():
            v[k] = x[-1]
    insts = sum(v[k] for k in v if k.startswith("SQ_INSTS_"))
    return {"wave_insts_per_decision": insts / n_decisions,
            "valu_per_decision": v["SQ_INSTS_VALU"] / n_decisions,
            "lds_per_decision": v["SQ_INSTS_LDS"] / n_decisions,
            "issue_frac": v["SQ_ACTIVE_INST_ANY"] / v["SQ_WAVE_CYCLES"],
            "parked_frac": v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"],
            "waves": v["SQ_WAVES"], "counters": v,
            "source": "rocprofv3 --pmc SQ passes (tools/pmc_traffic.py): SQ_INSTS_* / decisions, "
                      "SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES"}


def main():
    argv = sys.argv[1:]
    args = bench.parse(argv)
    n_ctl, shards = bench.cluster_geometry(args, 0, 1)
    w = bench.shard_workload(args, shards[0], n_ctl)
    key = f"{args.config}|n{len(w.stream.act)}|c{n_ctl}|s{args.slots}|k1"
    base = os.path.join(ROOT, "gpurun_out", "pmc_traffic")
    os.makedirs(base, exist_ok=True)
    fetch = run_pass("FETCH_SIZE", argv, os.path.join(base, "fetch"))
    write = run_pass("WRITE_SIZE", argv, os.path.join(base, "write"))
    # the last dispatch is the measured replay (the first warms up); the counters are in KiB
    f_kib, w_kib = fetch[-1], write[-1]
    entry = {"lib_sha": bench.lib_sha(), "bytes": int((2 * f_kib + w_kib) * 1024),
             "fetch_kib": f_kib, "write_kib": w_kib, "dispatches": [fetch, write],
             "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/pmc_traffic.py): 2 x FETCH + WRITE",
             "algorithmic_bytes": bench.algorithmic_bytes(w),
             "issue": issue_entry(argv, base, len(w.stream.act))}
    try:
        d = json.load(open(bench.PMC_FILE))
    except (OSError, ValueError):
        d = {}
    d[key] = entry
    os.makedirs(os.path.dirname(bench.PMC_FILE), exist_ok=True)
    with open(bench.PMC_FILE, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)
    # gpurun merges gpurun_out back; keep a copy there too
    shutil.copy(bench.PMC_FILE, os.path.join(base, "pmc_traffic.json"))
    print(json.dumps({key: entry}))


if __name__ == "__main__":
    main()
