#!/bin/bash
# copy the round-3 evidence (gpurun_out/r03, tools/gpu_final_r03.sh) into profiles/ and the bench's PMC table
cd "$(dirname "$0")/.."
O=gpurun_out/r03
cp_if() { [ -f "$1" ] && cp "$1" "$2" && echo "$2"; }
cp_if $O/pytest_gpu.log profiles/r03_pytest_gpu.log
cp_if $O/smoke.log profiles/r03_smoke.log
cp_if $O/bench.json profiles/r03_bench.json
cp_if $O/prof/run_kernel_stats.csv profiles/r03_kernel_stats.csv
cp_if $O/cfgs.jsonl profiles/r03_cfgs_bench.jsonl
cp_if $O/pmc_traffic.json profiles/r03_pmc_traffic.json
cp_if $O/pmc_traffic.json pmc_traffic.json
cp_if $O/sq_pmc.txt profiles/r03_sq_pmc.txt
cp_if $O/churn.jsonl profiles/r03_health_per_batch_bench.jsonl
cp_if $O/shimprof/run_kernel_stats.csv profiles/r03_shim_kernel_stats.csv
cp_if $O/phases.log profiles/r03_phases.log
for f in $O/ab_*.log; do [ -f "$f" ] && cp_if "$f" "profiles/r03b_$(basename $f)"; done
true
