#!/bin/bash
# copy the round-4 evidence (gpurun_out/r04f, tools/gpu_final_r04.sh) into profiles/ and the bench's PMC table
cd "$(dirname "$0")/.."
O=gpurun_out/r04f
cp_if() { [ -f "$1" ] && cp "$1" "$2" && echo "$2"; }
cp_if $O/pytest_gpu.log profiles/r04_pytest_gpu.log
cp_if $O/smoke.log profiles/r04_smoke.log
cp_if $O/bench.json profiles/r04_bench.json
cp_if $O/prof/run_kernel_stats.csv profiles/r04_kernel_stats.csv
cp_if $O/cfgs.jsonl profiles/r04_cfgs_bench.jsonl
cp_if $O/pmc_traffic.json profiles/r04_pmc_traffic.json
cp_if $O/pmc_traffic.json pmc_traffic.json
cp_if $O/sq_pmc.txt profiles/r04_sq_pmc.txt
cp_if $O/shim.json profiles/r04_shim_leg.json
cp_if $O/stream_cfgs.jsonl profiles/r04_stream_mode_cfgs_final.jsonl
cp_if $O/shimprof/run_kernel_stats.csv profiles/r04_shim_kernel_stats.csv
true
