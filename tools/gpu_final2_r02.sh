#!/bin/bash
# Round-2 evidence for the shipped build, in one call: GPU suite, smoke, PMC traffic for every bench key (N = 1, 2, 4, 8
# split shards and configs[1..3]), SQ counters, bench line, kernel trace, per-config lines, per-phase cycles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -f pmc_traffic.json
STEPS="tests smoke pmc sq phases" bash tools/gpu_final_r02.sh || exit $?
rm -rf gpurun_out/r02
STEPS="pmccfg bench prof cfgs" bash tools/gpu_r02.sh || exit $?
cp pmc_traffic.json gpurun_out/final/pmc_traffic.json
echo "gpu_final2_r02 done"
