#!/bin/bash
# Chunk-width sweep (OWGS_CW) of the current build on the given workloads (diagnostics)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
for cw in ${CWS:-128 336}; do
echo "== cw $cw"; OWGS_CW=$cw REPS=2 timeout -k 10 200 python tools/prof_phases.py ${SPECS:-headline:0/8 c2 headline} 2>&1 | grep -v amdgpu.ids | cut -c1-200 || exit 1
done
