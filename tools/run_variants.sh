#!/bin/bash
# Times every diagnostic engine variant on the given workloads (default headline); stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for so in openwhisk_amd/variants/libowgs_*.so; do
  echo "== $so"
  OWGS_LIB=$so timeout -k 10 120 python tools/prof_phases.py ${@:-headline} || exit $?
done
