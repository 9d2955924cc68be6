#!/bin/bash
# Re-decision iteration on one box: mismatch check, re-decision cost profile (diag/libowgs_xp.so), parity subset, A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 300 python tools/debug_ext.py c2 200000 openwhisk_amd/libowgs.so || exit $?
if [ -f openwhisk_amd/diag/libowgs_xp.so ]; then
  OWGS_LIB=openwhisk_amd/diag/libowgs_xp.so REPS=1 timeout -k 10 300 python tools/prof_phases.py headline c2 || exit $?
fi
TESTK="${TESTK:-stream_parity or baseline_configs_full or c5_shard or cluster_shard or multi_shard or shim or concurrency_map or golden}" \
  PHASES="${PHASES:-headline c2 c4 headline:0/8 headline:0/4}" tools/gpu_ab.sh
