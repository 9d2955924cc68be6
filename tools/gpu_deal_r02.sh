cd "${GRAFT_REPO_ROOT}"; export TMPDIR=/tmp
for d in 1 2 3 4 5; do echo "== deal $d"; OWGS_DEAL=$d REPS=3 timeout -k 10 300 python tools/prof_phases.py headline headline:0/2 headline:0/8 2>&1 | grep "ms (min" | cut -c1-110 || exit 1; done
