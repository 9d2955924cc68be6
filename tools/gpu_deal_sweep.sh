cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/deal
for d in 1 4 5 2 3; do
  OWGS_DEAL=$d REPS=3 timeout -k 10 200 python tools/prof_phases.py headline headline:0/8 > gpurun_out/deal/d$d.log 2>&1 || exit 1
  echo "deal $d"; grep "ms (min" gpurun_out/deal/d$d.log | cut -c1-110
done
