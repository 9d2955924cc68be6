cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/cw
for cw in 96 128 192 256 336; do for d in 1 2; do
echo "== cw $cw deal $d"; OWGS_CW=$cw OWGS_DEAL=$d REPS=2 timeout -k 10 200 python tools/prof_phases.py headline:0/8 c2 headline 2>&1 | grep -v amdgpu.ids | cut -c1-150 || exit 1
done; done
