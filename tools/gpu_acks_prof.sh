cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 python tools/time_acks.py > gpurun_out/time_acks.log 2>&1; cat gpurun_out/time_acks.log | tail -3; \
rm -rf gpurun_out/prof_acks && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_acks -o run --output-format csv -- python3 tools/time_acks.py > gpurun_out/prof_acks.log 2>&1; cut -c1-160 gpurun_out/prof_acks/run_kernel_stats.csv | head -12
