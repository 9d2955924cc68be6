cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_msgs.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_msgs.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_msgs.log; [ $rc -le 1 ] && \
timeout -k 10 300 python tools/time_msgs.py > gpurun_out/time_msgs.log 2>&1; cat gpurun_out/time_msgs.log; \
rm -rf gpurun_out/prof_msgs && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_msgs -o run --output-format csv -- python3 tools/time_msgs.py > gpurun_out/prof_msgs.log 2>&1; cut -c1-200 gpurun_out/prof_msgs/run_kernel_stats.csv | head -14
