cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_health.py tests/test_gpu_acks.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_health.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_health.log; [ $rc -le 1 ] && \
timeout -k 10 200 python tools/time_health.py > gpurun_out/time_health.log 2>&1; cat gpurun_out/time_health.log; \
rm -rf gpurun_out/prof_health && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_health -o run --output-format csv -- python3 tools/time_health.py > gpurun_out/prof_health.log 2>&1; head -12 gpurun_out/prof_health/*/run_kernel_stats.csv gpurun_out/prof_health/run_kernel_stats.csv 2>/dev/null
