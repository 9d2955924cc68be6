#!/bin/bash
# GPU suite, then the bench at 1 shard per GPU and with several controller shards per engine launch, then rocprof.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu3.log 2>&1 || { tail -30 gpurun_out/pytest_gpu3.log; exit 1; }
tail -1 gpurun_out/pytest_gpu3.log
timeout -k 10 300 python bench.py > gpurun_out/b1.log 2>&1 || { tail gpurun_out/b1.log; exit 1; }
tail -1 gpurun_out/b1.log | cut -c1-300
for k in ${KS:-2 4 8}; do
timeout -k 10 200 python bench.py --no-cpu-baseline --shards-per-gpu $k > gpurun_out/bk$k.log 2>&1 || { tail gpurun_out/bk$k.log; exit 1; }
tail -1 gpurun_out/bk$k.log | cut -c1-300; done
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/prof.log 2>&1 || { tail gpurun_out/prof.log; exit 1; }
echo prof done
