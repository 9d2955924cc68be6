#!/bin/bash
# rocprofv3 kernel-trace summaries of the per-config bench workloads (configs[1], configs[3], a C5 shard of 8)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/profcfg; mkdir -p $O; export TMPDIR=/tmp
for c in "--config c2" "--config c4" "--cluster-size 8"; do
  tag=$(echo $c | tr -d ' -')
  rm -rf $O/$tag
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv -- \
    python3 bench.py $c --steps 3 --warmup 1 --no-cpu-baseline --no-check --no-h2d > $O/$tag.log 2>&1
  rc=$?; tail -1 $O/$tag.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
