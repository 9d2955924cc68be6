#!/bin/bash
# Several controller shards of one split-slot cluster on ONE GPU (one engine launch, one workgroup per shard):
# bench.py --shards-per-gpu K with clusterSize K, 16 GiB invokers split K ways (configs[4]'s memory).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/shards; mkdir -p $O; export TMPDIR=/tmp
for k in 2 4 8; do
  timeout -k 10 600 python bench.py --shards-per-gpu $k --steps 3 --warmup 1 --no-h2d >> $O/shards.jsonl 2>> $O/shards.err
  rc=$?; tail -1 $O/shards.jsonl | cut -c1-260; [ $rc -eq 0 ] || { tail -20 $O/shards.err; exit $rc; }
done
