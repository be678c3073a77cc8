#!/bin/bash
# One rank's share of an N-GPU c4 run, measured on one GPU: c4's 1M pods against 100k/N nodes (the
# shard a rank scores), with the persistent grid at several sizes and the phase trace on.  Everything
# of the chain except the cross-GPU exchange (chain budget).
#   SHARDS="12500 25000" GRIDS="248 128 64" bash tools/shard_sweep.sh
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in ${SHARDS:-12500}; do
  for g in ${GRIDS:-248 128 64}; do
    KSCHED_PERSIST_G=$g KSCHED_PERSIST_TRACE=1 timeout -k 10 120 python -u bench.py --nodes $n --steps 1 --warmup 1 \
      --no-cpu-baseline --no-check > gpurun_out/shard_${n}_g$g.json 2> gpurun_out/shard_${n}_g$g.err
    echo "shard $n G $g ok"
  done
done
echo done
