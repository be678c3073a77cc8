#!/bin/bash
# Round-2 measurement batch: the c4 phase trace + rocprof kernel stats, the per-rank shard sweep, and
# KC / grid A/Bs.  Each GPU step has its own time limit; set -e ends the call at the first failure.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
CONFIGS="c4 c3" PROF=1 bash tools/persist_trace.sh
SHARDS="12500 50000" GRIDS="240 128 64" bash tools/shard_sweep.sh
for kc in 2 8; do
  KSCHED_CHUNK_TOPK=$kc timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab_kc$kc.json 2> gpurun_out/ab_kc$kc.err
done
echo all done
