#!/bin/bash
# A/B of the merger's issue priority (KSCHED_MERGE_LOW_PRIO: 0 -> 3 (default), 3 -> 2, 2 -> 1) at c4.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 3 2 0; do
  KSCHED_MERGE_LOW_PRIO=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-check --steps 3 --warmup 1 >> gpurun_out/ab_prio.jsonl 2> gpurun_out/ab_prio_$v.err
  echo "prio setting $v ok"
done
echo done
