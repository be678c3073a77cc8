#!/bin/bash
# Config sweep of the final tree (c2 exact, c3/c4/c5/c5hc batched) and a grid-size A/B at c4.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/sweep.py c2:exact c3:exact c3:batched:16:64 c5:batched:16:64 c5hc:batched:16:64 > gpurun_out/sweep.jsonl 2> gpurun_out/sweep.err
for g in 224 232; do
  KSCHED_PERSIST_G=$g timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-check --steps 3 --warmup 1 > gpurun_out/ab_g$g.json 2> gpurun_out/ab_g$g.err
done
echo all done
