#!/bin/bash
# Repeated c4 bench runs (robustness of the persistent pipeline); the first failure ends the call.
#   N=5 bash tools/repeat_bench.sh [bench args]
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in $(seq 1 "${N:-5}"); do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" >> gpurun_out/repeat.jsonl 2> gpurun_out/repeat_$i.err
  echo "run $i ok"
done
echo done
