#!/bin/bash
# Per-batch phase trace of the persistent pipeline (KSCHED_PERSIST_TRACE / COMMIT / MERGE stamps) on
# the bench workloads, one short bench per config; then the plain rocprofv3 kernel stats of the bench.
#   CONFIGS="c4 c3 c5" bash tools/persist_trace.sh
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in ${CONFIGS:-c4}; do
  KSCHED_PERSIST_TRACE=1 KSCHED_COMMIT_STAMPS=1 KSCHED_MERGE_STAMPS=1 timeout -k 10 120 python -u bench.py --config $c \
    --steps 1 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/trace_$c.json 2> gpurun_out/trace_$c.err
done
if [ -n "$PROF" ]; then
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --no-check --steps 2 --warmup 1 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
  rm -f gpurun_out/prof/*kernel_trace.csv
fi
echo done
