#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel stats, optional sweep.
# Each GPU step has its own time limit; steps are chained (set -e) so the first failure ends the call.
#   SKIP_TESTS=1  skip pytest -m gpu;  SWEEP="c4:batched:16:64 ..." run tools/sweep.py afterwards
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
fi
timeout -k 10 240 python -u bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
if [ -z "$SKIP_PROF" ]; then
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --no-check --steps 2 --warmup 1 "$@" > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
  # keep the per-kernel summary; the full trace (one row per launch) is summarised by tools/trace_gaps.py
  # here and then dropped (it exceeds what gpurun copies back)
  TRACE=$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)
  if [ -n "$TRACE" ]; then python3 tools/trace_gaps.py "$TRACE" > gpurun_out/trace_gaps.txt 2>&1 || true; rm -f "$TRACE"; fi
fi
if [ -n "$SWEEP" ]; then
  timeout -k 10 400 python -u tools/sweep.py $SWEEP > gpurun_out/sweep.jsonl 2> gpurun_out/sweep.err
fi
echo done
