#!/bin/bash
# GPU parity tests + smoke (+ optional short bench), each step under its own time limit; the first
# failure ends the call.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "${PYTEST_K:-}" > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python -u bench.py $BENCH > gpurun_out/bench.json 2> gpurun_out/bench.err
fi
echo done
