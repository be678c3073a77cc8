#!/bin/bash
# GPU tests, c4 repeats and a trace of the tree (merge head-state prefetch A/B).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/pytest_gpu.log)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
N=4 bash tools/repeat_bench.sh --steps 3 --warmup 1 || exit $?
CONFIGS=c4 bash tools/persist_trace.sh || exit $?
echo all done
