#!/bin/bash
# GPU tests, c4 repeats and trace of the tree; then the grid at CUs - 8 with the commit's agent release
# (stall experiment).  A test failure (rc 1) is recorded and the call goes on; time limits/crashes end it.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/pytest_gpu.log)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
N=4 bash tools/repeat_bench.sh --steps 3 --warmup 1 || exit $?
mv gpurun_out/repeat.jsonl gpurun_out/repeat_tree.jsonl
CONFIGS=c4 bash tools/persist_trace.sh || exit $?
KSCHED_PERSIST_G=248 KSCHED_COMMIT_RELEASE=1 KSCHED_PROG_WAVES=1 N=8 bash tools/repeat_bench.sh --steps 3 --warmup 1 --no-check || exit $?
echo all done
