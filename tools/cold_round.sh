#!/bin/bash
# The node-sharded exchange tests first on a fresh box (cold), then the full round (tools/gpu_round.sh).
# A test failure (rc 1) is recorded and the round goes on; a time limit or a crash ends the call.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_xchg.py -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/xchg_first.log 2>&1
rc=$?
echo "xchg first rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_round.sh
