#!/bin/bash
# Round-3 session 2: the tests the last run did not reach, smoke, the c4 bench and a c4 phase trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
S=tools/r03_gpu.sh
bash $S step pytest_rest 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_xchg.py tests/test_host_kube.py tests/test_gpu_persist_recovery.py &&
bash $S step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
bash $S step bench 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline &&
KSCHED_PERSIST_TRACE=1 KSCHED_COMMIT_STAMPS=1 KSCHED_MERGE_STAMPS=1 bash $S step trace_c4 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check
