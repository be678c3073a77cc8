#!/bin/bash
# lag-3 pipeline: the whole GPU suite, then the c4 phase trace and bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
S=tools/r03_gpu.sh
T="python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check"
bash $S step pytest_s6 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ || exit 1
KSCHED_PERSIST_TRACE=1 KSCHED_COMMIT_STAMPS=1 KSCHED_MERGE_STAMPS=1 bash $S step trace_main 200 $T || exit 1
bash $S step bench_main 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline || exit 1
