#!/bin/bash
# parity of the persistent pipeline (full size + parity + exchange), then the c4 trace and bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
S=tools/r03_gpu.sh
T="python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check"
bash $S step pytest_s8 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_xchg.py || exit 1
KSCHED_PERSIST_TRACE=1 KSCHED_COMMIT_STAMPS=1 KSCHED_MERGE_STAMPS=1 bash $S step trace_main 200 $T || exit 1
bash $S step bench_main 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline || exit 1
