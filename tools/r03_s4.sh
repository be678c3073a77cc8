#!/bin/bash
# parity of the screened scan (full-size configs + persistent-pipeline parity), then the c4 phase trace and bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
S=tools/r03_gpu.sh
bash $S step pytest_screen 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_parity.py &&
KSCHED_PERSIST_TRACE=1 KSCHED_COMMIT_STAMPS=1 KSCHED_MERGE_STAMPS=1 bash $S step trace_c4 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check &&
bash $S step bench 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline
