#!/bin/bash
# parity (full size + persistent parity + exchange) of the fast merge and branch-free screen, then the c4 phase
# trace and bench of the main build and of the variants given in VARIANTS (libksched_<v>.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
S=tools/r03_gpu.sh
T="python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check"
bash $S step pytest_s5 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_parity.py || exit 1
KSCHED_PERSIST_TRACE=1 KSCHED_COMMIT_STAMPS=1 KSCHED_MERGE_STAMPS=1 bash $S step trace_main 200 $T || exit 1
bash $S step bench_main 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline || exit 1
for v in $VARIANTS; do
  KSCHED_LIB=$PWD/k8s-scheduler_amd/libksched_$v.so KSCHED_PERSIST_TRACE=1 bash $S step trace_$v 200 $T || exit 1
  KSCHED_LIB=$PWD/k8s-scheduler_amd/libksched_$v.so bash $S step bench_$v 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline || exit 1
done
