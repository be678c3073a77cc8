#!/bin/bash
# A/B of the main build and the VARIANTS builds: c4 trace + bench each (no tests)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
S=tools/r03_gpu.sh
T="python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check"
KSCHED_PERSIST_TRACE=1 KSCHED_COMMIT_STAMPS=1 bash $S step trace_main 200 $T || exit 1
bash $S step bench_main 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline || exit 1
for v in $VARIANTS; do
  KSCHED_LIB=$PWD/k8s-scheduler_amd/libksched_$v.so KSCHED_PERSIST_TRACE=1 KSCHED_COMMIT_STAMPS=1 bash $S step trace_$v 200 $T || exit 1
  KSCHED_LIB=$PWD/k8s-scheduler_amd/libksched_$v.so bash $S step bench_$v 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline || exit 1
done
