#!/bin/bash
# A/B of library variants (KSCHED_LIB) on the c4 bench + trace; VARIANTS names libksched_<v>.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"
S=tools/r03_gpu.sh
T="python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check"
bash $S step bench_main 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline || exit 1
for v in $VARIANTS; do
  KSCHED_LIB=$PWD/k8s-scheduler_amd/libksched_$v.so KSCHED_PERSIST_TRACE=1 bash $S step trace_$v 200 $T || exit 1
  KSCHED_LIB=$PWD/k8s-scheduler_amd/libksched_$v.so bash $S step bench_$v 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline || exit 1
done
