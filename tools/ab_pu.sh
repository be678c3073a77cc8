#!/bin/bash
# A/B of the score scan's rows per step (KSCHED_PERSIST_PU 2 / 4 (tree) / 8) through KSCHED_LIB builds, c4.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in libksched.so libksched_pu2.so libksched_pu8.so libksched.so; do
  KSCHED_LIB=$PWD/k8s-scheduler_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --check-pods 2000 > gpurun_out/ab_pu_$lib.json 2> gpurun_out/ab_pu_$lib.err
  echo "$lib $(tail -1 gpurun_out/ab_pu_$lib.json | cut -c1-80)"
done
echo done
