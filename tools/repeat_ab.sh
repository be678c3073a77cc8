#!/bin/bash
# parity repeat on several library builds (in-tree libksched_<name>.so; "main" = the tree's): mismatch rates
#   bash tools/repeat_ab.sh <reps> <build...>
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
reps=$1; shift
for v in "$@"; do
  if [ "$v" = main ]; then L=; else L=$PWD/k8s-scheduler_amd/libksched_$v.so; fi
  KSCHED_LIB=$L timeout -k 10 400 python -u tests/diag/golden_repeat.py "$reps" $REP_ARGS > gpurun_out/rep_$v.log 2>&1
  rc=$?; echo "$v rc=$rc: $(tail -1 gpurun_out/rep_$v.log)"; grep "differ" gpurun_out/rep_$v.log | head -3
  if [ $rc -ge 124 ]; then exit $rc; fi
done
