#!/bin/bash
# the fresh-engine reproduction (tests/diag/jitter_case.py, JC_FRESH=2) on several library builds
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
N=${JC_RUNS:-30}
for v in "$@"; do
  if [ "$v" = main ]; then L=; else L=$PWD/k8s-scheduler_amd/libksched_$v.so; fi
  KSCHED_LIB=$L JC_FRESH=2 KSCHED_PERSIST_TIMEOUT_MS=3000 timeout -k 10 300 python -u tests/diag/jitter_case.py small1007 8 64 $N > gpurun_out/fab_$v.log 2>&1
  rc=$?; echo "$v rc=$rc: $(tail -1 gpurun_out/fab_$v.log | cut -c1-200)"; grep "^run" gpurun_out/fab_$v.log | head -2 | cut -c1-200
  if [ $rc -ge 124 ]; then exit $rc; fi
done
