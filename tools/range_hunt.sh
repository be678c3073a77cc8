#!/bin/bash
# commit-LDS range bisection: the fresh-engine case with only [lo, hi) of the commit's LDS filled (role 1, distinct pattern)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
N=${JC_RUNS:-30}
for rg in "$@"; do
  lo=${rg%:*}; hi=${rg#*:}
  KSCHED_LDS_FILL=0x40404040 KSCHED_LDS_ROLE=9 KSCHED_LDS_LO=$lo KSCHED_LDS_HI=$hi JC_FRESH=1 KSCHED_PERSIST_TIMEOUT_MS=2000 \
    timeout -k 10 200 python -u tests/diag/jitter_case.py small1007 8 64 $N > gpurun_out/rh_$lo.log 2>&1
  rc=$?; echo "[$lo,$hi) rc=$rc: $(tail -1 gpurun_out/rh_$lo.log | cut -c1-200)"; grep "^run" gpurun_out/rh_$lo.log | head -1 | cut -c1-160
  if [ $rc -ge 124 ]; then exit $rc; fi
done
