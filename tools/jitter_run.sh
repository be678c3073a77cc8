#!/bin/bash
# parity under KSCHED_JITTER (random delays at the persistent pipeline's protocol points), several seeds
#   bash tools/jitter_run.sh <reps> <seed...>
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
reps=$1; shift
for sd in "$@"; do
  KSCHED_JITTER=$sd timeout -k 10 500 python -u tests/diag/golden_repeat.py "$reps" $REP_ARGS > gpurun_out/jit_$sd.log 2>&1
  rc=$?; echo "seed $sd rc=$rc: $(tail -1 gpurun_out/jit_$sd.log)"; grep "differ" gpurun_out/jit_$sd.log | head -4 | cut -c1-250
  if [ $rc -ge 124 ]; then exit $rc; fi
done
