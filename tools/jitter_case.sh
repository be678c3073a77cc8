#!/bin/bash
# tests/diag/jitter_case.py variants, each its own process and time limit
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
run() {  # run <tag> <env...> -- <case args>
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u tests/diag/jitter_case.py "$@" > gpurun_out/jc_$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc: $(tail -1 gpurun_out/jc_$tag.log)"; grep "^run" gpurun_out/jc_$tag.log | head -3 | cut -c1-400
  [ $rc -lt 124 ]
}
N=${JC_RUNS:-150}
run fresh1 KSCHED_JITTER=7 JC_FRESH=1 -- small1007 8 64 $N &&
run fresh2 KSCHED_JITTER=7 JC_FRESH=2 -- small1007 8 64 $N &&
run fresh2_nojit JC_FRESH=2 -- small1007 8 64 $N &&
run fresh2_noscr KSCHED_JITTER=7 JC_FRESH=2 KSCHED_NO_TOUCH_SCREEN=1 -- small1007 8 64 $N &&
run fresh2_noresc KSCHED_JITTER=7 JC_FRESH=2 KSCHED_RESCUE_MAX=0 -- small1007 8 64 $N &&
run fresh2_traced KSCHED_JITTER=7 JC_FRESH=2 KSCHED_PERSIST_TRACE=1 KSCHED_TRACE_DUMP=/tmp/jc_trace.bin -- small1007 8 64 $N
