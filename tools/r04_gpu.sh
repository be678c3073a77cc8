#!/bin/bash
# Round-4 GPU session helper: build-free (the .so travels), each GPU step under its own time limit, chained:
# the first failing step ends the call.   usage: bash tools/r04_gpu.sh <preset> | step <name> <secs> <cmd...>
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/r04_steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r04_steps.log
  tail -3 "gpurun_out/$name.log"
  return $rc
}
soft() {  # soft <name> <seconds> <cmd...>: a step whose failure (rc 1: a failed test) does not end the call;
          # a crash, abort or time limit (rc >= 124) does
  step "$@"
  local rc=$?
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
trace() {  # trace <name> [bench args]: the c4 phase trace with the raw per-batch stamps dumped
  local name=$1; shift
  KSCHED_PERSIST_TRACE=1 KSCHED_COMMIT_STAMPS=1 KSCHED_MERGE_STAMPS=1 KSCHED_TRACE_DUMP=gpurun_out/$name.bin \
    step "$name" 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check "$@"
}
case "$1" in
  quick)
    step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
    step pytest_pipe 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
      -k "persistent or golden or edge or full_size_c3" &&
    step pytest_xchg 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_xchg.py &&
    trace trace_c4 &&
    step bench_c4 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline
    ;;
  all)
    step pytest_all 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/
    ;;
  exitprobe)  # one variant per step; the first that faults at exit ends the chain (tools/exit_probe.py)
    for v in ${EXIT_VARIANTS:-torch ksched oracle leak}; do
      step exit_$v 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_exit_$v -o run \
        -- python3 tools/exit_probe.py $v || exit 1
    done
    ;;
  s2)
    KSCHED_POISON=1 soft xchg_poison 200 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
      tests/test_gpu_xchg.py -k c4-100000 &&
    soft xchg_all 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_xchg.py &&
    trace trace_c4 &&
    KSCHED_RESCUE_MAX=0 soft bench_c4_norescue 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline &&
    soft bench_c4 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline &&
    KSCHED_RESCUE_MAX=2 soft bench_c4_resc2 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline
    ;;
  s3)
    step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
    step pytest_pipe 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
      -k "persistent or golden or edge or full_size_c3" &&
    step pytest_xchg 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_xchg.py &&
    trace trace_c4 &&
    step bench_c4 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline
    ;;
  trace) shift; trace "$@" ;;
  *) "$@" ;;
esac
