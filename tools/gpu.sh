#!/bin/bash
# GPU session helper (runs on the gpurun box; build-free: the in-tree .so travels).  Every GPU step runs under
# its own time limit and the steps are chained: the first failing step ends the call.
#   bash tools/gpu.sh <preset>            presets below
#   bash tools/gpu.sh trace <name> [bench args]
#   bash tools/gpu.sh step <name> <secs> <cmd...>
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
export TMPDIR=/tmp
mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu"
step() {  # step <name> <seconds> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -3 "gpurun_out/$name.log"
  return $rc
}
soft() {  # a step whose failure (rc 1: a failed test) does not end the call; a crash, abort or time limit does
  step "$@"
  local rc=$?
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
trace() {  # trace <name> [bench args]: the c4 phase trace, raw per-batch stamps dumped and summarised
  local name=$1; shift
  KSCHED_PERSIST_TRACE=1 KSCHED_COMMIT_STAMPS=1 KSCHED_MERGE_STAMPS=1 KSCHED_TRACE_DUMP=gpurun_out/$name.bin \
    step "$name" 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check "$@" &&
  python3 tools/trace_dist.py gpurun_out/$name.bin > gpurun_out/${name}_dist.txt
}
bench() {  # bench <name> [bench args]
  local name=$1; shift
  step "$name" 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" &&
  grep -o '"value": [0-9.e+]*\|"truncated_batches_per_step": [0-9]*\|"rescued_lists_per_step": [0-9]*\|"check_ok": [a-z]*' \
    "gpurun_out/$name.log" | tr '\n' ' '; echo
}
abl() {  # abl <label> <lib name or main> [bench args]: the bench on an in-tree A/B build (tools/build_base.sh)
  local name=$1 lib=$2; shift 2
  if [ "$lib" = main ]; then KSCHED_LIB= bench "ab_$name" "$@"; else KSCHED_LIB=$PWD/k8s-scheduler_amd/libksched_$lib.so bench "ab_$name" "$@"; fi
}
case "$1" in
  baseline)  # the tree as it stands: bench + phase trace
    bench bench_c4 && trace trace_c4
    ;;
  quick)  # a persistent-pipeline change: smoke, parity, exchange, trace, bench
    step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
    step pytest_pipe 600 $PYT tests/test_gpu_parity.py -k "persistent or golden or edge or full_size_c3" &&
    step pytest_xchg 600 $PYT tests/test_gpu_xchg.py &&
    trace trace_c4 &&
    bench bench_c4
    ;;
  xchg)
    step pytest_xchg 600 $PYT tests/test_gpu_xchg.py tests/test_gpu_multirank.py
    ;;
  ab)  # same-box A/B of libksched_base.so against the tree's build, alternated twice
    abl base1 base && abl main1 main && abl base2 base && abl main2 main
    ;;
  check_ab)  # a change: smoke, parity and exchange tests (failures reported, not fatal), A/B, trace
    step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
    soft pytest_pipe 600 $PYT tests/test_gpu_parity.py -k "persistent or golden or edge or full_size_c3" &&
    soft pytest_xchg 900 $PYT tests/test_gpu_xchg.py &&
    KSCHED_DEBUG=1 abl main0 main --steps 1 &&
    abl base1 base && abl main1 main && abl base2 base && abl main2 main &&
    trace trace_c4
    ;;
  full)  # a commit change: smoke, parity (persistent subset, full-size, exchange), screen counters, trace, bench
    step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
    step pytest_pipe 600 $PYT tests/test_gpu_parity.py -k "persistent or golden or edge or full_size_c3" &&
    step pytest_full 900 $PYT tests/test_gpu_fullsize.py &&
    step pytest_xchg 900 $PYT tests/test_gpu_xchg.py &&
    KSCHED_COMMIT_STAMPS=1 KSCHED_PERSIST_TRACE=1 step stamps_c4 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check &&
    trace trace_c4 &&
    bench bench_c4
    ;;
  full_ab)  # full's checks (failures reported, not fatal), then an A/B of the tree against two builds
    step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
    soft pytest_pipe 600 $PYT tests/test_gpu_parity.py -k "persistent or golden or edge or full_size_c3" &&
    soft pytest_full 900 $PYT tests/test_gpu_fullsize.py &&
    soft pytest_xchg 900 $PYT tests/test_gpu_xchg.py &&
    KSCHED_COMMIT_STAMPS=1 KSCHED_PERSIST_TRACE=1 step stamps_c4 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check &&
    trace trace_c4 &&
    abl main1 main && abl ${AB1:-base}1 ${AB1:-base} && abl ${AB2:-noscr}1 ${AB2:-noscr} &&
    abl main2 main && abl ${AB1:-base}2 ${AB1:-base} && abl ${AB2:-noscr}2 ${AB2:-noscr}
    ;;
  xchg_exp)  # DESIGN 6.1's ring experiment
    soft xchg_exp 900 python -u tests/diag/xchg_ring_experiment.py $XCHG_VARIANTS
    ;;
  all)
    step pytest_all 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/
    ;;
  trace) shift; trace "$@" ;;
  bench) shift; bench "$@" ;;
  *) "$@" ;;
esac
