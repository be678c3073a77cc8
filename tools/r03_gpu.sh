#!/bin/bash
# Round-3 GPU session: build-free (the .so travels), each GPU step under its own time limit, chained.
set -o pipefail
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/r03_steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03_steps.log
  tail -5 "gpurun_out/$name.log"
  return $rc
}
case "$1" in
  quick)
    step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
    step pytest_pipe 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "persistent or golden or edge or stream_pipeline or full_size_c3" &&
    step recovery 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_persist_recovery.py &&
    step bench_c4 600 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline
    ;;
  all)
    step pytest_all 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/
    ;;
  *) "$@" ;;
esac
