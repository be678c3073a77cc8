#!/bin/bash
# rocprofv3 kernel statistics and PMC passes of the default c4 bench itself (the binary and workload the bench
# line times: one warm-up step + one timed step), one counter group per profiled run, each under its own kill
# timer (MI355X_MICROARCH "rocprofv3 PMC slots": <= 8 SQ, <= 4 TCC -- FETCH_SIZE 3, WRITE_SIZE 2 -- per pass).
#   bash tools/pmc_passes.sh <tag> stats|fetch|write|sq|sq2|ic|list|all
# Output: gpurun_out/pmc_<tag>/<pass>/run_*.csv; then
#   python tools/pmc_summary.py profiles/<tag>_pmc_c4_pipe.json gpurun_out/pmc_<tag>/{fetch,write,sq,sq2}
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
export TMPDIR=/tmp
# the cooperative launch's runtime state faults in the HIP runtime's exit handler after rocprofv3's finalization
# (DESIGN.md section 6.1): profiled runs launch the same kernels plainly, after the same occupancy check
export KSCHED_PLAIN_LAUNCH=1
tag=$1; shift
out=gpurun_out/pmc_$tag
mkdir -p "$out"
BENCH="bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check"
pass() {  # pass <name> <counters...>
  local name=$1; shift
  echo "pass $name: $*"
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$out/$name" -o run \
    -- python3 $BENCH > "$out/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
stats() {
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run \
    -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > "$out/stats_bench.json" 2> "$out/stats.err"
  local rc=$?
  rm -f "$out"/stats/run_kernel_trace.csv  # one row per launch: large, summarised by run_kernel_stats.csv
  echo "stats rc=$rc"
  return $rc
}
run() {
  case "$1" in
    stats) stats ;;
    fetch) pass fetch FETCH_SIZE ;;
    write) pass write WRITE_SIZE ;;
    sq) pass sq SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
          SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE ;;
    sq2) pass sq2 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 \
           SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU ;;
    ic) pass ic SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES \
          SQ_BUSY_CYCLES GRBM_GUI_ACTIVE ;;
    list) timeout -s KILL 60 rocprofv3 -L > "$out/avail.txt" 2>&1; echo "list rc=$?" ;;
    all) run stats && run fetch && run write && run sq && run sq2 ;;
    *) echo "unknown pass $1"; return 2 ;;
  esac
}
run "${1:-all}"
