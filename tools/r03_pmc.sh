#!/bin/bash
# rocprofv3 kernel stats of the c4 bench + PMC passes (one counter group per run, each under its own
# kill timer) of the full c4 workload through tools/sweep.py; summary -> gpurun_out/pmc/r03_pmc_c4_pipe.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/pmc
W="tools/sweep.py c4:batched:16:64"
pass() {  # pass <name> <counters...>
  local name=$1; shift
  echo "pass $name: $*"
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc/$name -o run -- python3 $W > gpurun_out/pmc/$name.log 2>&1
}
[ "$1" = stats ] && { timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err; exit $?; }
# one pass per gpurun call: rocprofv3 segfaults in the profiled process's exit handlers after writing its
# output (both with bench.py and with tools/sweep.py), and nothing more may run on the GPU after that
case "$1" in
  fetch) pass fetch FETCH_SIZE ;;
  write) pass write WRITE_SIZE ;;
  sq) pass sq SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE ;;
  sq2) pass sq2 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU ;;
esac
echo "rc=$?"
