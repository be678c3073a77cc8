#!/bin/bash
# PMC passes (one counter group per run, each under its own kill limit) over ONE bench step of the
# persistent pipeline on c4; summarise with tools/pmc_summary.py.  Counters of a persistent kernel
# cover the whole call (its single launch).
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/pmc
B="bench.py --no-cpu-baseline --no-check --steps 1 --warmup 0 ${BENCH_ARGS:-}"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc/fetch -o run -- python3 $B > gpurun_out/pmc/fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc/write -o run -- python3 $B > gpurun_out/pmc/write.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmc/sq -o run -- python3 $B > gpurun_out/pmc/sq.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d gpurun_out/pmc/sq2 -o run -- python3 $B > gpurun_out/pmc/sq2.log 2>&1
python3 tools/pmc_summary.py gpurun_out/pmc/summary.json gpurun_out/pmc/fetch gpurun_out/pmc/write gpurun_out/pmc/sq gpurun_out/pmc/sq2 > gpurun_out/pmc/summary.txt
rm -f gpurun_out/pmc/*/run_kernel_trace.csv
echo done
