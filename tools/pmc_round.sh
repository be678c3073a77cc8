#!/bin/bash
# rocprofv3 kernel stats of the bench + PMC passes (one counter group per run) on a c4 prefix
# (1000 batches of 64 pods at 100k nodes); summarise with tools/pmc_summary.py.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/pmc
W="tools/sweep.py c4:batched:16:64:64000"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc/fetch -o run -- python3 $W > gpurun_out/pmc/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc/write -o run -- python3 $W > gpurun_out/pmc/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmc/sq -o run -- python3 $W > gpurun_out/pmc/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d gpurun_out/pmc/sq2 -o run -- python3 $W > gpurun_out/pmc/sq2.log 2>&1
echo done
