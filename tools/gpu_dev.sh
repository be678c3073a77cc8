#!/bin/bash
# Development GPU call: selected parity tests (PYTEST_K), then optional steps (BENCH args, PMC=1).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "${PYTEST_K:-}" > gpurun_out/pytest_dev.log 2>&1
if [ -n "$BENCH" ]; then
  timeout -k 10 200 python -u bench.py $BENCH > gpurun_out/bench_dev.json 2> gpurun_out/bench_dev.err
fi
if [ -n "$REHEARSE" ]; then
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $REHEARSE --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus $REHEARSE --same-device --steps 2 --warmup 1 > gpurun_out/rehearse_$REHEARSE.json 2> gpurun_out/rehearse_$REHEARSE.err
fi
if [ -n "$ARMS" ]; then ARMS="$ARMS" bash tools/ab_env.sh ${AB_ARGS:-} > gpurun_out/ab.txt 2>&1; fi
if [ -n "$PMC" ]; then bash tools/pmc_persist.sh; fi
echo done
