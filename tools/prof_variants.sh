#!/bin/bash
# rocprof kernel stats of a 1000-batch c4 prefix: default pipeline (a), single stream (b), KC=2 (c)
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_a -o run -- python3 tools/sweep.py c4:batched:16:64:64000 > gpurun_out/prof_a.log 2>&1
KSCHED_ONE_STREAM=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b -o run -- python3 tools/sweep.py c4:batched:16:64:64000 > gpurun_out/prof_b.log 2>&1
KSCHED_CHUNK_TOPK=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c -o run -- python3 tools/sweep.py c4:batched:16:64:64000 > gpurun_out/prof_c.log 2>&1
