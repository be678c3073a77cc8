#!/bin/bash
# A/B of the node-sharded exchange tests (ranks as processes sharing one GPU) between the tree's library
# and an alternative in-tree build (KSCHED_LIB); every run under its own limit, stop at the first hang.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3 4; do
  for lib in libksched.so libksched_prev.so; do
    KSCHED_LIB=$PWD/k8s-scheduler_amd/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_xchg.py -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/xchg_${lib}_$i.log 2>&1
    rc=$?
    echo "$lib run $i rc=$rc $(tail -1 gpurun_out/xchg_${lib}_$i.log)"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
done
echo done
