#!/bin/bash
# the persistent-pipeline parity subset, alternated over library builds (in-tree libksched_<name>.so; "main" = the
# tree's), <rounds> times: a rare parity failure as a count per build.   bash tools/pytest_ab.sh <rounds> <build...>
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
n=$1; shift
for i in $(seq 1 "$n"); do
  for v in "$@"; do
    if [ "$v" = main ]; then L=; else L=$PWD/k8s-scheduler_amd/libksched_$v.so; fi
    KSCHED_LIB=$L timeout -k 10 200 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu \
      tests/test_gpu_parity.py -k "persistent or golden or edge or full_size_c3" > gpurun_out/pab_${v}_$i.log 2>&1
    rc=$?; echo "$i $v rc=$rc $(tail -1 gpurun_out/pab_${v}_$i.log)"; grep "AssertionError:" gpurun_out/pab_${v}_$i.log | head -2 | cut -c1-300
    if [ $rc -ge 124 ]; then exit $rc; fi
  done
done
