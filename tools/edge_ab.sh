cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in main noscr oldlay main; do
  if [ $v = main ]; then L=; else L=$PWD/k8s-scheduler_amd/libksched_$v.so; fi
  KSCHED_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "edge" > gpurun_out/edge_$v.log 2>&1
  rc=$?; echo "$v rc=$rc $(tail -1 gpurun_out/edge_$v.log)"; grep "AssertionError:" gpurun_out/edge_$v.log | head -2
  if [ $rc -ge 124 ]; then exit $rc; fi
done
