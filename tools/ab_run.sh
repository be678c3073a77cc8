cd "$GRAFT_REPO_ROOT" || exit 1
B="python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline"
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "persistent or golden" > gpurun_out/ab_pytest.log 2>&1 && tail -1 gpurun_out/ab_pytest.log &&
for v in ${AB_VARIANTS:-main noearly}; do
  if [ $v = main ]; then L=""; else L="$PWD/k8s-scheduler_amd/libksched_$v.so"; fi
  KSCHED_LIB=$L timeout -k 10 200 $B > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || exit 1
  echo "$v $(grep -o '"value": [0-9.e+]*' gpurun_out/ab_$v.json) $(grep -o '"check_ok": [a-z]*' gpurun_out/ab_$v.json)"
done
