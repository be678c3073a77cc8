# quick validation of a persistent-pipeline change: smoke, parity, exchange, timeout recovery, trace, bench
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/r04_gpu.sh s3 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_persist_recovery.py > gpurun_out/pytest_recovery.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_recovery.log; exit $rc
