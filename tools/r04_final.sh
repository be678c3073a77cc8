# the round's final validation on one box: full GPU suite, smoke, default bench (with cpu_baseline), then the
# profiled runs (kernel stats + PMC passes) of the same binary
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/final/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/final/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/final/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { cat gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail -20 gpurun_out/final/bench.err; exit 1; }
grep -o '"value": [0-9.e+]*\|"check_ok": [a-z]*\|"cpu_baseline": {[^}]*}' gpurun_out/final/bench.json
bash tools/pmc_passes.sh final all
