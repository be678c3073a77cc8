# rescue budget A/B on c4 (bench) and c5hc / c3 (sweep), after a parity check of the persistent pipeline
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "persistent or golden" > gpurun_out/rab_pytest.log 2>&1 || { tail -30 gpurun_out/rab_pytest.log; exit 1; }
tail -1 gpurun_out/rab_pytest.log
for m in ${RESCUE_BUDGETS:-2 4 8}; do
  KSCHED_RESCUE_MAX=$m timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rab_c4_$m.json 2>/dev/null || exit 1
  echo "c4 budget $m: $(grep -o '"value": [0-9.e+]*\|"truncated_batches_per_step": [0-9]*\|"rescued_lists_per_step": [0-9]*\|"check_ok": [a-z]*' gpurun_out/rab_c4_$m.json | tr '\n' ' ')"
  KSCHED_RESCUE_MAX=$m timeout -k 10 200 python -u tools/sweep.py c5hc:batched:16:64 c3:batched:16:64 > gpurun_out/rab_sweep_$m.jsonl 2>/dev/null || exit 1
  python3 -c "
import json,sys
for l in open('gpurun_out/rab_sweep_$m.jsonl'):
    d=json.loads(l); print('   ', d['spec'], 'evals/s %.3e' % d['evals_per_s'], 'batches', d['batches'], 'truncations', d['truncations'], 'rescues', d['rescues'])"
done
