cd "$GRAFT_REPO_ROOT" || exit 1
for v in fixed main fixed main; do
  if [ $v = main ]; then L=""; else L="$PWD/k8s-scheduler_amd/libksched_$v.so"; fi
  KSCHED_LIB=$L timeout -k 10 200 python -u tools/sweep.py c5hc:batched:16:64 c4:batched:16:64:200000 > gpurun_out/ab2_$v.jsonl 2>/dev/null || exit 1
  python3 -c "
import json
for l in open('gpurun_out/ab2_$v.jsonl'):
    d=json.loads(l); print('$v', d['spec'], 'evals/s %.4e' % d['evals_per_s'], 'trunc', d['truncations'], 'resc', d['rescues'])"
done
