#!/bin/bash
# Same-box A/B of in-tree builds over several workloads (tools/sweep.py specs), alternated twice.
#   AB_VARIANTS="main norescan" AB_SPECS="c4:batched:16:64 c5hc:batched:16:64" bash tools/ab_sweep.sh
# (main = the tree's libksched.so; any other name = k8s-scheduler_amd/libksched_<name>.so, tools/build_base.sh)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
V=${AB_VARIANTS:-"main base"}
S=${AB_SPECS:-"c4:batched:16:64 c3:batched:16:64 c5hc:batched:16:64"}
for pass in 1 2; do
  for v in $V; do
    if [ "$v" = main ]; then L=""; else L="$PWD/k8s-scheduler_amd/libksched_$v.so"; fi
    KSCHED_LIB=$L timeout -k 10 300 python -u tools/sweep.py $S > gpurun_out/ab_${v}_$pass.jsonl 2>/dev/null || exit $?
    python3 -c "
import json
for l in open('gpurun_out/ab_${v}_$pass.jsonl'):
    d = json.loads(l)
    print('$pass', '$v', d['spec'].split(':')[0], 'evals/s %.4e' % d['evals_per_s'], 'trunc', d.get('truncations'), 'resc', d.get('rescues'))"
  done
done
