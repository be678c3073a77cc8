# same-binary A/B of environment settings on the default c4 bench: AB_ENVS="NAME=v1 NAME=v2 ..." (repeated twice)
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for kv in $AB_ENVS; do
    env "$kv" timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/abenv.json 2>/dev/null || exit 1
    echo "$kv $(grep -o '"value": [0-9.e+]*\|"truncated_batches_per_step": [0-9]*\|"check_ok": [a-z]*' gpurun_out/abenv.json | tr '\n' ' ')"
  done
done
