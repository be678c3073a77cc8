#!/bin/bash
# A/B of engine environment switches on the bench (no tests): each arm runs bench.py once.
#   ARMS="name:VAR=1 name2:VAR2=1,VAR3=0 base:" bash tools/ab_env.sh [bench args]
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for arm in $ARMS; do
  name=${arm%%:*}; vars=${arm#*:}
  env_args=""
  for kv in ${vars//,/ }; do env_args="$env_args $kv"; done
  timeout -k 10 200 env $env_args python -u bench.py --no-cpu-baseline --no-check "$@" > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err
  echo "$name $(python3 -c "import json;d=json.load(open('gpurun_out/ab_$name.json'));print(round(d['value']/1e9,2),'Geval/s',round(d['ms_per_step'],1),'ms',{k:round(v*1e3,1) for k,v in d['kernel_avg_ms'].items()})")"
done
