#!/bin/bash
# The rescue bucket sweep: c4, c3 and c5hc at each (KSCHED_RESCUE_MAX, KSCHED_RESCUE_RATE)
# (KSCHED_RESCUE_LOOK) (KSCHED_RESCUE_CAP, default max) (KSCHED_RESCUE_LOW, default max) set, one process per pass, two passes.  bash tools/rescue_sweep.sh "4,16,1 4,4,0,16 ..."
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
args=()
sets=${1:-"4,16,0 4,16,1 4,8,1 4,4,1 8,16,1 8,8,1"}
for s in $sets; do
  IFS=, read -r m r l c lo <<< "$s"
  args+=("@KSCHED_RESCUE_MAX=$m,KSCHED_RESCUE_RATE=$r,KSCHED_RESCUE_LOOK=$l,KSCHED_RESCUE_CAP=${c:-$m},KSCHED_RESCUE_LOW=${lo:-$m}" c4:batched:16:64 c3:batched:16:64 c5hc:batched:16:64)
done
for pass in 1 2; do
  timeout -k 10 500 python -u tools/sweep.py "${args[@]}" > gpurun_out/rescue_sweep_$pass.jsonl || exit $?
done
python3 - <<'PY'
import json
for p in (1, 2):
    for l in open(f"gpurun_out/rescue_sweep_{p}.jsonl"):
        d = json.loads(l)
        if "error" in d: print(p, d); continue
        print(p, d["env"], d["spec"].split(":")[0], "evals/s %.4e" % d["evals_per_s"], "batches", d["batches"],
              "trunc", d["truncations"], "resc", d["rescues"])
PY
