#!/bin/bash
# A/B phase traces of the c4 bench: screened scan (default) vs KSCHED_NO_SCREEN=1; each run its own time limit
set -o pipefail
cd "$GRAFT_REPO_ROOT"
S=tools/r03_gpu.sh
T="python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check"
for cfg in ${CONFIGS:-c4}; do
KSCHED_PERSIST_TRACE=1 KSCHED_COMMIT_STAMPS=1 KSCHED_MERGE_STAMPS=1 bash $S step trace_${cfg}_screen 200 $T --config $cfg &&
KSCHED_NO_SCREEN=1 KSCHED_PERSIST_TRACE=1 bash $S step trace_${cfg}_noscreen 200 $T --config $cfg || exit 1
done
bash $S step bench_screen 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check &&
KSCHED_NO_SCREEN=1 bash $S step bench_noscreen 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check
