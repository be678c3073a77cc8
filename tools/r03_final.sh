#!/bin/bash
# round-3 final validation of the tree: the whole GPU suite, smoke, the c4 phase trace, the default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
S=tools/r03_gpu.sh
bash $S step final_pytest 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ || exit 1
bash $S step final_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
KSCHED_PERSIST_TRACE=1 KSCHED_COMMIT_STAMPS=1 KSCHED_MERGE_STAMPS=1 bash $S step final_trace 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check || exit 1
bash $S step final_bench 600 python -u bench.py || exit 1
