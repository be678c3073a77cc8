#!/bin/bash
# each case in its own process under its own limit; stops at the first timeout / crash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in $CASES; do
  timeout -k 5 40 python -u tools/dbg_persist.py ${c//:/ } >> gpurun_out/dbg.log 2>&1 || { echo "case $c failed rc=$?" >> gpurun_out/dbg.log; exit 1; }
done
echo done >> gpurun_out/dbg.log
