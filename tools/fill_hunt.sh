#!/bin/bash
# LDS read-before-write hunt: the fresh-engine case with the LDS filled by chosen patterns / roles / ranges
#   FILLS="0 0x55555555" ROLES="7" bash tools/fill_hunt.sh
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
N=${JC_RUNS:-20}
for f in ${FILLS:-0}; do
  for r in ${ROLES:-7}; do
    tag="f${f}_r${r}_${KSCHED_LDS_LO:-0}_${KSCHED_LDS_HI:-x}"
    KSCHED_LDS_FILL=$f KSCHED_LDS_ROLE=$r JC_FRESH=${JC_FRESH:-1} KSCHED_PERSIST_TIMEOUT_MS=2000 timeout -k 10 200 \
      python -u tests/diag/jitter_case.py small1007 8 64 $N > gpurun_out/fh_$tag.log 2>&1
    rc=$?; echo "$tag rc=$rc: $(tail -1 gpurun_out/fh_$tag.log | cut -c1-160)"; grep "^run" gpurun_out/fh_$tag.log | head -1 | cut -c1-200
    if [ $rc -ge 124 ]; then exit $rc; fi
  done
done
