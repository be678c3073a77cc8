#!/usr/bin/env python3
"""Repeat the golden clusters (the committed expected outputs) and the edge clusters on the persistent pipeline's
modes, counting mismatches: a rare, timing-dependent parity failure shows up as a rate.
  python tests/diag/golden_repeat.py [reps]     (KSCHED_LIB selects the library build)"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "k8s-scheduler_amd"), os.path.join(ROOT, "oracle"), ROOT, os.path.join(ROOT, "tests")]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    all_modes = "--all-modes" in sys.argv  # every mode of the parity tests, in their order (exact first)
    from ksched import MODE_BATCHED
    from test_gpu_parity import modes, run_engine
    from test_oracle import _cluster_from
    with open(os.path.join(ROOT, "tests", "golden", "clusters.json")) as f:
        gold = json.load(f)
    cases = []
    for c in gold:
        cl = _cluster_from(c)
        cases.append((c["name"], cl, np.asarray(c["expect_idx"], np.int32)))
    kws = [(MODE_BATCHED, dict(topk=4, batch=32)), (MODE_BATCHED, dict(topk=8, batch=64)),
           (MODE_BATCHED, dict(topk=16, batch=64)), (MODE_BATCHED, dict(topk=16, batch=64, chunk_topk=2))]
    if all_modes:
        kws = [(mode, kw) for _, mode, kw in modes()]
    bad = 0
    runs = 0
    for r in range(reps):
        for name, cl, want in cases:
            for mode, kw in kws:
                got = run_engine(cl, mode, **kw)
                runs += 1
                d = np.nonzero(got[0] != want)[0]
                if d.size:
                    bad += 1
                    st = got[4]
                    print(f"rep {r} {name} {mode} {kw}: {d.size} differ from pod {d[0]} (got {got[0][d[:4]]} want {want[d[:4]]})"
                          f" pipeline {st['pipeline']} batches {st['batches']} truncations {st['truncations']}", flush=True)
        print(f"rep {r}: {bad} of {runs} runs mismatched", flush=True)


if __name__ == "__main__":
    main()
