#!/usr/bin/env python3
"""Repeat the edge-cluster parity cases on the persistent pipeline (batched, K 16, B 64) to measure how often a
mismatch occurs and whether it repeats on the same inputs.  python tests/diag/edge_repeat.py [reps] [seeds...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "k8s-scheduler_amd"), os.path.join(ROOT, "oracle"), ROOT, os.path.join(ROOT, "tests")]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    seeds = [int(x) for x in sys.argv[2:]] or list(range(12))
    import oracle as om
    from ksched import MODE_BATCHED, cluster
    from test_gpu_parity import run_engine
    combos = [(0, 0, False), (0, 1, False), (1, 1, False), (0, 1, True), (1, 1, True), (0, 0, True)]
    cases = []
    for seed in seeds:
        pr, dm, lb = combos[seed % 6]
        cl = cluster.random_small(500 + seed, n_nodes=37 + 61 * seed, n_pods=700, priority=pr, domain=dm, use_labels=lb)
        cases.append((seed, cl, om.schedule(cl)))
    bad = 0
    for r in range(reps):
        for seed, cl, want in cases:
            for kw in (dict(topk=4, batch=32), dict(topk=8, batch=64), dict(topk=16, batch=64)):
                got = run_engine(cl, MODE_BATCHED, **kw)
                d = np.nonzero(got[0] != want[0])[0]
                st = got[4]
                if d.size:
                    bad += 1
                    print(f"rep {r} seed {seed} {kw}: {d.size} differ from pod {d[0]} (got {got[0][d[:4]]} want "
                          f"{want[0][d[:4]]}) pipeline {st['pipeline']} batches {st['batches']} truncations "
                          f"{st['truncations']} rescues {st['rescues']}", flush=True)
        print(f"rep {r} done, {bad} mismatching runs so far", flush=True)


if __name__ == "__main__":
    main()
