#!/usr/bin/env python3
"""One golden cluster under KSCHED_JITTER, run many times in one process (the seed advances per call): mismatch count,
and for the first mismatches the device's per-batch trace (rounds, rescues, resolved pods).
  KSCHED_JITTER=7 python tests/diag/jitter_case.py small1007 8 64 [runs=200]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "k8s-scheduler_amd"), os.path.join(ROOT, "oracle"), ROOT, os.path.join(ROOT, "tests")]


def main():
    name, K, B = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    runs = int(sys.argv[4]) if len(sys.argv) > 4 else 200
    from ksched import MODE_BATCHED, Engine
    from test_oracle import _cluster_from
    with open(os.path.join(ROOT, "tests", "golden", "clusters.json")) as f:
        fx = next(c for c in json.load(f) if c["name"] == name)
    cl = _cluster_from(fx)
    want = np.asarray(fx["expect_idx"], np.int32)
    bad = 0
    dump = os.environ.get("KSCHED_TRACE_DUMP")
    fresh = os.environ.get("JC_FRESH", "0")  # 1: a new engine per run; 2: also a K 4, B 32 run before each

    def one(e, i):
        nonlocal bad
        e.restore_state()
        oi, _, _ = e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)
        st = e.stats()
        d = np.nonzero(oi != want)[0]
        if d.size:
            bad += 1
            msg = (f"run {i}: {d.size} differ from pod {d[0]} (got {oi[d[:4]]} want {want[d[:4]]}) batches {st['batches']}"
                   f" truncations {st['truncations']} rescues {st['rescues']}")
            if dump and os.path.exists(dump) and bad <= 3:
                t = np.fromfile(dump, dtype=np.uint64).reshape(-1, 54)
                rows = []
                for b in range(min(12, t.shape[0])):
                    c = int(t[b, 16])
                    if t[b, 4] == 0 and c == 0:
                        continue
                    rows.append(f"b{b}: rounds {c & 0xffff} rescues {(c >> 16) & 0xff} done {(c >> 24) & 0xff}"
                                f" failed {(c >> 32) & 0xffff} seq {c >> 48}")
                msg += " | " + "; ".join(rows)
            print(msg, flush=True)

    def engine(k, b):
        e = Engine(mode=MODE_BATCHED, priority=cl.priority, domain=cl.domain, use_labels=cl.use_labels, topk=k, batch=b)
        e.load_nodes(cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods, labels=cl.labels, price=cl.price)
        e.save_state()
        return e

    if fresh == "0":
        with engine(K, B) as e:
            for i in range(runs):
                one(e, i)
    else:
        for i in range(runs):
            if fresh == "2":
                with engine(4, 32) as e0:
                    e0.restore_state()
                    e0.schedule(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)
            with engine(K, B) as e:
                one(e, i)
    print(f"{name} K {K} B {B}: {bad} of {runs} runs mismatched", flush=True)


if __name__ == "__main__":
    main()
