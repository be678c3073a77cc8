#!/usr/bin/env python3
"""Debug helper: one configuration against the oracle, first mismatches and the engine's stats.

  python tests/diag/dbg_case.py <config> <nodes> <pods> [wgs=0] [ranks=1]
ranks > 1: a local exchange group (threads of this process, ksched_xchg_join_local).  Environment variables
of the engine (KSCHED_NO_SCREEN, KSCHED_DEBUG, ...) apply as usual."""
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "k8s-scheduler_amd"), os.path.join(ROOT, "oracle")]


def pre_groups(spec):
    """DBG_PRE="cfg:nodes:pods:ranks,...": local exchange groups run (2 calls each, unchecked) before the case,
    as earlier tests of the same process would"""
    from ksched import cluster
    from ksched.dist import make_local_xchg_group
    for item in filter(None, spec.split(",")):
        c, n_, p_, r_ = item.split(":")
        cl = cluster.make_cluster(c, n_nodes=int(n_), n_pods=int(p_))
        grp = make_local_xchg_group(cl, int(r_), device=0, topk=16, batch=64)

        def work(e):
            e.save_state()
            for _ in range(2):
                e.restore_state()
                e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)
        th = [threading.Thread(target=work, args=(e,)) for e, _ in grp]
        [t.start() for t in th]
        [t.join() for t in th]
        for e, _ in grp:
            e.close()
        print(f"pre-group {item} done", flush=True)


def main():
    cfg, nn, pp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    if os.environ.get("DBG_TORCH"):  # as the GPU tests' gpu_available fixture does
        import torch
        print("torch cuda:", torch.cuda.is_available(), flush=True)
    pre_groups(os.environ.get("DBG_PRE", ""))
    wgs = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    ranks = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    import oracle as O
    from ksched import MODE_BATCHED, Engine, cluster
    from ksched.dist import make_local_xchg_group
    cl = cluster.make_cluster(cfg, n_nodes=nn, n_pods=pp)
    want = O.schedule(cl, nthreads=8)
    outs = []
    if ranks == 1:
        with Engine(mode=MODE_BATCHED, priority=cl.priority, domain=cl.domain, use_labels=cl.use_labels, topk=16,
                    batch=64, device=0, pipe_wgs=wgs) as e:
            e.load_nodes(cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods, labels=cl.labels, price=cl.price)
            oi, os_, of = e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)
            outs.append((oi, os_, of, e.stats()))
    else:
        grp = make_local_xchg_group(cl, ranks, device=0, topk=16, batch=64, pipe_wgs=wgs)
        res = [None] * ranks

        calls = int(os.environ.get("DBG_CALLS", "1"))

        def work(r):
            e = grp[r][0]
            e.save_state()
            for c in range(calls):
                e.restore_state()
                oi, os_, of = e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)
                bad = np.nonzero(oi != want[0])[0]
                print(f"rank {r} call {c}: {len(bad)} assignment mismatches, first {bad[:6].tolist()}", flush=True)
            res[r] = (oi, os_, of, e.stats())
        th = [threading.Thread(target=work, args=(r,)) for r in range(ranks)]
        [t.start() for t in th]
        [t.join() for t in th]
        outs = res
        for e, _ in grp:
            e.close()
    if len(outs) > 1:
        print("ranks agree:", all(np.array_equal(outs[0][0], o[0]) for o in outs), flush=True)
    for r, (oi, os_, of, st) in enumerate(outs):
        bad = np.nonzero((oi != want[0]) | (of != want[2]) | (os_.view(np.int64) != want[1].view(np.int64)))[0]
        print(f"rank {r}: {len(bad)} mismatches, first {bad[:6].tolist()} | pipeline {st['pipeline']} batches "
              f"{st['batches']} trunc {st['truncations']} rescues {st['rescues']} exact_rows {st['exact_rows']} "
              f"scan_rows {st['scan_rows']}", flush=True)
        for i in bad[:4]:
            print(f"   pod {i}: got ({oi[i]}, {os_[i]!r}, {of[i]}) want ({want[0][i]}, {want[1][i]!r}, {want[2][i]})")


if __name__ == "__main__":
    main()
