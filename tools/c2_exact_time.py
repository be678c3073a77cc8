#!/usr/bin/env python3
"""c2 (10k pods x 5k nodes, best-price) in exact mode: wall time per pod of ksched_schedule (inputs resident,
results on the host), one call after a warm-up call, for the one-workgroup kernel and the exchange kernel
(exact_wgs=3).   python tools/c2_exact_time.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "k8s-scheduler_amd")]
from ksched import MODE_EXACT, Engine, cluster  # noqa: E402

cl = cluster.make_cluster(sys.argv[1] if len(sys.argv) > 1 else "c2")
for wgs in (0, 3):
    with Engine(mode=MODE_EXACT, priority=cl.priority, domain=cl.domain, use_labels=cl.use_labels, exact_wgs=wgs) as e:
        e.load_nodes(cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods, labels=cl.labels, price=cl.price)
        e.save_state()
        best = None
        for _ in range(3):
            e.restore_state()
            t0 = time.perf_counter()
            e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        print(f"{cl.name} exact, exact_wgs={wgs}: {best * 1e3:.2f} ms per call, {best / cl.n_pods * 1e6:.3f} us per pod, "
              f"{cl.n_pods * cl.n_nodes / best:.3e} evals/s", flush=True)
