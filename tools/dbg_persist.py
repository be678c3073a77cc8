"""Runs one (config, topk, batch, chunk_topk) case of the batched engine against the oracle; used to
bisect persistent-pipeline problems in subprocesses with their own time limit."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "k8s-scheduler_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
from ksched import MODE_BATCHED, Engine, cluster  # noqa: E402

name, nn, pp, K, B, KC = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6])
cl = cluster.make_cluster(name, n_nodes=nn, n_pods=pp)
want = O.schedule(cl, nthreads=8)
t = time.time()
with Engine(mode=MODE_BATCHED, priority=cl.priority, domain=cl.domain, use_labels=cl.use_labels, topk=K, batch=B,
            chunk_topk=KC) as e:
    e.load_nodes(cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods, labels=cl.labels, price=cl.price)
    oi, os_, of = e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)
    st = e.stats()
ok = np.array_equal(oi, want[0]) and np.array_equal(os_.view(np.int64), want[1].view(np.int64))
bad = np.nonzero(oi != want[0])[0]
print(name, nn, pp, K, B, KC, "ok" if ok else f"MISMATCH first {bad[:5]}", f"{time.time() - t:.2f}s", st["batches"],
      st["truncations"], flush=True)
