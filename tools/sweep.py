#!/usr/bin/env python3
"""Parameter sweep of the engine on one GPU (exploration helper; prints one JSON line per run).

  python tools/sweep.py c3:exact c3:batched:16:128 c4:batched:16:256 ...
spec = config[:mode[:topk[:batch[:pods[:nodes]]]]]
An argument @NAME=V[,NAME=V...] sets engine environment switches (read at engine creation) for the specs after it,
e.g. @KSCHED_RESCUE_MAX=4,KSCHED_RESCUE_RATE=4; each line names them in "env".
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "k8s-scheduler_amd"))


def run(spec, reps=2):
    from ksched import MODE_BATCHED, MODE_EXACT, Engine, cluster
    parts = spec.split(":")
    cfg = parts[0]
    mode = parts[1] if len(parts) > 1 else "exact"
    topk = int(parts[2]) if len(parts) > 2 else 16
    batch = int(parts[3]) if len(parts) > 3 else 0
    pods = int(parts[4]) if len(parts) > 4 and parts[4] else None
    nodes = int(parts[5]) if len(parts) > 5 and parts[5] else None
    cl = cluster.make_cluster(cfg, n_pods=pods, n_nodes=nodes)
    m = MODE_EXACT if mode == "exact" else MODE_BATCHED
    with Engine(mode=m, priority=cl.priority, domain=cl.domain, use_labels=cl.use_labels, topk=topk, batch=batch,
                device=0, timing=True) as e:
        e.load_nodes(cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods, labels=cl.labels, price=cl.price)
        e.save_state()
        e.upload_pods(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)
        best = None
        for _ in range(reps):
            e.restore_state()
            t0 = time.perf_counter()
            e.run()
            e.sync()
            dt = time.perf_counter() - t0
            st = e.stats()
            if best is None or dt < best[0]:
                best = (dt, st)
        dt, st = best
        oi, _, _ = e.results()
    out = dict(spec=spec, pods=cl.n_pods, nodes=cl.n_nodes, wall_s=dt, evals_per_s=cl.n_pods * cl.n_nodes / dt,
               pods_per_s=cl.n_pods / dt, placed=int((oi >= 0).sum()), batches=st["batches"],
               truncations=st["truncations"], rescues=st.get("rescues"), pipeline=st.get("pipeline"),
               device_ms=st["device_ms"],
               fam_avg_ms=[st["kernel_ms"][f] / max(st["kernel_launches"][f], 1) for f in range(4)],
               fam_timed=st["kernel_launches"], env=ENV_TAG)
    print(json.dumps(out), flush=True)


ENV_TAG = ""

if __name__ == "__main__":
    for s in sys.argv[1:]:
        if s.startswith("@"):
            ENV_TAG = s[1:]
            for kv in ENV_TAG.split(","):
                k, v = kv.split("=", 1)
                os.environ[k] = v
            continue
        try:
            run(s)
        except Exception as ex:
            print(json.dumps(dict(spec=s, error=repr(ex))), flush=True)
