import os, sys
sys.path.insert(0, "k8s-scheduler_amd")
os.environ["KSCHED_DEBUG"] = "1"
from ksched import MODE_BATCHED, Engine, cluster
cl = cluster.make_cluster("c3", n_nodes=30000, n_pods=2000)
for kw in (dict(topk=16, batch=64), dict(topk=8, batch=64, chunk_topk=8), dict(topk=4, batch=32, chunk_topk=4),
           dict(topk=16, batch=16), dict(topk=16, batch=64, pipe_wgs=9)):
    with Engine(mode=MODE_BATCHED, priority=cl.priority, domain=cl.domain, use_labels=cl.use_labels, **kw) as e:
        e.load_nodes(cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods, labels=cl.labels, price=cl.price)
        oi, os_, of = e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)
        print(kw, e.stats()["pipeline"], flush=True)
