"""Worker of tests/test_gpu_xchg.py: one rank of the node-sharded persistent pipeline with the
device-side exchange, as its own process (several ranks share the test box's one GPU).  Not a test
module: spawned by the test with multiprocessing."""
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "k8s-scheduler_amd")]


def run_rank(rank, world, port, cfg, nn, pp, calls, q):
    try:
        # ranks on ONE device (test harness only; one GPU per rank in production): each rank's kernel is a
        # plain launch of opts.pipe_wgs workgroups, one CU each, and the ranks wait on one another, so they
        # must all be resident at once -- which nothing guarantees for independent launches of separate
        # processes.  Half the CUs in total leaves every XCD room for an uneven placement (at 3 x 80 of 256
        # a rank once started only after the others' waits expired)
        os.environ.setdefault("KSCHED_PERSIST_TIMEOUT_MS", "20000")
        import numpy as np
        import torch.distributed as dist
        from ksched import MODE_BATCHED, cluster
        from ksched.dist import make_sharded_engine
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        cl = cluster.make_cluster(cfg, n_nodes=nn, n_pods=pp)
        eng, (lo, hi) = make_sharded_engine(cl, rank, world, device=0, mode=MODE_BATCHED, comm=False, xchg=True,
                                            topk=16, batch=64, pipe_wgs=128 // world)
        assert eng.xchg_ready, "exchange setup failed"
        out = []
        eng.save_state()
        for c in range(calls):  # repeated calls: the granule tags advance across calls
            eng.restore_state()
            oi, os_, of = eng.schedule(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)
            st = eng.stats()
            out.append((oi, os_.view(np.int64), of, st["pipeline"], st["batches"], st["truncations"]))
        state = eng.read_nodes()
        eng.close()
        dist.destroy_process_group()
        q.put((rank, "ok", out, (lo, hi), state))
    except Exception:
        q.put((rank, "error", traceback.format_exc(), None, None))
