"""Node-sharded persistent pipeline with the device-side exchange (ksched_xchg_*), R processes on the
one GPU of the test box: every rank's results must equal the CPU oracle's sequential schedule, bit for
bit, and the ranks' node shards together must equal the oracle's final state.  Exercises the product
multi-rank code: global node indices at node_offset > 0, granule exchange through IPC-mapped rings,
the rank merge in the merger workgroups and the owner-only write-back (the xGMI transport itself needs
several GPUs)."""
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "k8s-scheduler_amd"), os.path.join(ROOT, "oracle"), os.path.dirname(__file__)]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,nn,pp,world", [("c3", 24000, 3000, 2), ("c5hc", 20000, 3000, 2), ("c4", 30000, 2500, 3),
                                                     ("c4", 100000, 2500, 2)])
def test_xchg_ranks_match_oracle(cfg, nn, pp, world):
    import oracle as O
    import xchg_worker
    from ksched import cluster
    cl = cluster.make_cluster(cfg, n_nodes=nn, n_pods=pp)
    want = O.schedule(cl, nthreads=8)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=xchg_worker.run_rank, args=(r, world, port, cfg, nn, pp, 2, q)) for r in range(world)]
    for p in procs:
        p.start()
    res, errs = {}, {}
    try:
        for _ in range(world):
            r, status, out, rng, state = q.get(timeout=110)
            if status == "ok":
                res[r] = (out, rng, state)
            else:
                errs[r] = out
    finally:
        for p in procs:
            p.join(timeout=15)
            if p.is_alive():
                p.kill()
    assert not errs, "\n".join(f"rank {r}: {t}" for r, t in sorted(errs.items()))
    for r in range(world):
        out, rng, state = res[r]
        for oi, osb, of, pipe, nb, ntr in out:
            assert pipe == "persistent", f"rank {r} ran the {pipe} pipeline"
            assert np.array_equal(oi, want[0]), f"rank {r}: assignments differ at {np.nonzero(oi != want[0])[0][:5]}"
            assert np.array_equal(osb, want[1].view(np.int64)), f"rank {r}: score bits differ"
            assert np.array_equal(of, want[2]), f"rank {r}: feasible counts differ"
    got = [np.concatenate([res[r][2][k] for r in range(world)]) for k in range(3)]
    for k in range(3):
        assert np.array_equal(got[k], want[3][k]), f"final node state (resource {k}) differs"
