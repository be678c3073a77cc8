"""Multi-rank (node-sharded) scheduling on CPU with torch.distributed gloo, world_size 2 and 3.

Each rank owns a contiguous node shard and computes local top-K candidate records for every pod of a
batch (the CPU restatement of k_score_topk + k_merge), the records are exchanged with a real
all-gather (the engine uses RCCL ncclAllGather for the same bytes), merged identically on every rank
(k_merge<INPUT_REC>), and every rank replays the same ordered commit (k_commit), writing back only
the nodes it owns.  The result must equal the unsharded sequential semantics bit for bit, and all
ranks must agree.  Also covers the 128-byte unique-id broadcast used to set up RCCL.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cfg, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (os.path.join(root, "k8s-scheduler_amd"), os.path.join(root, "oracle"), here):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    import oracle as O
    from ksched import cluster
    from ksched.dist import broadcast_bytes, shard_range
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # unique-id broadcast (ksched.dist -> ksched_set_comm on GPU)
        uid = bytes(range(128)) if rank == 0 else None
        uid = broadcast_bytes(uid, rank)
        assert uid == bytes(range(128))

        name, nn, pp, K, B, combo = cfg
        if name == "small":
            cl = cluster.random_small(4242, n_nodes=nn, n_pods=pp, priority=combo[0], domain=combo[1],
                                      use_labels=combo[2])
        else:
            cl = cluster.make_cluster(name, n_nodes=nn, n_pods=pp)
        lo, hi = shard_range(cl.n_nodes, rank, world)
        ac = cl.alloc_cpu[lo:hi].copy(); am = cl.alloc_mem[lo:hi].copy(); ap = cl.alloc_pods[lo:hi].copy()
        lab = None if cl.labels is None else np.ascontiguousarray(cl.labels[lo:hi])
        pr = None if cl.price is None else np.ascontiguousarray(cl.price[lo:hi])
        opts = (cl.priority, cl.domain, cl.use_labels)
        P = cl.n_pods
        out_i = np.empty(P, np.int32); out_s = np.empty(P, np.float64); out_f = np.empty(P, np.int32)
        pos, batches = 0, 0
        while pos < P:
            nb = min(B, P - pos)
            sl = slice(pos, pos + nb)
            sel = None if cl.selector is None else np.ascontiguousarray(cl.selector[sl])
            recs, fc = O.local_topk(opts, K, lo, ac, am, ap, lab, pr, np.ascontiguousarray(cl.req_cpu[sl]),
                                    np.ascontiguousarray(cl.req_mem[sl]), np.ascontiguousarray(cl.req_pods[sl]), sel)
            # one all-gather of {records, feasible counts} (the RCCL exchange)
            payload = np.concatenate([recs.view(np.uint8), fc.view(np.uint8)])
            t = torch.from_numpy(payload.copy())
            parts = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(parts, t)
            rb = recs.nbytes
            recs_all = np.concatenate([p.numpy()[:rb].view(O.REC_DTYPE) for p in parts])
            fc_all = np.concatenate([p.numpy()[rb:].view(np.int64) for p in parts])
            lists, fc0 = O.merge_topk(K, world, nb, recs_all, fc_all)
            done, touched, oi, os_, of = O.commit_batch(opts, K, np.ascontiguousarray(cl.req_cpu[sl]),
                                                        np.ascontiguousarray(cl.req_mem[sl]),
                                                        np.ascontiguousarray(cl.req_pods[sl]), sel, lists, fc0, B)
            assert done >= 1
            out_i[pos:pos + done] = oi[:done]; out_s[pos:pos + done] = os_[:done]; out_f[pos:pos + done] = of[:done]
            for x in touched:
                j = int(x["idx"])
                if lo <= j < hi:
                    ac[j - lo], am[j - lo], ap[j - lo] = x["cur"]
            pos += done
            batches += 1
        # every rank must hold the same decisions
        mine = torch.from_numpy(np.concatenate([out_i.view(np.uint8), out_s.view(np.uint8), out_f.view(np.uint8)]))
        allv = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine)
        for v in allv:
            assert torch.equal(v, mine)
        st = [None] * world
        dist.all_gather_object(st, (ac, am, ap))
        if rank == 0:
            q.put(("ok", out_i, out_s, out_f, [np.concatenate([s[k] for s in st]) for k in range(3)], batches))
    except Exception as e:  # surface the failure to the parent
        q.put(("err", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


CASES = [
    ("c3", 900, 500, 8, 64, None, 2),
    ("c5", 1200, 500, 16, 128, None, 2),
    ("c2", 700, 600, 4, 32, None, 3),
    ("small", 130, 400, 4, 48, (0, 0, False), 2),
    ("small", 130, 400, 8, 48, (1, 1, True), 2),
    ("small", 131, 400, 4, 16, (0, 1, True), 3),
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-w{c[-1]}-{i}" for i, c in enumerate(CASES)])
def test_sharded_equals_sequential(oracle_mod, case):
    from ksched import cluster
    name, nn, pp, K, B, combo, world = case
    if name == "small":
        cl = cluster.random_small(4242, n_nodes=nn, n_pods=pp, priority=combo[0], domain=combo[1], use_labels=combo[2])
    else:
        cl = cluster.make_cluster(name, n_nodes=nn, n_pods=pp)
    wi, ws, wf, wst = oracle_mod.schedule(cl)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, (name, nn, pp, K, B, combo), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert res[0] == "ok", res
    _, oi, os_, of, st, batches = res
    assert np.array_equal(oi, wi)
    assert np.array_equal(os_.view(np.int64), ws.view(np.int64))
    assert np.array_equal(of, wf)
    for a, b in zip(st, wst):
        assert np.array_equal(a, b)
    assert batches >= 1


class _FakeXchgEngine:
    """Stands in for ksched.Engine in the exchange setup (CPU): export returns a per-rank handle or
    fails, import records what it was given, close turns the (imported) exchange off again."""

    def __init__(self, rank, fail_export=False, fail_import=False):
        self.rank, self.fail_export, self.fail_import = rank, fail_export, fail_import
        self.imported = None
        self.ready = False

    def xchg_close(self):
        self.ready = False

    def xchg_export(self):
        if self.fail_export:
            raise RuntimeError("no IPC")
        return bytes([self.rank]) * 64

    def xchg_import(self, handles):
        if self.fail_import:
            raise RuntimeError("cannot map")
        self.imported = list(handles)
        self.ready = True


def _xchg_worker(rank, world, port, fail_rank, fail_where, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "k8s-scheduler_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    from ksched.dist import setup_exchange
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = _FakeXchgEngine(rank, fail_export=(rank == fail_rank and fail_where == "export"),
                              fail_import=(rank == fail_rank and fail_where == "import"))
        ok = setup_exchange(eng, rank, world)
        q.put((rank, ok, eng.imported, eng.ready))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,fail_rank,fail_where", [(2, -1, ""), (3, -1, ""), (2, 1, "export"), (3, 0, "import")])
def test_exchange_setup_agreement(world, fail_rank, fail_where):
    """ksched.dist.setup_exchange (device-side exchange of the persistent pipeline): the ranks'
    IPC handles are all-gathered in rank order, and every rank reports the same outcome -- one
    rank failing to export or map makes ALL ranks fall back together (bench.py relies on it)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_xchg_worker, args=(r, world, port, fail_rank, fail_where, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (ok, imp, ready)) for r, ok, imp, ready in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=30)
    oks = {ok for ok, _, _ in res.values()}
    assert oks == {fail_rank < 0}, res
    # a rank whose import succeeded while a peer failed has closed its exchange again (ksched_xchg_close)
    assert {ready for _, _, ready in res.values()} == {fail_rank < 0}, res
    if fail_rank < 0:
        for r in range(world):
            assert res[r][1] == [bytes([k]) * 64 for k in range(world)]
