"""The node-sharded multi-rank product path executed on ONE GPU (it had only run with one
rank at offset 0).

RCCL admits one rank per device, so R ranks run as R contexts of this process on GPU 0, one thread
each, joined by an in-process rank group (ksched_group): the per-batch all-gather of the local
candidate lists goes through a shared device ring instead of ncclAllGather, and everything around it
is the RCCL path's code -- global indices at node_offset > 0, the rank merge k_merge<INPUT_REC> over R
rank blocks with their cut flags, the identical commit replay on every rank and the owner-only
write-back of committed rows.  Every rank's outputs must equal the sequential oracle's, and the shards'
final states concatenated must equal the oracle's final state.
"""
import threading

import numpy as np
import pytest

from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


def run_group(cl, R, **kw):
    from ksched import Group, MODE_BATCHED
    from ksched.dist import make_sharded_engine, shard_range
    g = Group(R, device=0)
    engines = []
    for r in range(R):
        eng, _ = make_sharded_engine(cl, r, R, device=0, mode=MODE_BATCHED, group=g, **kw)
        engines.append(eng)
    out = [None] * R
    errs = []

    def work(r):
        try:
            e = engines[r]
            oi, os_, of = e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)
            out[r] = (oi, os_, of, e.read_nodes(), e.stats())
        except Exception as ex:  # surfaced below
            errs.append((r, ex))

    th = [threading.Thread(target=work, args=(r,)) for r in range(R)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    for e in engines:
        e.close()
    g.close()
    assert not errs, errs
    assert all(o is not None for o in out), "a rank did not finish"
    final = tuple(np.concatenate([out[r][3][k] for r in range(R)]) for k in range(3))
    for r in range(R):
        assert shard_range(cl.n_nodes, r, R)[1] - shard_range(cl.n_nodes, r, R)[0] == out[r][3][0].shape[0]
    return out, final


CASES = [("c3", 20000, 1500, 16, 64), ("c5", 30000, 1500, 8, 64), ("c2", 5000, 1500, 4, 32),
         ("c5hc", 40000, 1200, 16, 64)]


@pytest.mark.parametrize("R", [2, 3, 8])
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_rank_group_equals_sequential(gpu_available, oracle_mod, R, case):
    from ksched import cluster
    name, nn, pp, K, B = case
    cl = cluster.make_cluster(name, n_nodes=nn, n_pods=pp)
    want = oracle_mod.schedule(cl, nthreads=8)
    out, final = run_group(cl, R, topk=K, batch=B)
    for r in range(R):
        assert_same(out[r][:3] + ((),), want, f"{name} R={R} rank {r}")
    assert_same((want[0], want[1], want[2], final), want, f"{name} R={R} final state")
    # every rank made the same decisions in the same number of batches
    assert len({(o[4]["batches"], o[4]["truncations"], o[4]["placed"]) for o in out}) == 1


@pytest.mark.parametrize("R", [2, 4, 8])
def test_rank_group_c4_full_nodes(gpu_available, oracle_mod, R):
    """c4 node-sharded at the FULL 100k nodes (R = 2, 4, 8: BASELINE's 2/4/8-GPU splits, 50k / 25k / 12.5k per
    rank), a 5k-pod prefix against the sequential oracle, final state included."""
    from ksched import cluster
    cl = cluster.make_cluster("c4", n_pods=5000)
    assert cl.n_nodes == 100_000
    want = oracle_mod.schedule(cl, nthreads=16)
    out, final = run_group(cl, R, topk=16, batch=64)
    for r in range(R):
        assert_same(out[r][:3] + ((),), want, f"c4 R={R} rank {r}")
    assert_same((want[0], want[1], want[2], final), want, f"c4 R={R} final state")


@pytest.mark.parametrize("seed", range(4))
def test_rank_group_edge_clusters(gpu_available, oracle_mod, seed):
    """Adversarial small clusters (negative / zero allocatable, 2^53+ values, ties, labels, best price)
    split over 3 ranks: rank blocks with short, cut and empty lists."""
    from ksched import cluster
    combos = [(0, 0, False), (0, 1, True), (1, 1, False), (1, 1, True)]
    pr, dm, lb = combos[seed]
    cl = cluster.random_small(900 + seed, n_nodes=300 + 97 * seed, n_pods=500, priority=pr, domain=dm, use_labels=lb)
    want = oracle_mod.schedule(cl)
    out, final = run_group(cl, 3, topk=8, batch=64)
    for r in range(3):
        assert_same(out[r][:3] + ((),), want, f"edge{seed} rank {r}")
    assert_same((want[0], want[1], want[2], final), want, f"edge{seed} final state")


def test_one_rank_at_node_offset(gpu_available, oracle_mod):
    """A single rank owning nodes [lo, hi) of a larger cluster: its indices are global (offset by lo)
    and the write-back maps them back to local rows."""
    from ksched import Engine, MODE_BATCHED, cluster
    full = cluster.make_cluster("c3", n_nodes=30000, n_pods=1500)
    lo, hi = 12000, 27000
    shard = cluster.Cluster(name="shard", alloc_cpu=full.alloc_cpu[lo:hi].copy(), alloc_mem=full.alloc_mem[lo:hi].copy(),
                            alloc_pods=full.alloc_pods[lo:hi].copy(), req_cpu=full.req_cpu, req_mem=full.req_mem,
                            req_pods=full.req_pods)
    want = oracle_mod.schedule(shard, nthreads=8)
    wi = np.where(want[0] >= 0, want[0] + lo, want[0]).astype(np.int32)
    for kw in (dict(topk=16, batch=64), dict(topk=8, batch=128)):
        with Engine(mode=MODE_BATCHED, node_offset=lo, nodes_global=full.n_nodes, **kw) as e:
            e.load_nodes(shard.alloc_cpu, shard.alloc_mem, shard.alloc_pods)
            oi, os_, of = e.schedule(shard.req_cpu, shard.req_mem, shard.req_pods)
            st = e.read_nodes()
        assert_same((oi, os_, of, st), (wi, want[1], want[2], want[3]), f"offset {lo} {kw}")


def test_rank_group_c5_full_nodes_r8(gpu_available, oracle_mod):
    """c5 -- BASELINE's 8-GPU config: 200k heterogeneous near-full nodes, label bitsets, feasible-only argmax --
    at its FULL node count split over R = 8 ranks (25k nodes each), a 5k-pod prefix against the oracle."""
    from ksched import cluster
    cl = cluster.make_cluster("c5", n_pods=5000)
    assert cl.n_nodes == 200_000 and cl.use_labels
    want = oracle_mod.schedule(cl, nthreads=16)
    out, final = run_group(cl, 8, topk=16, batch=64)
    for r in range(8):
        assert_same(out[r][:3] + ((),), want, f"c5 R=8 rank {r}")
    assert_same((want[0], want[1], want[2], final), want, "c5 R=8 final state")
