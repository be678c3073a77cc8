"""FailedScheduling diagnostics of a whole batch on the device.

For every NO_FIT pod of a schedule call, the reference's failures list is evaluated against the
cluster state that pod saw at its turn (anchor/predicate.go:127-173, after the placements of every
earlier pod, anchor/schedule.go:185-197).  ksched_explain_batch reconstructs those states from the
call's placements on the device; the oracle replays the call pod by pod (or_schedule_reasons)."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def run(cl, mode, **kw):
    from ksched import Engine
    e = Engine(mode=mode, priority=cl.priority, domain=cl.domain, use_labels=cl.use_labels, **kw)
    e.load_nodes(cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods, labels=cl.labels, price=cl.price)
    res = e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)
    return e, res


def check_against_oracle(cl, oracle_mod, mode, **kw):
    wi, ws, wf, wc, _ = oracle_mod.schedule_reasons(cl)
    e, (oi, _, _) = run(cl, mode, **kw)
    try:
        assert np.array_equal(oi, wi)
        cnt, nf = e.explain_batch()
        fails = np.nonzero(wi == -1)[0]
        assert nf == fails.size
        assert np.array_equal(cnt[fails], wc[fails]), "NO_FIT pod histograms differ from the oracle"
        assert not cnt[wi != -1].any()
        # the per-node list of a few of them (the event's "fit failure on node" lines)
        for i in fails[:: max(1, fails.size // 7)]:
            c1, rs = e.explain_pod(int(i))
            assert np.array_equal(c1, wc[i])
        return fails.size
    finally:
        e.close()


@pytest.mark.parametrize("mode_kw", [(0, {}), (1, dict(topk=16, batch=64)), (1, dict(topk=8, batch=128))],
                         ids=["exact", "b16_64", "b8_128"])
def test_explain_batch_matches_oracle(gpu_available, oracle_mod, mode_kw):
    from ksched import cluster
    mode, kw = mode_kw
    # c5hc prefix: near-full nodes, labels, many NO_FIT pods late in the call
    cl = cluster.make_cluster("c5hc", n_nodes=2000, n_pods=6000)
    assert check_against_oracle(cl, oracle_mod, mode, **kw) > 1000
    # adversarial: negative / zero / 2^53+ allocatables, wrapping requests
    for seed in range(3):
        cl = cluster.random_small(70 + seed, n_nodes=211, n_pods=600, domain=1, use_labels=seed % 2 == 1)
        check_against_oracle(cl, oracle_mod, mode, **kw)


def test_explain_state_rules(gpu_available):
    """Valid only while the call's placements are the last state change (KSCHED_E_STATE after)."""
    from ksched import KschedError, MODE_BATCHED, cluster
    cl = cluster.make_cluster("c5hc", n_nodes=2000, n_pods=500)
    e, _ = run(cl, MODE_BATCHED, topk=16, batch=64)
    try:
        e.explain_batch()
        e.apply_delta([0], [0], [0], [0])
        with pytest.raises(KschedError):
            e.explain_batch()
    finally:
        e.close()


def test_explain_batch_full_c4(gpu_available, oracle_mod):
    """BASELINE c4 (1M pods x 100k nodes, ~220k NO_FIT pods): every NO_FIT pod explained in < 1 s.
    Each histogram covers every node and has no fitting node; sampled pods are checked against the
    oracle's node_reasons on the state at their turn, rebuilt on the host from the GPU's placements."""
    from ksched import MODE_BATCHED, cluster
    cl = cluster.make_cluster("c4")
    e, (oi, _, _) = run(cl, MODE_BATCHED, topk=16, batch=64)
    try:
        final = e.read_nodes()
        e.sync()
        t0 = time.perf_counter()
        cnt, nf = e.explain_batch()
        dt = time.perf_counter() - t0
        fails = np.nonzero(oi == -1)[0]
        assert nf == fails.size > 100000
        assert dt < 1.0, f"explain_batch took {dt:.2f} s"
        assert (cnt[fails].sum(1) == cl.n_nodes).all() and (cnt[fails, 0] == 0).all()
        rng = np.random.default_rng(3)
        for i in rng.choice(fails, 12, replace=False):
            after = np.arange(cl.n_pods) > i
            placed = after & (oi >= 0)
            st = [final[0].copy(), final[1].copy(), final[2].copy()]
            np.add.at(st[0], oi[placed], cl.req_cpu[placed])
            np.add.at(st[1], oi[placed], cl.req_mem[placed])
            np.add.at(st[2], oi[placed], 1)
            wc, _ = oracle_mod.node_reasons(cl, st, cl.req_cpu[i], cl.req_mem[i], cl.req_pods[i])
            assert np.array_equal(cnt[i], wc), f"pod {i}"
    finally:
        e.close()
