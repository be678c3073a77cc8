"""Full-size BASELINE configurations on the GPU (the headline config had never been
checked).  At 1M pods x 100k nodes the CPU oracle cannot replay every pod in test time, so each
configuration is pinned three ways:
  - a prefix of >= 20k pods at the FULL node count against the (OpenMP) oracle -- pods resolve in order,
    so the first k results of the full run are the results of a k-pod run;
  - the two independent GPU paths (persistent exact kernel vs the speculative batched pipeline at the
    bench's K16/B64) bit-equal over ALL pods;
  - conservation: final node state == initial - sum of the committed requests (+1 pod each).
"""
import numpy as np
import pytest

from test_gpu_parity import assert_same, run_engine

pytestmark = pytest.mark.gpu


def conservation(cl, oi, final):
    placed = oi >= 0
    exp_c, exp_m, exp_p = cl.node_state()
    np.subtract.at(exp_c, oi[placed], cl.req_cpu[placed])
    np.subtract.at(exp_m, oi[placed], cl.req_mem[placed])
    np.subtract.at(exp_p, oi[placed], 1)
    assert np.array_equal(final[0], exp_c) and np.array_equal(final[1], exp_m) and np.array_equal(final[2], exp_p)


def full_check(cl, oracle_mod, prefix, batched_kw):
    from ksched import MODE_BATCHED, MODE_EXACT
    b = run_engine(cl, MODE_BATCHED, **batched_kw)
    want = oracle_mod.schedule(cl, nthreads=16, n_pods=prefix)
    assert_same((b[0][:prefix], b[1][:prefix], b[2][:prefix], ()), want, f"{cl.name} prefix {prefix} vs oracle")
    a = run_engine(cl, MODE_EXACT)
    assert_same(b, a[:4], f"{cl.name} full batched {batched_kw} vs exact")
    conservation(cl, a[0], a[3])
    placed = a[0] >= 0
    assert (a[1][placed] > 0).all()  # only s > 0 can win (anchor/priorities.go:55-61)
    return a, b


def test_full_size_c4_bench_config(gpu_available, oracle_mod):
    """BASELINE config 4 at full size (1M pending pods x 100k nodes), the bench's exact configuration."""
    from ksched import cluster
    cl = cluster.make_cluster("c4")
    a, b = full_check(cl, oracle_mod, 20000, dict(topk=16, batch=64))
    st = b[4]
    assert st["placed"] == int((a[0] >= 0).sum())
    assert 0.7 < st["placed"] / cl.n_pods < 0.9  # the no-fit regime the bench runs in (~22 % NO_FIT)


def test_full_size_c5(gpu_available, oracle_mod):
    """BASELINE config 5 at full size (500k pods x 200k nodes, labels, feasible-only argmax)."""
    from ksched import cluster
    full_check(cluster.make_cluster("c5"), oracle_mod, 20000, dict(topk=16, batch=64))


def test_full_size_c5_high_conflict(gpu_available, oracle_mod):
    """c5hc: many exhausted lists -- rescued within the batch's budget, the rest truncating the batch and
    re-scored (the machinery the easy configs barely touch); both paths must be exercised."""
    from ksched import cluster
    cl = cluster.make_cluster("c5hc")
    a, b = full_check(cl, oracle_mod, 20000, dict(topk=16, batch=64))
    st = b[4]
    assert st["truncations"] > 0.05 * st["batches"], st
    assert st["rescues"] > st["truncations"], st


@pytest.mark.parametrize("mode", ["exact", "batched"])
def test_full_size_c2(gpu_available, oracle_mod, mode):
    """BASELINE config 2 at full size (10k pods x 5k nodes, best-price, feasible-only): every pod against
    the oracle (5e7 pairs), in the sequential exact mode the config names and in the batched pipeline."""
    from ksched import MODE_BATCHED, MODE_EXACT, cluster
    cl = cluster.make_cluster("c2")
    assert (cl.n_pods, cl.n_nodes) == (10_000, 5_000)
    want = oracle_mod.schedule(cl, nthreads=8)
    if mode == "exact":
        got = run_engine(cl, MODE_EXACT)
    else:
        got = run_engine(cl, MODE_BATCHED, topk=16, batch=64)
    assert_same(got, want, f"c2 full {mode}")
    assert got[4]["pipeline"] == ("exact" if mode == "exact" else "persistent")


def test_full_size_c3_all_pods_vs_oracle(gpu_available, oracle_mod):
    """BASELINE config 3 (100k pods x 50k nodes) through the batched pipeline, every pod against the oracle
    (5e9 pairs, OpenMP)."""
    from ksched import MODE_BATCHED, cluster
    cl = cluster.make_cluster("c3")
    want = oracle_mod.schedule(cl, nthreads=16)
    assert_same(run_engine(cl, MODE_BATCHED, topk=16, batch=64), want, "c3 full batched vs oracle")
