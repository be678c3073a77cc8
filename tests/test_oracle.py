"""CPU tests of the oracle itself: pinned to the known-answer tests and the committed golden vectors,
C and pure-Python restatements cross-checked, batched restatement == sequential semantics."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN


def _load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_parse_vectors_c_oracle(oracle_mod):
    for v in _load("parse_vectors.json"):
        try:
            got = oracle_mod.parse(v["kind"], v["s"])
        except ValueError:
            got = "fatal"
        assert got == v["value"], v


def test_parse_vectors_py_oracle():
    import ref_py as R
    fns = {"cpu": R.parse_cpu, "memory": R.parse_memory, "pods": R.parse_pods}
    for v in _load("parse_vectors.json"):
        s = v["s"]
        try:
            got = fns[v["kind"]](s)
        except R.Fatal:
            got = "fatal"
        assert got == v["value"], v


def test_survey_cpu_quirks(oracle_mod):
    # CPU decimals parse through float32
    for s, want in [("0.7", 699), ("2.3", 2299), ("3.3", 3299), ("0.35", 349), ("0.1", 100), ("0.0015", 1)]:
        assert oracle_mod.parse("cpu", s) == want
    assert oracle_mod.parse("memory", "1Gi") == 0  # only Ki / Mi are understood
    assert oracle_mod.parse("memory", "64Mi") == 65536


def test_score_kats(oracle_mod):
    import ref_py as R
    for k in _load("score_kats.json"):
        s = oracle_mod.score(*k["req"], *k["alloc"])
        assert float(s).hex() == k["score_hex"]
        assert s == R.score(*k["req"], *k["alloc"])
        assert abs(s - k["score"]) <= 1e-12 * max(1.0, abs(k["score"]))


def _cluster_from(fx):
    from ksched.cluster import Cluster
    cl = Cluster(name=fx["name"], alloc_cpu=np.array(fx["alloc_cpu"], np.int64),
                 alloc_mem=np.array(fx["alloc_mem"], np.int64), alloc_pods=np.array(fx["alloc_pods"], np.int64),
                 req_cpu=np.array(fx["req_cpu"], np.int64), req_mem=np.array(fx["req_mem"], np.int64),
                 req_pods=np.array(fx["req_pods"], np.int64), priority=fx["priority"], domain=fx["domain"],
                 use_labels=fx["use_labels"])
    if fx["labels"] is not None:
        cl.labels = np.array(fx["labels"], dtype=np.uint64)
    if fx["selector"] is not None:
        cl.selector = np.array(fx["selector"], dtype=np.uint64)
    if fx["price"] is not None:
        cl.price = np.array(fx["price"], dtype=np.float32)
    return cl


def golden_clusters():
    return [(fx["name"], fx) for fx in _load("clusters.json")]


@pytest.mark.parametrize("name,fx", golden_clusters(), ids=[n for n, _ in golden_clusters()])
def test_golden_cluster_c_oracle(oracle_mod, name, fx):
    cl = _cluster_from(fx)
    oi, os_, of, st = oracle_mod.schedule(cl)
    assert oi.tolist() == fx["expect_idx"]
    assert [float(x).hex() for x in os_] == fx["expect_score_hex"]
    assert of.tolist() == fx["expect_feasible"]
    assert [s.tolist() for s in st] == fx["expect_final"]


def test_readme_kat(oracle_mod):
    """README.md:43-58: the nginx pod (cpu 200m) lands on ...-pxee, the cheapest node (0.05)."""
    from ksched import cluster
    cl = cluster.readme_demo()
    oi, os_, of, _ = oracle_mod.schedule(cl)
    assert oi.tolist() == [3]
    assert cl.node_names[3].endswith("pxee")
    assert os_[0] == np.float32(0.05)
    assert of.tolist() == [6]


@pytest.mark.parametrize("name,nn,pp,K,B", [("c2", 800, 600, 4, 32), ("c3", 1500, 500, 8, 64),
                                            ("c5", 2000, 600, 16, 128), ("c3", 700, 300, 4, 256)])
def test_batched_restatement_equals_sequential(oracle_mod, name, nn, pp, K, B):
    from ksched import cluster
    cl = cluster.make_cluster(name, n_nodes=nn, n_pods=pp)
    oi, os_, of, st = oracle_mod.schedule(cl)
    bi, bs, bf, bst, stats = oracle_mod.schedule_batched(cl, K, B)
    assert np.array_equal(oi, bi)
    assert np.array_equal(os_.view(np.int64), bs.view(np.int64))
    assert np.array_equal(of, bf)
    for a, b in zip(st, bst):
        assert np.array_equal(a, b)
    assert stats["batches"] >= 1


@pytest.mark.parametrize("seed", range(6))
def test_batched_restatement_edge_clusters(oracle_mod, seed):
    from ksched import cluster
    combos = [(0, 0, False), (0, 1, False), (1, 1, False), (0, 1, True), (1, 1, True), (0, 0, True)]
    pr, dm, lb = combos[seed]
    cl = cluster.random_small(77 + seed, n_nodes=96, n_pods=400, priority=pr, domain=dm, use_labels=lb)
    oi, os_, of, _ = oracle_mod.schedule(cl)
    for K, B in ((4, 16), (8, 64), (16, 400)):
        bi, bs, bf, _, _ = oracle_mod.schedule_batched(cl, K, B)
        assert np.array_equal(oi, bi) and np.array_equal(of, bf)
        assert np.array_equal(os_.view(np.int64), bs.view(np.int64))


def test_openmp_oracle_matches_single_thread(oracle_mod):
    from ksched import cluster
    cl = cluster.make_cluster("c3", n_nodes=3000, n_pods=200)
    a = oracle_mod.schedule(cl, nthreads=1)
    b = oracle_mod.schedule(cl, nthreads=4)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1].view(np.int64), b[1].view(np.int64))


@pytest.mark.parametrize("name,nn,pp,K,B", [("c2", 800, 700, 4, 32), ("c3", 1500, 600, 8, 64),
                                            ("c5", 2000, 700, 16, 128), ("c3", 700, 500, 4, 128)])
def test_pipelined_restatement_equals_sequential(oracle_mod, name, nn, pp, K, B):
    """The GPU pipeline's algorithm (lag-one snapshot, speculative plan, inherited touched set,
    skip + resync on truncation) equals the sequential semantics."""
    from ksched import cluster
    cl = cluster.make_cluster(name, n_nodes=nn, n_pods=pp)
    oi, os_, of, st = oracle_mod.schedule(cl)
    bi, bs, bf, bst, stats = oracle_mod.schedule_pipelined(cl, K, B)
    assert np.array_equal(oi, bi) and np.array_equal(of, bf)
    assert np.array_equal(os_.view(np.int64), bs.view(np.int64))
    for a, b in zip(st, bst):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("seed", range(6))
def test_pipelined_restatement_edge_clusters(oracle_mod, seed):
    from ksched import cluster
    combos = [(0, 0, False), (0, 1, False), (1, 1, False), (0, 1, True), (1, 1, True), (0, 0, True)]
    pr, dm, lb = combos[seed]
    cl = cluster.random_small(91 + seed, n_nodes=96, n_pods=500, priority=pr, domain=dm, use_labels=lb)
    oi, os_, of, st = oracle_mod.schedule(cl)
    for K, B in ((4, 16), (8, 64), (16, 128)):
        bi, bs, bf, bst, stats = oracle_mod.schedule_pipelined(cl, K, B)
        assert np.array_equal(oi, bi) and np.array_equal(of, bf)
        assert np.array_equal(os_.view(np.int64), bs.view(np.int64))
        for a, b in zip(st, bst):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("lag", [2, 3, 4])
@pytest.mark.parametrize("name,nn,pp,K,B", [("c2", 800, 700, 4, 32), ("c3", 1500, 600, 8, 64),
                                            ("c5", 2000, 700, 16, 64), ("c3", 700, 500, 4, 64)])
def test_lagged_restatement_equals_sequential(oracle_mod, name, nn, pp, K, B, lag):
    """The persistent pipeline at lag 2, 3 (the device's) and 4: score(b) against commit(b - lag), commit(b)
    inheriting the exports of b - lag + 1 .. b - 1 with the oldest start state as snapshot state."""
    from ksched import cluster
    cl = cluster.make_cluster(name, n_nodes=nn, n_pods=pp)
    oi, os_, of, st = oracle_mod.schedule(cl)
    bi, bs, bf, bst, stats = oracle_mod.schedule_lagged(cl, K, B, lag)
    assert np.array_equal(oi, bi) and np.array_equal(of, bf)
    assert np.array_equal(os_.view(np.int64), bs.view(np.int64))
    for a, b in zip(st, bst):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("seed", range(6))
def test_lagged_restatement_edge_clusters(oracle_mod, seed):
    """Small adversarial clusters (high conflict: many truncations, skips and re-plans) at lag 3."""
    from ksched import cluster
    combos = [(0, 0, False), (0, 1, False), (1, 1, False), (0, 1, True), (1, 1, True), (0, 0, True)]
    pr, dm, lb = combos[seed]
    cl = cluster.random_small(91 + seed, n_nodes=96, n_pods=500, priority=pr, domain=dm, use_labels=lb)
    oi, os_, of, st = oracle_mod.schedule(cl)
    for K, B in ((4, 16), (8, 64), (16, 64)):
        bi, bs, bf, bst, stats = oracle_mod.schedule_lagged(cl, K, B, 3)
        assert np.array_equal(oi, bi) and np.array_equal(of, bf)
        assert np.array_equal(os_.view(np.int64), bs.view(np.int64))
        for a, b in zip(st, bst):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("lag", [2, 3, 4])
def test_lagged_restatement_skip_accounting(oracle_mod, lag):
    """Each truncation voids up to lag - 1 batches already planned behind it (fewer when the pods run out
    before them), which is why the device's truncations cost more at lag 3."""
    from ksched import cluster
    cl = cluster.random_small(92, n_nodes=96, n_pods=500, priority=0, domain=1, use_labels=False)
    st = oracle_mod.schedule_lagged(cl, 4, 16, lag)[4]
    assert st["truncations"] > 10
    assert st["skipped"] <= (lag - 1) * st["truncations"]
    assert st["skipped"] >= 0.9 * (lag - 1) * st["truncations"]


@pytest.mark.parametrize("seed", range(6))
def test_lagged_rescue_equals_sequential(oracle_mod, seed):
    """The device's rescue of an exhausted candidate list (a full scan of the nodes outside the batch's touched
    set, at their current state) restated at lag 3: the same sequential result with no truncation at all, on
    the high-conflict clusters where the truncating pipeline truncates most."""
    from ksched import cluster
    combos = [(0, 0, False), (0, 1, False), (1, 1, False), (0, 1, True), (1, 1, True), (0, 0, True)]
    pr, dm, lb = combos[seed]
    cl = cluster.random_small(91 + seed, n_nodes=96, n_pods=500, priority=pr, domain=dm, use_labels=lb)
    oi, os_, of, st = oracle_mod.schedule(cl)
    for K, B in ((4, 16), (8, 64), (16, 64)):
        plain = oracle_mod.schedule_lagged(cl, K, B, 3)[4]
        bi, bs, bf, bst, stats = oracle_mod.schedule_lagged(cl, K, B, 3, rescue=True)
        assert np.array_equal(oi, bi) and np.array_equal(of, bf)
        assert np.array_equal(os_.view(np.int64), bs.view(np.int64))
        for a, b in zip(st, bst):
            assert np.array_equal(a, b)
        assert stats["truncations"] == 0 and stats["skipped"] == 0
        assert stats["rescues"] >= plain["truncations"]  # every truncation became a rescue (or more: later batches differ)


def test_lagged_rescue_c4_like(oracle_mod):
    """A c4-shaped cluster (the bench's distribution, fewer nodes): rescue on, still the sequential result."""
    from ksched import cluster
    cl = cluster.make_cluster("c4", n_nodes=2000, n_pods=3000)
    oi, os_, of, st = oracle_mod.schedule(cl)
    bi, bs, bf, bst, stats = oracle_mod.schedule_lagged(cl, 16, 64, 3, rescue=True)
    assert np.array_equal(oi, bi) and np.array_equal(of, bf) and np.array_equal(os_.view(np.int64), bs.view(np.int64))
    assert stats["truncations"] == 0


@pytest.mark.parametrize("seed", range(4))
def test_lagged_rescue_sharded_budgeted_equals_sequential(oracle_mod, seed):
    """The node-sharded rescue (each of R contiguous shards scanned for its best untouched node, the R bests
    folded: the device's per-rank merger scan + rank fold) under the device's per-batch budget: the sequential
    result for every shard count and budget; the shard split changes nothing (a fold of per-shard arg-bests is
    the arg-best), and the budget only trades rescues for truncations."""
    from ksched import cluster
    combos = [(0, 0, False), (0, 1, True), (1, 1, False), (0, 0, True)]
    pr, dm, lb = combos[seed]
    cl = cluster.random_small(191 + seed, n_nodes=97, n_pods=500, priority=pr, domain=dm, use_labels=lb)
    oi, os_, of, st = oracle_mod.schedule(cl)
    for K, B in ((4, 16), (8, 64)):
        seen = {}
        for budget in (0, 1, 4, None):
            for shards in (1, 2, 3, 8):
                bi, bs, bf, bst, stats = oracle_mod.schedule_lagged(cl, K, B, 3, rescue=True, rescue_max=budget,
                                                                    shards=shards)
                assert np.array_equal(oi, bi) and np.array_equal(of, bf)
                assert np.array_equal(os_.view(np.int64), bs.view(np.int64))
                for a, b in zip(st, bst):
                    assert np.array_equal(a, b)
                key = (stats["truncations"], stats["rescues"], stats["batches"])
                assert seen.setdefault(budget, key) == key, "the shard count changed the schedule of rescues"
                if budget == 0:
                    assert stats["rescues"] == 0
                if budget is None:
                    assert stats["truncations"] == 0
        assert seen[0][0] >= seen[1][0] >= seen[4][0] >= seen[None][0] == 0
