"""GPU parity: libksched (HIP, gfx950) against the CPU oracle, bit-exact.

Every test goes through the C-ABI (ctypes -> libksched.so -> HIP kernels); there is no CPU fallback.
Outputs compared: node index per pod (exact), score bits (exact: 0 ulp, stricter than the
north_star's 1e-6 relative), feasible count per pod (exact) and the final node state (exact).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

MODES = None


def modes():
    from ksched import MODE_BATCHED, MODE_EXACT
    return [("exact", MODE_EXACT, {}), ("batched_k4", MODE_BATCHED, dict(topk=4, batch=32)),
            ("batched_k8", MODE_BATCHED, dict(topk=8, batch=64)), ("batched_k16", MODE_BATCHED, dict(topk=16, batch=128)),
            ("batched_k16_b64", MODE_BATCHED, dict(topk=16, batch=64)),
            ("batched_k16_b64_c2", MODE_BATCHED, dict(topk=16, batch=64, chunk_topk=2)),
            ("batched_k8_b128_c8", MODE_BATCHED, dict(topk=8, batch=128, chunk_topk=8)),
            ("batched_k8_b48_seq", MODE_BATCHED, dict(topk=8, batch=48, commit_impl=1))]


def run_engine(cl, mode, **kw):
    from ksched import Engine
    with Engine(mode=mode, priority=cl.priority, domain=cl.domain, use_labels=cl.use_labels, **kw) as e:
        e.load_nodes(cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods, labels=cl.labels, price=cl.price)
        oi, os_, of = e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)
        st = e.read_nodes()
        stats = e.stats()
    return oi, os_, of, st, stats


def assert_same(got, want, label=""):
    oi, os_, of, st = got[:4]
    wi, ws, wf, wst = want[:4]
    bad = np.nonzero(oi != wi)[0]
    assert bad.size == 0, f"{label}: first idx mismatch at pod {bad[:5]}: got {oi[bad[:5]]} want {wi[bad[:5]]}"
    sb = np.nonzero(os_.view(np.int64) != ws.view(np.int64))[0]
    assert sb.size == 0, f"{label}: score bits differ at {sb[:5]}: {os_[sb[:5]]} vs {ws[sb[:5]]}"
    fb = np.nonzero(of != wf)[0]
    assert fb.size == 0, f"{label}: feasible count differs at {fb[:5]}: {of[fb[:5]]} vs {wf[fb[:5]]}"
    for a, b in zip(st, wst):
        assert np.array_equal(a, b), f"{label}: final node state differs"


def check_same(cl, mode, want, label, **kw):
    """run_engine + assert_same; on a mismatch the case runs twice more -- as is, and with the commit's touched-node
    screen off (KSCHED_NO_TOUCH_SCREEN=1) -- and the message says which of those matched (a rare mismatch then
    names its cause: one that does not repeat, or the screen)."""
    got = run_engine(cl, mode, **kw)
    try:
        assert_same(got, want, label)
    except AssertionError as ex:
        again = run_engine(cl, mode, **kw)
        os.environ["KSCHED_NO_TOUCH_SCREEN"] = "1"
        try:
            off = run_engine(cl, mode, **kw)
        finally:
            del os.environ["KSCHED_NO_TOUCH_SCREEN"]
        same = lambda g: bool(np.array_equal(g[0], want[0]))  # noqa: E731
        raise AssertionError(f"{ex} | stats {got[4]} | again: matches {same(again)}, screen off: matches {same(off)}")


def golden():
    with open(os.path.join(GOLDEN, "clusters.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("mi", range(8), ids=["exact", "b4", "b8", "b16", "b16_64", "b16_64_c2", "b8_128_c8",
                                             "b8_48_seq"])
def test_golden_clusters(gpu_available, mi):
    from test_oracle import _cluster_from
    name, mode, kw = modes()[mi]
    for fx in golden():
        cl = _cluster_from(fx)
        got = run_engine(cl, mode, **kw)
        want = (np.array(fx["expect_idx"], np.int32),
                np.array([float.fromhex(x) for x in fx["expect_score_hex"]], np.float64),
                np.array(fx["expect_feasible"], np.int32), [np.array(x, np.int64) for x in fx["expect_final"]])
        assert_same(got, want, f"{fx['name']}/{name}")


def test_readme_demo_best_price(gpu_available):
    from ksched import MODE_EXACT, cluster
    cl = cluster.readme_demo()
    oi, os_, of, _, _ = run_engine(cl, MODE_EXACT)
    assert oi.tolist() == [3] and os_[0] == np.float32(0.05) and of.tolist() == [6]


@pytest.mark.parametrize("seed", range(12))
def test_edge_clusters_all_modes(gpu_available, oracle_mod, seed):
    from ksched import cluster
    combos = [(0, 0, False), (0, 1, False), (1, 1, False), (0, 1, True), (1, 1, True), (0, 0, True)]
    pr, dm, lb = combos[seed % 6]
    cl = cluster.random_small(500 + seed, n_nodes=37 + 61 * seed, n_pods=700, priority=pr, domain=dm, use_labels=lb)
    want = oracle_mod.schedule(cl)
    for name, mode, kw in modes():
        check_same(cl, mode, want, f"seed{seed}/{name}", **kw)


@pytest.mark.parametrize("name,nn,pp", [("c2", 5000, 2000), ("c3", 20000, 1500), ("c5", 30000, 1500)])
def test_config_prefix_parity(gpu_available, oracle_mod, name, nn, pp):
    from ksched import cluster
    cl = cluster.make_cluster(name, n_nodes=nn, n_pods=pp)
    want = oracle_mod.schedule(cl, nthreads=8)
    for mname, mode, kw in modes():
        check_same(cl, mode, want, f"{name}/{mname}", **kw)


@pytest.mark.parametrize("kc", [2, 4, 16])
def test_tie_storm_chunk_cut(gpu_available, oracle_mod, kc):
    """Identical nodes and identical pods: every key ties and ranks by node index, so the merged list's
    exact prefix depends entirely on the strided chunking + cut rule; zero-request pods mixed in."""
    from ksched import MODE_BATCHED, cluster
    n, p = 3000, 900
    cl = cluster.Cluster(name="ties", alloc_cpu=np.full(n, 4000, np.int64), alloc_mem=np.full(n, 8388608, np.int64),
                         alloc_pods=np.full(n, 110, np.int64), req_cpu=np.where(np.arange(p) % 3 == 0, 0, 200).astype(np.int64),
                         req_mem=np.where(np.arange(p) % 3 == 0, 0, 65536).astype(np.int64), req_pods=np.ones(p, np.int64))
    want = oracle_mod.schedule(cl)
    for b, impl in ((64, 0), (64, 1), (128, 0)):
        assert_same(run_engine(cl, MODE_BATCHED, topk=16, batch=b, chunk_topk=kc, commit_impl=impl), want,
                    f"ties kc={kc} b={b} impl={impl}")


def test_exact_mode_workgroup_counts(gpu_available, oracle_mod):
    """Exact mode with 1..many workgroups (cross-workgroup granule exchange) gives identical results."""
    from ksched import MODE_EXACT, cluster
    cl = cluster.make_cluster("c3", n_nodes=6000, n_pods=600)
    want = oracle_mod.schedule(cl, nthreads=8)
    for g in (1, 2, 3, 7, 24, 64, 200):
        if 6000 > g * 256 * 8:
            continue
        assert_same(run_engine(cl, MODE_EXACT, exact_wgs=g), want, f"G={g}")


@pytest.mark.parametrize("case", ["c2", "c2_16k", "c3_4k", "c5_3k", "edge_res", "edge_price", "ties_price"])
def test_exact_one_workgroup(gpu_available, oracle_mod, case):
    """Exact mode on ONE workgroup (k_exact1: every node in a register slot of one 1024-thread workgroup, one
    barrier per pod; best-price as the first feasible node in (price, index) order): bit-exact against the oracle,
    and equal to the multi-workgroup exchange kernel where that one fits."""
    from ksched import MODE_EXACT, cluster
    if case == "c2":
        cl = cluster.make_cluster("c2", n_pods=2000)
    elif case == "c2_16k":
        cl = cluster.make_cluster("c2", n_nodes=16000, n_pods=600)
    elif case == "c3_4k":
        cl = cluster.make_cluster("c3", n_nodes=4000, n_pods=800)
    elif case == "c5_3k":
        cl = cluster.make_cluster("c5", n_nodes=3000, n_pods=800)
    elif case == "edge_res":
        cl = cluster.random_small(31, n_nodes=900, n_pods=700)
    elif case == "edge_price":
        cl = cluster.random_small(32, n_nodes=900, n_pods=700, priority=cluster.PRIORITY_BEST_PRICE,
                                  domain=cluster.DOMAIN_FEASIBLE, use_labels=True)
    else:  # every node the same price: the lowest index wins each time
        cl = cluster.make_cluster("c2", n_nodes=3000, n_pods=900)
        cl.price = np.full(cl.n_nodes, 0.5, np.float32)
        cl.price[::7] = -0.0  # "-0" is "0": ties with the zero-priced nodes by index
        cl.price[::11] = 0.0
    want = oracle_mod.schedule(cl, nthreads=8)
    got = run_engine(cl, MODE_EXACT)
    assert_same(got, want, f"{case} one workgroup")
    assert got[4]["pipeline"] == "exact"
    if cl.n_nodes <= 2 * 256 * 8:
        assert_same(run_engine(cl, MODE_EXACT, exact_wgs=2), want, f"{case} two workgroups")


def test_apply_delta_and_state_roundtrip(gpu_available, oracle_mod):
    from ksched import Engine, MODE_EXACT, cluster
    cl = cluster.make_cluster("c3", n_nodes=2000, n_pods=300)
    with Engine(mode=MODE_EXACT, priority=cl.priority, domain=cl.domain) as e:
        e.load_nodes(cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods)
        e.save_state()
        idx = np.array([5, 7, 5, 1999], np.int32)
        d = np.array([100, -50, 25, 1 << 40], np.int64)
        e.apply_delta(idx, d, d * 3, -np.ones(4, np.int64))
        ac, am, ap = e.read_nodes()
        exp_c = cl.alloc_cpu.copy(); exp_m = cl.alloc_mem.copy(); exp_p = cl.alloc_pods.copy()
        for i, x in zip(idx, d):
            exp_c[i] += x; exp_m[i] += 3 * x; exp_p[i] -= 1
        assert np.array_equal(ac, exp_c) and np.array_equal(am, exp_m) and np.array_equal(ap, exp_p)
        e.restore_state()
        ac, am, ap = e.read_nodes()
        assert np.array_equal(ac, cl.alloc_cpu)
        got1 = e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods)
        e.restore_state()
        got2 = e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods)
        want = oracle_mod.schedule(cl)
        for g in (got1, got2):
            assert np.array_equal(g[0], want[0]) and np.array_equal(g[1].view(np.int64), want[1].view(np.int64))


def test_host_mirror_fake_cluster(gpu_available, oracle_mod):
    """schedulePods through the k8s-shaped mirror: packing, engine, ordered binds."""
    from ksched import cluster
    from ksched.host import Container, FakeCluster, FitError, Node, Pod
    cl = cluster.make_cluster("c3", n_nodes=200, n_pods=400, with_strings=True)
    nodes = [Node(nm, cap) for nm, cap in zip(cl.node_names, cl.node_capacity)]
    bound = [Pod(f"b{i}", [Container(requests=r) for r in conts], node_name=nm)
             for i, (nm, conts) in enumerate(cl.bound_pods)]
    pend = [Pod(f"p{i}", [Container(requests=r) for r in conts]) for i, conts in enumerate(cl.pending_pods)]
    fc = FakeCluster(nodes, bound + pend, priority=cl.priority, domain=cl.domain)
    assert fc.schedule_pods() == []  # none carries the scheduler annotation (anchor/schedule.go:176)
    res = fc.schedule_pods(pend)
    want = oracle_mod.schedule(cl)
    for (pod, r), wi in zip(res, want[0]):
        if wi >= 0:
            assert r.name == cl.node_names[wi] and pod.node_name == r.name
        else:
            assert isinstance(r, Exception)
    # a pod that fits nowhere raises the reference's fit error
    huge = Pod("huge", [Container(requests=dict(cpu="100000000m"))])
    with pytest.raises(FitError):
        fc.schedule_pod(huge)


def test_full_size_c3_batched_equals_exact(gpu_available):
    """Size-independent property at BASELINE size (100k pods x 50k nodes): the two independent GPU
    paths (persistent exact kernel vs speculative batched kernels) agree bit for bit, and the final
    node state equals the initial state minus the committed requests (conservation)."""
    from ksched import MODE_BATCHED, MODE_EXACT, cluster
    cl = cluster.make_cluster("c3")
    a = run_engine(cl, MODE_EXACT)
    for kw in (dict(topk=16, batch=128), dict(topk=16, batch=64), dict(topk=8, batch=32),
               dict(topk=16, batch=64, commit_impl=1)):
        b = run_engine(cl, MODE_BATCHED, **kw)
        assert_same(b, a[:4], f"c3 full exact-vs-batched {kw}")
    oi = a[0]
    placed = oi >= 0
    exp_c = cl.alloc_cpu.copy(); exp_m = cl.alloc_mem.copy(); exp_p = cl.alloc_pods.copy()
    np.subtract.at(exp_c, oi[placed], cl.req_cpu[placed])
    np.subtract.at(exp_m, oi[placed], cl.req_mem[placed])
    np.subtract.at(exp_p, oi[placed], 1)
    assert np.array_equal(a[3][0], exp_c) and np.array_equal(a[3][1], exp_m) and np.array_equal(a[3][2], exp_p)
    # the committed pods' recorded scores are positive (only s > 0 can win)
    assert (a[1][placed] > 0).all()


def test_hoisted_reciprocal_division_is_bit_exact(gpu_available):
    """qdiv(a, b, recip(b)) == hipcc's a / b, bit for bit, over the operand classes of the score:
    integer-valued numerators/divisors across magnitudes and signs (incl. > 2^53 and near 2^63),
    the /3 of sums of fractions and of squared deviations, and the *10 least-requested numerators."""
    import ctypes as C
    from ksched import Engine
    from ksched import _lib as L
    rng = np.random.default_rng(11)
    n = 1 << 21
    mags = rng.integers(0, 63, size=n)
    ai = (rng.integers(0, 1 << 62, size=n, dtype=np.int64) >> (62 - np.minimum(mags, 62))).astype(np.int64)
    ai[rng.random(n) < 0.3] *= -1
    bi = (rng.integers(1, 1 << 62, size=n, dtype=np.int64) >> (62 - np.minimum(rng.integers(0, 63, size=n), 62))).astype(np.int64)
    bi[bi == 0] = 1
    bi[rng.random(n) < 0.3] *= -1
    a = ai.astype(np.float64)
    b = bi.astype(np.float64)
    # fraction-like numerators over 3.0
    k = n // 4
    fr = (rng.integers(1, 1 << 40, size=k) / rng.integers(1, 1 << 50, size=k).astype(np.float64))
    a[:k] = fr + fr[::-1] + (fr * fr)
    b[:k] = 3.0
    # tiny squared deviations over 3.0
    a[k:2 * k] = (fr - fr[::-1]) ** 2
    b[k:2 * k] = 3.0
    # least-requested numerators: (cap - req) * 10 over cap
    cap = rng.integers(1, 1 << 45, size=k).astype(np.int64)
    req = rng.integers(0, 1 << 45, size=k).astype(np.int64) % cap
    a[2 * k:3 * k] = (cap - req).astype(np.float64) * 10.0
    b[2 * k:3 * k] = cap.astype(np.float64)
    native = np.empty(n); fast = np.empty(n)
    with Engine() as e:
        rc = L.lib().ksched_selftest_fastdiv(e._ctx, n, L.ptr(a, C.c_double), L.ptr(b, C.c_double),
                                             L.ptr(native, C.c_double), L.ptr(fast, C.c_double))
        assert rc == 0
    # nonzero numerators: identical bits; zero numerators: identical value (signed zero may differ,
    # and never reaches a score -- DESIGN.md)
    nz = a != 0
    bad = np.nonzero(native[nz].view(np.int64) != fast[nz].view(np.int64))[0]
    assert bad.size == 0, f"{bad.size} mismatches, e.g. {a[nz][bad[:3]]}/{b[nz][bad[:3]]}"
    assert np.array_equal(native[~nz], fast[~nz])
    # and both equal the correctly rounded CPU quotient
    assert np.array_equal(native[nz].view(np.int64), (a[nz] / b[nz]).view(np.int64))


def test_collective_path_one_rank(gpu_available, oracle_mod):
    """The node-sharded path (RCCL all-gather of the local candidate records + rank merge) on a 1-rank
    communicator: same bits as the oracle.  Exercises ksched_get_unique_id / ksched_set_comm,
    ncclAllGather inside the engine and k_merge<INPUT_REC>."""
    from ksched import Engine, MODE_BATCHED, cluster
    for name, nn, pp, K in (("c3", 20000, 1500, 16), ("c5", 30000, 1500, 8), ("c2", 5000, 1500, 4)):
        cl = cluster.make_cluster(name, n_nodes=nn, n_pods=pp)
        want = oracle_mod.schedule(cl, nthreads=8)
        with Engine(mode=MODE_BATCHED, priority=cl.priority, domain=cl.domain, use_labels=cl.use_labels,
                    topk=K, batch=8 * K, nranks=1, nodes_global=cl.n_nodes) as e:
            e.set_comm(Engine.unique_id())
            e.load_nodes(cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods, labels=cl.labels, price=cl.price)
            oi, os_, of = e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)
            st = e.read_nodes()
        assert_same((oi, os_, of, st), want, f"{name}/collective")


def test_sharded_engine_helper_world1(gpu_available, oracle_mod):
    from ksched import cluster
    from ksched.dist import make_sharded_engine
    cl = cluster.make_cluster("c3", n_nodes=8000, n_pods=800)
    eng, (lo, hi) = make_sharded_engine(cl, 0, 1, device=0, topk=8, batch=64)
    assert (lo, hi) == (0, 8000)
    oi, os_, of = eng.schedule(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)
    st = eng.read_nodes()
    eng.close()
    assert_same((oi, os_, of, st), oracle_mod.schedule(cl), "sharded-helper")


def test_stream_pipeline_parity(gpu_available, oracle_mod):
    """The stream pipeline (per-batch score / merge / commit launches: the RCCL and rank-group multi-rank
    path, and the single-rank fallback where the persistent kernel does not fit) stays bit-exact;
    opts.pipeline = KSCHED_PIPELINE_STREAM selects it."""
    from ksched import MODE_BATCHED, cluster
    from ksched._lib import PIPELINE_STREAM
    for name, nn, pp in (("c3", 30000, 2000), ("c5", 40000, 1500), ("c5hc", 20000, 3000)):
        cl = cluster.make_cluster(name, n_nodes=nn, n_pods=pp)
        want = oracle_mod.schedule(cl, nthreads=8)
        for kw in (dict(topk=16, batch=64), dict(topk=8, batch=32, chunk_topk=2), dict(topk=16, batch=128)):
            got = run_engine(cl, MODE_BATCHED, pipeline=PIPELINE_STREAM, **kw)
            assert_same(got, want, f"{name}/stream/{kw}")
            assert got[4]["pipeline"] in ("stream", "stream-sequential"), got[4]


@pytest.mark.parametrize("name,nn,pp", [("c3", 30000, 2000), ("c5", 40000, 1500), ("c5hc", 20000, 3000),
                                         ("c2", 5000, 2000), ("c1", 700, 300)])
def test_persistent_pipeline_parity(gpu_available, oracle_mod, name, nn, pp):
    """The default batched path is the persistent pipeline (ksched_pipe.hip: ONE cooperative kernel, the
    commit workgroup + up to CUs - 1 score workgroups whose merge waves merge one pod each); the stats say
    it ran, and it is bit-exact at every (topk, batch, chunk_topk) it accepts -- including the grid sizes
    where the score workgroups outnumber the batch (workgroups without a pod to merge run ahead) and
    small grids where one workgroup merges several pods of a batch (pipe_wgs)."""
    from ksched import MODE_BATCHED, cluster
    cl = cluster.make_cluster(name, n_nodes=nn, n_pods=pp)
    want = oracle_mod.schedule(cl, nthreads=8)
    for kw in (dict(topk=16, batch=64), dict(topk=8, batch=64, chunk_topk=8), dict(topk=4, batch=32, chunk_topk=4),
               dict(topk=16, batch=16), dict(topk=16, batch=64, pipe_wgs=66)):
        got = run_engine(cl, MODE_BATCHED, **kw)
        assert_same(got, want, f"{name}/{kw}")
        assert got[4]["pipeline"] == "persistent", got[4]


@pytest.mark.parametrize("policy", ["none", "fixed4", "bucket", "scarce", "look"])
def test_rescue_policies_same_results(gpu_available, oracle_mod, monkeypatch, policy):
    """The rescue policy (KSCHED_RESCUE_*, DESIGN 4.1: truncate always, a fixed budget per batch, the default
    credit bucket, a scarce bucket, the look-ahead) decides only whether an exhausted candidate list is rescued
    or truncates its batch -- never a result: every policy is bit-exact against the oracle on a high-conflict
    cluster with short lists, and the counters show which path ran."""
    from ksched import MODE_BATCHED, cluster
    env = {"none": dict(KSCHED_RESCUE_MAX="0"),
           "fixed4": dict(KSCHED_RESCUE_MAX="4", KSCHED_RESCUE_RATE="16", KSCHED_RESCUE_CAP="4", KSCHED_RESCUE_LOW="4"),
           "bucket": {},
           "scarce": dict(KSCHED_RESCUE_MAX="2", KSCHED_RESCUE_RATE="1", KSCHED_RESCUE_CAP="2", KSCHED_RESCUE_LOW="1"),
           "look": dict(KSCHED_RESCUE_LOOK="1")}[policy]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cl = cluster.make_cluster("c5hc", n_nodes=20000, n_pods=3000)
    want = oracle_mod.schedule(cl, nthreads=8)
    got = run_engine(cl, MODE_BATCHED, topk=4, batch=64, chunk_topk=4)
    assert_same(got, want, f"c5hc/{policy}")
    st = got[4]
    print(f"{policy}: batches {st['batches']} truncations {st['truncations']} rescues {st['rescues']}")
    assert st["pipeline"] == "persistent", st
    if policy == "none":
        assert st["rescues"] == 0 and st["truncations"] > 0, st
    else:
        assert st["rescues"] > 0, st
