"""Node-sharded persistent pipeline with the device-side exchange, R ranks on the one GPU of the test box:
every rank's results must equal the CPU oracle's sequential schedule, bit for bit, and the ranks' node
shards together must equal the oracle's final state.  Exercises the product multi-rank code: global node
indices at node_offset > 0, granule exchange through the ranks' receive rings, the rank merge in the merger
workgroups and the owner-only write-back.

The ranks are threads of this process joined by ksched_xchg_join_local_ex: their kernels run as ONE cooperative
launch, so every rank's grid is resident at once by construction.  (Round 3 ran them as separate processes
with separate plain launches; one rank's kernel was once descheduled for the whole 10 s timeout -- nothing
makes the launches of different processes co-resident.)  The rings come in the three kinds the join offers:
"plain" device memory, "uncached" -- allocated, zeroed and tagged exactly as the multi-process transport's
ksched_xchg_export does -- and "ipc", which also maps every peer's ring through its IPC handle as
ksched_xchg_import does.  The xGMI hop itself needs several GPUs."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def run_local(cl, world, calls=2, rings="plain", batch=64, engines=None):
    """`calls` schedule calls of cluster `cl` on `world` local ranks; returns ([per call results], final node
    shard) per rank.  engines: an already joined group to reuse (closed by the caller)."""
    from ksched.dist import make_local_xchg_group
    from ksched.engine import Engine
    own = engines is None
    ranks = make_local_xchg_group(cl, world, device=0, topk=16, batch=batch, rings=rings) if own else engines
    try:
        for e, (lo, hi) in ranks:
            assert e.xchg_ready, "exchange join failed"
            if own:
                st0 = e.read_nodes()
                assert all(np.array_equal(st0[k], a[lo:hi]) for k, a in
                           enumerate((cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods))), \
                    f"rank node state after load differs from the input (shard {lo}:{hi})"
                e.save_state()
        out = [None] * world
        errs = []

        def work(r):
            try:
                e = ranks[r][0]
                res = []
                for _ in range(calls):  # repeated calls: the granule tags advance across calls
                    e.restore_state()
                    oi, os_, of = e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)
                    st = e.stats()
                    res.append((oi, os_.view(np.int64), of, st["pipeline"], st["batches"], st["truncations"],
                                st["exact_rows"], st["rescues"]))
                out[r] = (res, e.read_nodes())
            except Exception as ex:  # surfaced below
                errs.append((r, repr(ex)))

        th = [threading.Thread(target=work, args=(r,)) for r in range(world)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=150)
        hung = [r for r, t in enumerate(th) if t.is_alive()]
        if hung:
            # a rank still inside schedule/sync may be running a kernel that reads its peers' rings: closing the
            # group under it could turn a hang into a fault -- leave the contexts alone and report
            own = False
            raise AssertionError(f"ranks {hung} did not finish within 150 s (group left open)")
        assert not errs, errs
        assert all(o is not None for o in out), "a rank did not finish"
        return out
    finally:
        if own:
            Engine.close_group([e for e, _ in ranks])


def check_oracle(cl, out, want, world):
    for r in range(world):
        for c, (oi, osb, of, pipe, nb, ntr, exr, nres) in enumerate(out[r][0]):
            assert pipe == "persistent", f"rank {r} ran the {pipe} pipeline"
            if not np.array_equal(oi, want[0]):
                agree = [all(np.array_equal(out[0][0][k][0], out[q][0][k][0]) for q in range(world))
                         for k in range(len(out[0][0]))]
                bad = np.nonzero(oi != want[0])[0][:5]
                raise AssertionError(
                    f"rank {r} call {c} ({nb} batches, {ntr} truncated, {exr} exact rows): assignments differ at {bad} "
                    f"(got {oi[bad]}, oracle {want[0][bad]}; ranks agree per call: {agree}; "
                    f"other calls: {[(x[4], x[5], x[6], int((x[0] != want[0]).sum())) for x in out[r][0]]})")
            assert np.array_equal(osb, want[1].view(np.int64)), f"rank {r}: score bits differ"
            assert np.array_equal(of, want[2]), f"rank {r}: feasible counts differ"
    got = [np.concatenate([out[r][1][k] for r in range(world)]) for k in range(3)]
    for k in range(3):
        assert np.array_equal(got[k], want[3][k]), f"final node state (resource {k}) differs"


@pytest.mark.parametrize("cfg,nn,pp,world", [("c3", 24000, 3000, 2), ("c5hc", 20000, 3000, 2), ("c4", 30000, 2500, 3),
                                             ("c4", 100000, 2500, 2), ("c5", 40000, 2000, 4), ("c4", 100000, 5000, 4)])
def test_xchg_ranks_match_oracle(gpu_available, oracle_mod, cfg, nn, pp, world):
    from ksched import cluster
    cl = cluster.make_cluster(cfg, n_nodes=nn, n_pods=pp)
    want = oracle_mod.schedule(cl, nthreads=8)
    check_oracle(cl, run_local(cl, world), want, world)


def test_xchg_eight_ranks_c4_full_nodes(gpu_available, oracle_mod):
    """R = 8 on c4's full 100k nodes (12.5k per rank) over rings of xchg_export's kind.  Eight ranks share the
    256 CUs (31 each): a batch of 32 (11 merger workgroups, 18 score workgroups of 695 rows per rank) fits."""
    from ksched import cluster
    cl = cluster.make_cluster("c4", n_nodes=100000, n_pods=3000)
    want = oracle_mod.schedule(cl, nthreads=8)
    check_oracle(cl, run_local(cl, 8, rings="uncached", batch=32), want, 8)


def test_xchg_groups_in_one_process_uncached(gpu_available, oracle_mod):
    """Several groups in ONE process over uncached rings, in the order that failed in round 4 (two-rank groups,
    a three-rank group, then a two-rank group whose rings can land where the earlier groups' were): each group's
    rings are zeroed at its setup and its tags start past every tag this process used, so no
    group may see an earlier group's granules."""
    from ksched import cluster
    for cfg, nn, pp, world in (("c3", 24000, 3000, 2), ("c4", 30000, 2500, 3), ("c4", 100000, 2500, 2),
                               ("c3", 24000, 3000, 2)):
        cl = cluster.make_cluster(cfg, n_nodes=nn, n_pods=pp)
        want = oracle_mod.schedule(cl, nthreads=8)
        check_oracle(cl, run_local(cl, world, rings="uncached"), want, world)


def test_xchg_rejoin_reuses_rings(gpu_available, oracle_mod):
    """One group joined, run, joined AGAIN (the same contexts: the rings are reused, zeroed again and the tags
    start past the process's used ones -- the rule of a second ksched_xchg_export/import) and run again: bit-exact
    both times."""
    from ksched import cluster
    from ksched.dist import make_local_xchg_group
    from ksched.engine import Engine
    cl = cluster.make_cluster("c4", n_nodes=60000, n_pods=2500)
    want = oracle_mod.schedule(cl, nthreads=8)
    ranks = make_local_xchg_group(cl, 2, device=0, topk=16, batch=64, rings="uncached")
    try:
        for e, _ in ranks:
            e.save_state()
        check_oracle(cl, run_local(cl, 2, calls=3, engines=ranks), want, 2)
        Engine.xchg_join_local([e for e, _ in ranks], rings="uncached")
        check_oracle(cl, run_local(cl, 2, calls=2, engines=ranks), want, 2)
    finally:
        Engine.close_group([e for e, _ in ranks])


def test_xchg_ipc_mapped_rings(gpu_available, oracle_mod):
    """The multi-process transport's ring setup on one device: every ring allocated and zeroed as
    ksched_xchg_export does and every peer's ring opened from its IPC handle as ksched_xchg_import does; the
    ranks still launch as one grid.  Skipped where the runtime does not open a handle of the same process."""
    from ksched import cluster
    from ksched._lib import KschedError
    cl = cluster.make_cluster("c4", n_nodes=60000, n_pods=2500)
    want = oracle_mod.schedule(cl, nthreads=8)
    try:
        out = run_local(cl, 2, rings="ipc")
    except KschedError as ex:
        if "hipIpcOpenMemHandle" in str(ex):
            pytest.skip(f"same-process IPC open refused by the runtime: {ex}")
        raise
    check_oracle(cl, out, want, 2)


@pytest.mark.parametrize("world", [2, 4])
def test_xchg_sharded_rescue(gpu_available, oracle_mod, world):
    """Node-sharded ranks rescue exhausted candidate lists instead of truncating (each rank's mergers scan its own
    shard, the R bests fold through the rings: ksched_commit.h rescue_rank_fold; restated by the oracle's
    or_schedule_lagged_rescue2 with shards): bit-exact, rescues happen, and the truncations stay within 2x of one
    rank's on the same cluster (where each rank alone would have truncated at every exhausted list)."""
    from ksched import Engine, MODE_BATCHED, cluster
    cl = cluster.make_cluster("c4", n_nodes=100000, n_pods=6000)
    want = oracle_mod.schedule(cl, nthreads=8)
    with Engine(mode=MODE_BATCHED, priority=cl.priority, domain=cl.domain, device=0, topk=16, batch=64) as e:
        e.load_nodes(cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods)
        oi, _, _ = e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods)
        one = e.stats()
    assert np.array_equal(oi, want[0])
    out = run_local(cl, world, calls=1, rings="uncached")
    check_oracle(cl, out, want, world)
    st = [x for r in range(world) for x in out[r][0]]
    resc = {x[7] for x in st}
    trunc = {x[5] for x in st}
    assert len(resc) == 1 and len(trunc) == 1, f"ranks disagree on rescues {resc} / truncations {trunc}"
    nres, ntr = resc.pop(), trunc.pop()
    print(f"sharded rescue R={world}: {nres} rescues, {ntr} truncated batches; one rank: {one['rescues']} rescues, "
          f"{one['truncations']} truncated")
    assert nres > 0, f"no rescue in {world} ranks (one rank: {one['rescues']} rescues, {one['truncations']} truncated)"
    assert ntr <= 2 * one["truncations"] + 2, f"{world} ranks truncated {ntr} batches, one rank {one['truncations']}"


def test_xchg_tags_wrap_across_calls(gpu_available, oracle_mod, monkeypatch):
    """Granule tags keep 15 bits (ksched_kernels.h gran_tag).  Tags started just below 2^15 (KSCHED_XCHG_EPOCH_BASE)
    cross the wrap during these calls, and calls with rescues alternate with short calls that write only some
    message slots and no rescue area: every call zeroes its ring's message and rescue areas before the rank barrier
    (ksched_engine.hip rx_zero_regions), so no wait can take an earlier call's granule.  Bit-exact."""
    from ksched import cluster
    from ksched.dist import make_local_xchg_group
    from ksched.engine import Engine
    monkeypatch.setenv("KSCHED_XCHG_EPOCH_BASE", str(32768 - 150))
    big = cluster.make_cluster("c4", n_nodes=100000, n_pods=6000)   # ~100 active batches and rescues per call
    small = big.subset_pods(70)                                    # two active batches, no rescue
    want_big = oracle_mod.schedule(big, nthreads=8)
    want_small = oracle_mod.schedule(small, nthreads=8)
    ranks = make_local_xchg_group(big, 2, device=0, topk=16, batch=64, rings="uncached")
    try:
        for e, _ in ranks:
            e.save_state()
        for rep in range(3):
            check_oracle(big, run_local(big, 2, calls=1, engines=ranks), want_big, 2)
            check_oracle(small, run_local(small, 2, calls=2, engines=ranks), want_small, 2)
    finally:
        Engine.close_group([e for e, _ in ranks])


def _full_c4_sharded(world, batch):
    """All 1M c4 pods at the full 100k nodes on `world` local ranks (batch `batch`) against one rank: the same
    assignments, score bits and feasible counts for every pod, every rank the same truncation and rescue counts,
    and the ranks' shards together conserving the requests (final state = initial - sum of the placed requests)."""
    from ksched import Engine, MODE_BATCHED, cluster
    cl = cluster.make_cluster("c4")
    with Engine(mode=MODE_BATCHED, priority=cl.priority, domain=cl.domain, device=0, topk=16, batch=batch) as e:
        e.load_nodes(cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods)
        oi, os_, of = e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods)
        one = e.stats()
        fin1 = e.read_nodes()
    assert one["pipeline"] == "persistent"
    out = run_local(cl, world, calls=1, rings="uncached", batch=batch)
    for r in range(world):
        ri, rs, rf, pipe, nb, ntr, exr, nres = out[r][0][0]
        assert pipe == "persistent"
        bad = np.nonzero(ri != oi)[0][:5]
        assert bad.size == 0, f"rank {r} of {world}: assignments differ from one rank at pods {bad}"
        assert np.array_equal(rs, os_.view(np.int64)), f"rank {r}: score bits differ from one rank"
        assert np.array_equal(rf, of), f"rank {r}: feasible counts differ from one rank"
    st = [out[r][0][0] for r in range(world)]
    assert len({x[5] for x in st}) == 1 and len({x[7] for x in st}) == 1, "ranks disagree on truncations / rescues"
    got = [np.concatenate([out[r][1][k] for r in range(world)]) for k in range(3)]
    placed = oi >= 0
    for k, (a0, req) in enumerate(((cl.alloc_cpu, cl.req_cpu), (cl.alloc_mem, cl.req_mem), (cl.alloc_pods, None))):
        d = np.zeros_like(a0)
        np.add.at(d, oi[placed], 1 if req is None else req[placed])
        assert np.array_equal(got[k], a0 - d), f"resource {k}: the shards do not conserve the placed requests"
        assert np.array_equal(got[k], fin1[k]), f"resource {k}: the shards differ from one rank's final state"
    print(f"c4 full size, {world} ranks at batch {batch}: {st[0][4]} batches, {st[0][5]} truncated, {st[0][7]} rescues "
          f"(one rank: {one['batches']}, {one['truncations']}, {one['rescues']})")


def test_xchg_full_c4_four_ranks(gpu_available):
    """the sharded path through the whole c4 sequence, high-conflict stretch included."""
    _full_c4_sharded(4, 64)


def test_xchg_full_c4_eight_ranks(gpu_available):
    _full_c4_sharded(8, 32)
