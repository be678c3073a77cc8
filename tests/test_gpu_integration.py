"""The Go shim's call sequence, compiled: integration/ksched_driver (C, linked to libksched.so) runs
create -> load_nodes -> schedule -> explain_batch -> ordered binds, with a simulated bind failure
undone through apply_delta and the rest rescheduled (integration/anchor_ksched.go is the same sequence
in Go).  Expected: the reference's sequential semantics (anchor/schedule.go:68-89,185-197,200-237) --
a pod whose bind fails stays unbound and every later pod sees the cluster without it -- replayed by
the oracle segment by segment."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
DRIVER = os.path.join(ROOT, "integration", "ksched_driver")
BIND_FAILED = -3


def write_input(path, cl, fails, events=()):
    """events: the bound-pod watch's (type 1 ADDED | 2 DELETED, node index or -1, cpu, mem, ours)"""
    n, p = cl.n_nodes, cl.n_pods
    lab = cl.labels if cl.labels is not None else np.zeros(n, np.uint64)
    pr = cl.price if cl.price is not None else np.zeros(n, np.float32)
    sel = cl.selector if cl.selector is not None else np.zeros(p, np.uint64)
    hdr = np.array([n, p, len(fails), cl.priority, cl.domain, int(cl.use_labels), int(cl.price is not None),
                    len(events)], np.int64)
    ev = np.asarray(events, np.int64).reshape(-1, 5)
    with open(path, "wb") as f:
        for a, t in ((hdr, np.int64), (cl.alloc_cpu, np.int64), (cl.alloc_mem, np.int64), (cl.alloc_pods, np.int64),
                     (lab, np.uint64), (pr, np.float32), (cl.req_cpu, np.int64), (cl.req_mem, np.int64),
                     (cl.req_pods, np.int64), (sel, np.uint64), (np.asarray(fails, np.int64), np.int64), (ev, np.int64)):
            f.write(np.ascontiguousarray(a, dtype=t).tobytes())


def read_output(path, n, p):
    b = open(path, "rb").read()
    o = 0

    def take(dt, k):
        nonlocal o
        a = np.frombuffer(b, dtype=dt, count=k, offset=o)
        o += a.nbytes
        return a
    stats = take(np.int64, 4)
    idx, score, feas = take(np.int32, p), take(np.float64, p), take(np.int32, p)
    counts = take(np.int64, p * 5).reshape(p, 5)
    final = (take(np.int64, n), take(np.int64, n), take(np.int64, n))
    return stats, idx, score, feas, counts, final


def expected(cl, fails, oracle_mod):
    """Sequential reference semantics with failed binds, by oracle segments."""
    import dataclasses
    fails = set(int(x) for x in fails)
    p = cl.n_pods
    state = cl.node_state()
    idx = np.empty(p, np.int32); score = np.empty(p); feas = np.empty(p, np.int32)
    counts = np.zeros((p, 5), np.int64)
    start = 0
    while start < p:
        seg = dataclasses.replace(cl, alloc_cpu=state[0], alloc_mem=state[1], alloc_pods=state[2],
                                  req_cpu=cl.req_cpu[start:], req_mem=cl.req_mem[start:], req_pods=cl.req_pods[start:],
                                  selector=None if cl.selector is None else cl.selector[start:])
        si, ss, sf, sc, fin = oracle_mod.schedule_reasons(seg)
        bad = [i for i in range(start, p) if i in fails and si[i - start] >= 0]
        stop = bad[0] if bad else p
        k = stop - start
        idx[start:stop], score[start:stop], feas[start:stop] = si[:k], ss[:k], sf[:k]
        counts[start:stop] = np.where((si[:k] == -1)[:, None], sc[:k], 0)
        if not bad:
            state = fin
            break
        idx[stop], score[stop], feas[stop] = BIND_FAILED, ss[k], sf[k]
        head = dataclasses.replace(seg, req_cpu=seg.req_cpu[:k], req_mem=seg.req_mem[:k], req_pods=seg.req_pods[:k],
                                   selector=None if seg.selector is None else seg.selector[:k])
        state = oracle_mod.schedule(head)[3] if k > 0 else state
        start = stop + 1
    return idx, score, feas, counts, state


@pytest.mark.parametrize("case", ["c5hc", "c3", "best_price"])
def test_driver_call_sequence(gpu_available, oracle_mod, tmp_path, case):
    from ksched import cluster
    assert os.path.exists(DRIVER), "integration/ksched_driver not built (build() / make -C integration)"
    if case == "c5hc":
        cl = cluster.make_cluster("c5hc", n_nodes=2000, n_pods=4000)
    elif case == "c3":
        cl = cluster.make_cluster("c3", n_nodes=3000, n_pods=2000)
    else:
        cl = cluster.make_cluster("c2", n_nodes=800, n_pods=1500)
    rng = np.random.default_rng(5)
    fails = np.sort(rng.choice(cl.n_pods, 6, replace=False))
    write_input(tmp_path / "in.bin", cl, fails)
    for mode, k, b in (("1", "16", "64"), ("0", "16", "64")):
        r = subprocess.run([DRIVER, str(tmp_path / "in.bin"), str(tmp_path / "out.bin"), mode, k, b],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        stats, idx, score, feas, counts, final = read_output(tmp_path / "out.bin", cl.n_nodes, cl.n_pods)
        wi, ws, wf, wc, wst = expected(cl, fails, oracle_mod)
        assert np.array_equal(idx, wi), f"mode {mode}: assignments differ"
        assert np.array_equal(score.view(np.int64), ws.view(np.int64)) and np.array_equal(feas, wf)
        assert np.array_equal(counts, wc), f"mode {mode}: FailedScheduling counts differ"
        assert all(np.array_equal(a, b) for a, b in zip(final, wst)), f"mode {mode}: final state differs"
        assert stats[2] == (wi == BIND_FAILED).sum() and stats[2] <= stats[0] <= 1 + stats[2]


def test_driver_watch_events(gpu_available, oracle_mod, tmp_path):
    """The shim's onPodEvent path: after a pass, pods bound / deleted by others move the device state by their
    requests (one pod each), the ADDED echo of this run's own binds is skipped, and an event on a node missing
    from the node list ends the driver with KSCHED_E_UNKNOWN_NODE (the reference's usedResource panics there,
    anchor/predicate.go:94-99)."""
    from ksched import cluster
    cl = cluster.make_cluster("c3", n_nodes=1500, n_pods=800)
    wi, _, _, _, wst = expected(cl, [], oracle_mod)
    j0 = int(wi[wi >= 0][0])
    events = [(1, 7, 900, 1 << 20, 0),   # another scheduler bound a pod on node 7
              (2, 11, 250, 4096, 0),     # a bound pod on node 11 was deleted
              (1, j0, 12345, 6789, 1),   # the echo of this run's first bind: skipped
              (1, 7, 100, 2048, 0)]
    write_input(tmp_path / "in.bin", cl, [], events)
    r = subprocess.run([DRIVER, str(tmp_path / "in.bin"), str(tmp_path / "out.bin"), "1", "16", "64"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    _, idx, _, _, _, final = read_output(tmp_path / "out.bin", cl.n_nodes, cl.n_pods)
    assert np.array_equal(idx, wi)
    want = [a.copy() for a in wst]
    for t, j, c, m, ours in events:
        if t == 1 and ours:
            continue
        s = -1 if t == 1 else 1
        want[0][j] += s * c; want[1][j] += s * m; want[2][j] += s
    assert all(np.array_equal(a, b) for a, b in zip(final, want)), "watch deltas differ"
    write_input(tmp_path / "in2.bin", cl, [], events + [(1, -1, 100, 100, 0)])
    r = subprocess.run([DRIVER, str(tmp_path / "in2.bin"), str(tmp_path / "out2.bin"), "1", "16", "64"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 6 and "unknown node" in r.stderr, (r.returncode, r.stderr)


@pytest.mark.parametrize("case", ["c3", "best_price", "c5hc"])
def test_driver_watch_path(gpu_available, oracle_mod, tmp_path, case):
    """The shim's schedulePodGPU for monitorUnscheduledPods (anchor/schedule.go:47-89): one ksched_schedule call per
    watched pod (KSCHED_MODE_AUTO: the exact kernel for one pod), explain_pod on NO_FIT, the bind, and a failed
    bind's commit undone -- the same sequential semantics as the batch driver, pod by pod."""
    from ksched import cluster
    assert os.path.exists(DRIVER), "integration/ksched_driver not built (build() / make -C integration)"
    if case == "c3":
        cl = cluster.make_cluster("c3", n_nodes=3000, n_pods=400)
    elif case == "c5hc":
        cl = cluster.make_cluster("c5hc", n_nodes=2000, n_pods=400)
    else:
        cl = cluster.make_cluster("c2", n_nodes=800, n_pods=400)
    rng = np.random.default_rng(9)
    fails = np.sort(rng.choice(cl.n_pods, 5, replace=False))
    write_input(tmp_path / "in.bin", cl, fails)
    r = subprocess.run([DRIVER, str(tmp_path / "in.bin"), str(tmp_path / "out.bin"), "2", "16", "64", "watch"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    stats, idx, score, feas, counts, final = read_output(tmp_path / "out.bin", cl.n_nodes, cl.n_pods)
    wi, ws, wf, wc, wst = expected(cl, fails, oracle_mod)
    assert np.array_equal(idx, wi), "watch path: assignments differ"
    assert np.array_equal(score.view(np.int64), ws.view(np.int64)) and np.array_equal(feas, wf)
    assert np.array_equal(counts, wc), "watch path: FailedScheduling counts differ"
    assert all(np.array_equal(a, b) for a, b in zip(final, wst)), "watch path: final state differs"
    assert stats[0] == cl.n_pods and stats[2] == (wi == BIND_FAILED).sum()
