"""Host mirror over Kubernetes JSON, watch events and FailedScheduling diagnostics.

CPU part: the JSON decoding (anchor/types.go:48-123), the label vocabulary and the oracle's reason
restatement (anchor/predicate.go:127-157).  GPU part (-m gpu): the same clusters scheduled through
FakeCluster -> libksched; placements, FailedScheduling messages, per-node reasons and the node state
after watch events must equal the oracle exactly.
"""
import json

import numpy as np
import pytest

from kube_json import mask_labels, to_kube


def _c5_small(n_nodes=48, n_pods=300):
    from ksched import cluster
    cl = cluster.make_cluster("c5", n_nodes=n_nodes, n_pods=n_pods, with_strings=True)
    return mask_labels(cl)


# --------------------------------------------------------------------------------------------- CPU
def test_node_and_pod_decoding():
    from ksched.host import LabelVocab, node_from_kube, pod_from_kube
    nd = node_from_kube({"metadata": {"name": "n1", "labels": {"zone": "a"}, "annotations": {"hightower.com/cost": "0.40"}},
                         "status": {"capacity": {"cpu": "2", "memory": "7659876Ki", "pods": "110"},
                                    "allocatable": {"cpu": "1"}}})
    # allocatable comes from Capacity, not Status.Allocatable (anchor/predicate.go:58-60)
    assert nd.capacity == {"cpu": "2", "memory": "7659876Ki", "pods": "110"} and nd.price == "0.40"
    pd = pod_from_kube({"metadata": {"name": "p", "annotations": {"scheduler.alpha.kubernetes.io/name": "hightower"}},
                        "spec": {"nodeName": "", "nodeSelector": {"zone": "a"},
                                 "containers": [{"name": "a", "resources": {"requests": {"cpu": "200m"},
                                                                            "limits": {"cpu": "4"}}},
                                                {"name": "b"}]}})
    assert [c.requests for c in pd.containers] == [{"cpu": "200m"}, {}] and pd.node_name == ""
    v = LabelVocab()
    b = v.node_bits(nd.label_map)
    assert v.selector_bits(pd.node_selector) == b == 1
    assert v.selector_bits({"zone": "b"}) == 1 << LabelVocab.UNSATISFIABLE


def test_kube_json_packs_like_the_generator():
    """NodeList/PodList JSON -> C-ABI packer -> the generator's packed SoA (no device needed)."""
    from ksched.host import node_from_kube, pack_nodes, pack_pods, pod_from_kube
    cl = _c5_small()
    nl, pl = to_kube(cl)
    nl, pl = json.loads(json.dumps(nl)), json.loads(json.dumps(pl))
    nodes = [node_from_kube(x) for x in nl["items"]]
    pods = [pod_from_kube(x) for x in pl["items"]]
    ac, am, ap = pack_nodes(nodes, [p for p in pods if p.node_name])
    assert np.array_equal(ac, cl.alloc_cpu) and np.array_equal(am, cl.alloc_mem) and np.array_equal(ap, cl.alloc_pods)
    rc, rm, rp = pack_pods([p for p in pods if not p.node_name])
    assert np.array_equal(rc, cl.req_cpu) and np.array_equal(rm, cl.req_mem) and np.array_equal(rp, cl.req_pods)


def test_oracle_reason_order_kat(oracle_mod):
    """First failing check wins, in the reference's order CPU, Memory, Pod (anchor/predicate.go:134-148)."""
    from ksched import cluster
    cl = cluster.Cluster(name="kat", alloc_cpu=np.array([100, 100, 500, 500, 500, 500], np.int64),
                         alloc_mem=np.array([10, 999, 10, 999, 999, 999], np.int64),
                         alloc_pods=np.array([0, 0, 0, 0, 5, 5], np.int64),
                         req_cpu=np.array([200], np.int64), req_mem=np.array([100], np.int64),
                         req_pods=np.array([1], np.int64), labels=np.array([0, 0, 0, 0, 1, 2], np.uint64),
                         selector=np.array([1], np.uint64), use_labels=True)
    counts, reason = oracle_mod.node_reasons(cl, (cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods), 200, 100, 1, 1)
    assert reason.tolist() == [1, 1, 2, 3, 0, 4] and counts.tolist() == [1, 2, 1, 1, 1]


def test_oracle_reason_counts_match_feasible(oracle_mod):
    cl = _c5_small()
    oi, os_, of, counts, _ = oracle_mod.schedule_reasons(cl)
    wi, ws, wf, _ = oracle_mod.schedule(cl)
    assert np.array_equal(oi, wi) and np.array_equal(of, wf)
    assert np.array_equal(counts[:, 0], of) and np.all(counts.sum(1) == cl.n_nodes)
    assert (oi == -1).sum() > 5, "fixture should exercise NO_FIT pods"


# --------------------------------------------------------------------------------------------- GPU
def _expected_messages(O, cl, names):
    """FailedScheduling text of every NO_FIT pod from the oracle (state at the pod's turn)."""
    wi = O.schedule(cl)[0]
    msgs = {}
    for i in np.nonzero(wi == -1)[0]:
        state = O.schedule(cl, n_pods=int(i))[3]
        sel = 0 if cl.selector is None else int(cl.selector[i])
        _, reason = O.node_reasons(cl, state, cl.req_cpu[i], cl.req_mem[i], cl.req_pods[i], sel)
        text = {1: "Insufficient CPU", 2: "Insufficient Memory", 3: "Insufficient Pod",
                4: "node labels do not match the pod's selector"}
        lines = [f"fit failure on node ({names[j]}): {text[int(r)]}" for j, r in enumerate(reason) if r]
        msgs[f"pending-{i}"] = f"pod (pending-{i}) failed to fit in any node\n" + "\n".join(lines)
    return wi, msgs


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["exact", "batched"])
def test_fake_cluster_from_kube_json(gpu_available, oracle_mod, mode):
    from ksched import MODE_BATCHED, MODE_EXACT
    from ksched.host import FakeCluster, FitError
    cl = _c5_small()
    nl, pl = to_kube(cl)
    kw = dict(topk=8, batch=32) if mode == "batched" else {}
    fc = FakeCluster.from_kube_json(json.dumps(nl), json.dumps(pl), domain=cl.domain, use_labels=True,
                                    mode=MODE_BATCHED if mode == "batched" else MODE_EXACT, **kw)
    pending = fc.unscheduled_pods()
    assert len(pending) == cl.n_pods
    res = fc.schedule_pods(pending)
    wi, msgs = _expected_messages(oracle_mod, cl, cl.node_names)
    got = np.array([-1 if isinstance(r, FitError) else (-2 if isinstance(r, Exception) else
                                                         cl.node_names.index(r.name)) for _, r in res], np.int32)
    assert np.array_equal(got, wi)
    ev = {e["involved"]: e["message"] for e in fc.events if e["reason"] == "FailedScheduling"}
    assert ev == msgs
    # the explain walk leaves the device state where the schedule left it
    st = fc.engine.read_nodes()
    want = oracle_mod.schedule(cl)[3]
    assert all(np.array_equal(a, b) for a, b in zip(st, want))


@pytest.mark.gpu
def test_explain_matches_oracle(gpu_available, oracle_mod):
    from ksched import Engine, MODE_EXACT
    cl = _c5_small(n_nodes=3000, n_pods=64)
    with Engine(mode=MODE_EXACT, priority=cl.priority, domain=cl.domain, use_labels=True) as e:
        e.load_nodes(cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods, labels=cl.labels)
        state = (cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods)
        for i in range(cl.n_pods):
            cnt, rs = e.explain(cl.req_cpu[i], cl.req_mem[i], cl.req_pods[i], int(cl.selector[i]))
            wc, wr = oracle_mod.node_reasons(cl, state, cl.req_cpu[i], cl.req_mem[i], cl.req_pods[i], int(cl.selector[i]))
            assert np.array_equal(rs, wr) and np.array_equal(cnt, wc), f"pod {i}"
        cnt, rs = e.explain(0, 0, 0, 0, per_node=False)
        assert rs is None and cnt[0] == cl.n_nodes


@pytest.mark.gpu
def test_watch_events_maintain_node_state(gpu_available, oracle_mod):
    from ksched.host import FakeCluster, pack_nodes
    cl = _c5_small(n_nodes=32, n_pods=8)
    nl, pl = to_kube(cl)
    fc = FakeCluster.from_kube_json(nl, pl, domain=cl.domain, use_labels=True)
    before = fc.engine.read_nodes()
    # a pod bound by someone else: used += (cpu, mem, 1) on its node (anchor/predicate.go:83-105)
    ev = {"type": "ADDED", "object": {"metadata": {"name": "other"},
                                      "spec": {"nodeName": cl.node_names[5], "containers": [
                                          {"name": "x", "resources": {"requests": {"cpu": "0.7", "memory": "3Mi"}}}]}}}
    assert fc.handle_event(json.dumps(ev)) is None
    after = fc.engine.read_nodes()
    assert after[0][5] == before[0][5] - 699 and after[1][5] == before[1][5] - 3072 and after[2][5] == before[2][5] - 1
    want = pack_nodes(fc.nodes, [p for p in fc.pods if p.node_name])
    assert all(np.array_equal(a, b) for a, b in zip(after, want))
    fc.handle_event({"type": "DELETED", "object": ev["object"]})
    assert all(np.array_equal(a, b) for a, b in zip(fc.engine.read_nodes(), before))
    # a new unscheduled pod is scheduled on arrival (watch path, anchor/schedule.go:45-58)
    newp = {"type": "ADDED", "object": {"metadata": {"name": "late"}, "spec": {"nodeName": "", "containers": [
        {"name": "x", "resources": {"requests": {"cpu": "100m", "memory": "1Mi"}}}]}}}
    pod, res = fc.handle_event(newp)
    one = oracle_mod.schedule(type(cl)(name="one", alloc_cpu=before[0], alloc_mem=before[1], alloc_pods=before[2],
                                       req_cpu=np.array([100], np.int64), req_mem=np.array([1024], np.int64),
                                       req_pods=np.array([1], np.int64), labels=cl.labels,
                                       selector=np.array([0], np.uint64), domain=cl.domain, use_labels=True))[0]
    if one[0] >= 0:
        assert res.name == cl.node_names[int(one[0])] and pod.node_name == res.name
    else:
        assert isinstance(res, Exception)


@pytest.mark.gpu
def test_readme_demo_through_kube_json(gpu_available):
    from ksched import PRIORITY_BEST_PRICE, DOMAIN_FEASIBLE, cluster
    from ksched.host import FakeCluster
    cl = cluster.readme_demo()
    nl, pl = to_kube(cl)
    fc = FakeCluster.from_kube_json(nl, pl, priority=PRIORITY_BEST_PRICE, domain=DOMAIN_FEASIBLE)
    (pod, node), = fc.schedule_pods(fc.unscheduled_pods())
    assert node.name.endswith("-pxee") and fc.events[-1]["reason"] == "Scheduled"
