"""Kubernetes-JSON form of a synthetic cluster (test helper).

Turns a ksched.cluster.Cluster built with `with_strings=True` into the NodeList / PodList documents the
reference decodes (anchor/types.go:48-123): node capacity strings under status.capacity, already
bound pods (spec.nodeName set) carrying the used resources, and pending pods annotated with the
scheduler name (anchor/schedule.go:176).  Label bitsets become label maps {"bit<k>": "on"} and
selectors become spec.nodeSelector maps of the same pairs.
"""
from __future__ import annotations

import numpy as np

SCHED_ANN = "scheduler.alpha.kubernetes.io/name"
PRICE_ANN = "hightower.com/cost"


def _bits(v) -> list:
    v = int(v)
    return [k for k in range(64) if (v >> k) & 1]


def _containers(conts):
    return [{"name": f"c{k}", "resources": {"requests": dict(c)}} for k, c in enumerate(conts)]


def to_kube(cl):
    nodes = []
    for i, name in enumerate(cl.node_names):
        md = {"name": name}
        if cl.labels is not None and cl.use_labels:
            md["labels"] = {f"bit{k}": "on" for k in _bits(cl.labels[i])}
        if cl.node_price_str is not None:
            md["annotations"] = {PRICE_ANN: cl.node_price_str[i]}
        nodes.append({"metadata": md, "status": {"capacity": dict(cl.node_capacity[i])}})
    pods = []
    for j, (node, conts) in enumerate(cl.bound_pods or []):
        pods.append({"metadata": {"name": f"bound-{j}"}, "spec": {"nodeName": node, "containers": _containers(conts)}})
    for q, conts in enumerate(cl.pending_pods):
        spec = {"nodeName": "", "containers": _containers(conts)}
        if cl.selector is not None and cl.use_labels:
            spec["nodeSelector"] = {f"bit{k}": "on" for k in _bits(cl.selector[q])}
        pods.append({"metadata": {"name": f"pending-{q}", "annotations": {SCHED_ANN: "hightower"}}, "spec": spec})
    return ({"apiVersion": "v1", "kind": "NodeList", "items": nodes},
            {"apiVersion": "v1", "kind": "PodList", "metadata": {"resourceVersion": "1"}, "items": pods})


def mask_labels(cl, bits: int = 32):
    """Keep the label/selector bitsets within `bits` bits (the JSON vocabulary holds at most 63 pairs)."""
    m = np.uint64((1 << bits) - 1)
    if cl.labels is not None:
        cl.labels = cl.labels & m
    if cl.selector is not None:
        cl.selector = cl.selector & m
    return cl
