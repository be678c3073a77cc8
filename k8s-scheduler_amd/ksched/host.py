"""Host-side mirror of the reference's scheduling surface over an in-memory cluster.

The reference drives its hot path through
    schedulePod(pod)  -> predicate(pod) -> priorities(pod, nodes) -> bind(pod, node)
        anchor/schedule.go:68-89, anchor/predicate.go:107-176, anchor/priorities.go:25-63
    schedulePods()    -> for pod in pending: schedulePod(pod)     anchor/schedule.go:185-197
against kube-apiserver (getNodes/getPods, anchor/tools.go:53-108).  FakeCluster keeps the same
function names, argument meaning and error behaviour, with the apiserver replaced by in-memory lists
and the compute by the GPU engine (packing via the C-ABI's Go-exact parser, scoring/commit on device).
"""
from __future__ import annotations

import ctypes as C
import dataclasses
from typing import Dict, List, Optional

import numpy as np

from . import _lib as L
from .engine import Engine


class FitError(Exception):
    """schedulePod's "Unable to schedule pod (%s) failed to fit in any node" (anchor/schedule.go:74-76)."""


class NilNodeError(Exception):
    """The reference binds a nil *Node when no node scores > 0 and panics (anchor/priorities.go:55-62,
    anchor/schedule.go:208); the build reports it instead."""


class FatalParse(Exception):
    """The reference's errFatal on an unparseable quantity (anchor/predicate.go:15,31,39,49)."""


@dataclasses.dataclass
class Container:
    name: str = "c"
    requests: Dict[str, str] = dataclasses.field(default_factory=dict)


@dataclasses.dataclass
class Pod:
    name: str
    containers: List[Container]
    node_name: str = ""
    annotations: Dict[str, str] = dataclasses.field(default_factory=dict)


@dataclasses.dataclass
class Node:
    name: str
    capacity: Dict[str, str]
    labels: int = 0
    price: Optional[str] = None  # price annotation (README.md:43-48)


def _strv(items):
    arr = (C.c_char_p * max(1, len(items)))()
    for i, s in enumerate(items):
        arr[i] = None if s is None else s.encode()
    return arr


def pack_nodes(nodes: List[Node], bound: List[Pod]):
    """allocatableResource for every node given the bound pods (anchor/predicate.go:56-105)."""
    n = len(nodes)
    names = _strv([x.name for x in nodes])
    cc = _strv([x.capacity.get("cpu") for x in nodes])
    cm = _strv([x.capacity.get("memory") for x in nodes])
    cp = _strv([x.capacity.get("pods") for x in nodes])
    off = [0]
    ccpu, cmem, bnode = [], [], []
    for p in bound:
        bnode.append(p.node_name)
        for c in p.containers:
            ccpu.append(c.requests.get("cpu"))
            cmem.append(c.requests.get("memory"))
        off.append(len(ccpu))
    offa = np.asarray(off, dtype=np.int64)
    ac = np.zeros(n, np.int64); am = np.zeros(n, np.int64); ap = np.zeros(n, np.int64)
    rc = L.lib().ksched_pack_nodes(n, names, cc, cm, cp, len(bound), _strv(bnode), L.ptr(offa, C.c_int64),
                                   _strv(ccpu), _strv(cmem), L.ptr(ac, C.c_int64), L.ptr(am, C.c_int64),
                                   L.ptr(ap, C.c_int64))
    if rc == L.E_PARSE:
        raise FatalParse("quantity parse failed")
    if rc == L.E_UNKNOWN_NODE:
        raise KeyError("a bound pod names a node that is not in the node list")
    L.check(rc, what="pack_nodes")
    return ac, am, ap


def pack_pods(pods: List[Pod]):
    """requestedResource for every pending pod (anchor/predicate.go:69-81)."""
    off = [0]
    ccpu, cmem = [], []
    for p in pods:
        for c in p.containers:
            ccpu.append(c.requests.get("cpu"))
            cmem.append(c.requests.get("memory"))
        off.append(len(ccpu))
    offa = np.asarray(off, dtype=np.int64)
    k = len(pods)
    rc = np.zeros(k, np.int64); rm = np.zeros(k, np.int64); rp = np.zeros(k, np.int64)
    r = L.lib().ksched_pack_pods(k, L.ptr(offa, C.c_int64), _strv(ccpu), _strv(cmem), L.ptr(rc, C.c_int64),
                                 L.ptr(rm, C.c_int64), L.ptr(rp, C.c_int64))
    if r == L.E_PARSE:
        raise FatalParse("quantity parse failed")
    L.check(r, what="pack_pods")
    return rc, rm, rp


def parse_price(s: str) -> float:
    out = C.c_float(0)
    r = L.lib().ksched_parse_price(s.encode(), C.byref(out))
    if r != L.OK:
        raise FatalParse(f"price {s!r}")
    return out.value


class FakeCluster:
    """In-memory stand-in for kube-apiserver + the reference's scheduling functions."""

    def __init__(self, nodes: List[Node], pods: List[Pod], priority: int = L.PRIORITY_RESOURCE,
                 domain: int = L.DOMAIN_ALL, use_labels: bool = False, mode: int = L.MODE_AUTO, **engine_kw):
        self.nodes = list(nodes)
        self.pods = list(pods)
        self.events: List[dict] = []
        self.priority, self.domain, self.use_labels = priority, domain, use_labels
        self.engine = Engine(mode=mode, priority=priority, domain=domain, use_labels=use_labels, **engine_kw)
        self._sync_engine()

    # getNodes / getPods analogues
    def get_nodes(self) -> List[Node]:
        return self.nodes

    def get_pods(self) -> List[Pod]:
        return self.pods

    def _sync_engine(self):
        ac, am, ap = pack_nodes(self.nodes, [p for p in self.pods if p.node_name])
        labels = np.array([x.labels for x in self.nodes], dtype=np.uint64) if self.use_labels else None
        price = None
        if self.priority == L.PRIORITY_BEST_PRICE:
            price = np.array([parse_price(x.price) for x in self.nodes], dtype=np.float32)
        self.engine.load_nodes(ac, am, ap, labels=labels, price=price)

    def bind(self, pod: Pod, node: Node) -> None:
        """POST Binding + Scheduled event (anchor/schedule.go:200-261), in memory."""
        pod.node_name = node.name
        self.events.append(dict(reason="Scheduled", message=f"Successfully assigned {pod.name} to {node.name}"))

    def schedule_pods(self, pending: Optional[List[Pod]] = None, selectors=None):
        """schedulePods (anchor/schedule.go:185-197): one engine call resolves every pending pod in order;
        binds follow in the same order.  Returns a list of (pod, node | Exception)."""
        pending = [p for p in self.pods if not p.node_name] if pending is None else pending
        rc, rm, rp = pack_pods(pending)
        sel = None if not self.use_labels else np.asarray(selectors if selectors is not None else [0] * len(pending),
                                                          dtype=np.uint64)
        idx, score, feas = self.engine.schedule(rc, rm, rp, sel)
        out = []
        for pod, i in zip(pending, idx):
            if i == L.NO_FIT:
                self.events.append(dict(reason="FailedScheduling", message=f"pod ({pod.name}) failed to fit in any node"))
                out.append((pod, FitError(f"Unable to schedule pod ({pod.name}) failed to fit in any node")))
            elif i == L.NO_POSITIVE_SCORE:
                out.append((pod, NilNodeError(pod.name)))
            else:
                node = self.nodes[int(i)]
                self.bind(pod, node)
                out.append((pod, node))
        return out

    def schedule_pod(self, pod: Pod, selector: int = 0):
        """schedulePod (anchor/schedule.go:68-89) for a single pod."""
        res = self.schedule_pods([pod], selectors=[selector] if self.use_labels else None)[0][1]
        if isinstance(res, Exception):
            raise res
        return res
