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
import json
from typing import Dict, List, Optional, Union

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
    uid: str = ""
    node_selector: Dict[str, str] = dataclasses.field(default_factory=dict)


@dataclasses.dataclass
class Node:
    name: str
    capacity: Dict[str, str]
    labels: int = 0
    price: Optional[str] = None  # price annotation (README.md:43-48)
    label_map: Dict[str, str] = dataclasses.field(default_factory=dict)


SCHEDULER_NAME = "hightower"                                # anchor/schedule.go:30
SCHEDULER_ANNOTATION = "scheduler.alpha.kubernetes.io/name"  # anchor/schedule.go:176
# The README's per-node price (README.md:37-48) has no key in the reference's code; the build reads
# it from this annotation (the upstream Hightower scheduler's key; build-defined).
PRICE_ANNOTATION = "hightower.com/cost"


def _as_obj(x):
    return json.loads(x) if isinstance(x, (str, bytes)) else x


class LabelVocab:
    """Build-defined label bitsets: every distinct "key=value" pair seen on a node
    gets one of 64 bits; a pod's nodeSelector becomes the OR of its pairs' bits.  A selector pair no
    node carries maps to a reserved bit no node has, so it fits nowhere (k8s nodeSelector meaning)."""
    UNSATISFIABLE = 63

    def __init__(self):
        self.bits: Dict[str, int] = {}

    def node_bits(self, labels: Dict[str, str]) -> int:
        v = 0
        for k, x in sorted(labels.items()):
            key = f"{k}={x}"
            if key not in self.bits:
                if len(self.bits) >= self.UNSATISFIABLE:
                    raise ValueError("more than 63 distinct node label pairs: widen the bitset")
                self.bits[key] = len(self.bits)
            v |= 1 << self.bits[key]
        return v

    def selector_bits(self, sel: Dict[str, str]) -> int:
        v = 0
        for k, x in sel.items():
            v |= 1 << self.bits.get(f"{k}={x}", self.UNSATISFIABLE)
        return v


def node_from_kube(obj: dict) -> Node:
    """One NodeList item (anchor/types.go:94-106): metadata.name/labels/annotations, status.capacity
    (allocatable is computed from Capacity, anchor/predicate.go:58-60)."""
    md = obj.get("metadata") or {}
    st = obj.get("status") or {}
    ann = md.get("annotations") or {}
    return Node(name=md.get("name", ""), capacity=dict(st.get("capacity") or {}), price=ann.get(PRICE_ANNOTATION),
                label_map=dict(md.get("labels") or {}))


def pod_from_kube(obj: dict) -> Pod:
    """One PodList item / watch event object (anchor/types.go:57-80): containers' resources.requests
    (limits are ignored, anchor/predicate.go:73-77) and spec.nodeName."""
    md = obj.get("metadata") or {}
    sp = obj.get("spec") or {}
    conts = [Container(name=c.get("name", ""), requests=dict((c.get("resources") or {}).get("requests") or {}))
             for c in (sp.get("containers") or [])]
    return Pod(name=md.get("name", ""), containers=conts, node_name=sp.get("nodeName") or "",
               annotations=dict(md.get("annotations") or {}), uid=md.get("uid", ""),
               node_selector=dict(sp.get("nodeSelector") or {}))


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
                 domain: int = L.DOMAIN_ALL, use_labels: bool = False, mode: int = L.MODE_AUTO, explain_failures: bool = True,
                 **engine_kw):
        self.nodes = list(nodes)
        self.pods = list(pods)
        self.events: List[dict] = []
        self.priority, self.domain, self.use_labels = priority, domain, use_labels
        self.explain_failures = explain_failures
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

    @classmethod
    def from_kube_json(cls, node_list: Union[str, dict], pod_list: Union[str, dict], **kw) -> "FakeCluster":
        """A cluster from the apiserver's NodeList / PodList JSON (what getNodes/getPods decode,
        anchor/tools.go:53-108, anchor/types.go:48-123).  Node label maps become bitsets when
        use_labels is set; the best-price priority reads PRICE_ANNOTATION."""
        nl, pl = _as_obj(node_list), _as_obj(pod_list)
        nodes = [node_from_kube(x) for x in (nl.get("items") or [])]
        pods = [pod_from_kube(x) for x in (pl.get("items") or [])]
        vocab = LabelVocab()
        for nd in nodes:
            nd.labels = vocab.node_bits(nd.label_map)
        c = cls(nodes, pods, **kw)
        c.vocab = vocab
        return c

    def unscheduled_pods(self) -> List[Pod]:
        """getUnscheduledPods (anchor/schedule.go:148-183): pods with no nodeName that name this
        scheduler in their annotation, in list order."""
        return [p for p in self.pods
                if not p.node_name and p.annotations.get(SCHEDULER_ANNOTATION) == SCHEDULER_NAME]

    def selector_of(self, pod: Pod) -> int:
        vocab = getattr(self, "vocab", None)
        return vocab.selector_bits(pod.node_selector) if vocab is not None else 0

    def _node_index(self, name: str) -> int:
        for i, nd in enumerate(self.nodes):
            if nd.name == name:
                return i
        raise KeyError(f"pod bound to unknown node {name!r} (reference: nil dereference, anchor/predicate.go:94-99)")

    def _charge(self, pod: Pod, sign: int) -> None:
        rc, rm, _ = pack_pods([pod])
        i = self._node_index(pod.node_name)
        # used += (cpu, mem, 1) per bound pod (anchor/predicate.go:83-105) => allocatable -= ...
        self.engine.apply_delta([i], [-sign * int(rc[0])], [-sign * int(rm[0])], [-sign])

    def handle_event(self, event: Union[str, dict]):
        """One pod watch event (PodWatchEvent, anchor/types.go:54-57).  The reference's watch loop
        schedules every ADDED unscheduled pod (anchor/schedule.go:45-58, 91-143) and re-counts every
        bound pod on each predicate call (anchor/predicate.go:83-105); here bound pods maintain the
        device node state incrementally (ksched_apply_delta) instead.  Returns the schedule result
        (pod, node | Exception) for an ADDED pending pod, else None."""
        ev = _as_obj(event)
        typ, pod = ev.get("type"), pod_from_kube(ev.get("object") or {})
        known = {p.name: p for p in self.pods}
        if typ == "ADDED":
            if pod.name in known:
                return None
            self.pods.append(pod)
            if pod.node_name:
                self._charge(pod, +1)
                return None
            # the watch selects spec.nodeName= only, with no scheduler-name check (anchor/schedule.go:
            # 94-95, 127-129, 52-56), unlike getUnscheduledPods
            return self.schedule_pods([pod])[0]
        if typ == "MODIFIED":
            old = known.get(pod.name)
            if old is not None and not old.node_name and pod.node_name:  # bound by someone else
                old.node_name = pod.node_name
                old.containers = pod.containers
                self._charge(old, +1)
            return None
        if typ == "DELETED":
            old = known.get(pod.name)
            if old is not None:
                self.pods.remove(old)
                if old.node_name:
                    self._charge(old, -1)
            return None
        return None

    def failed_scheduling_message(self, pod: Pod, reasons) -> str:
        """The FailedScheduling event text (anchor/predicate.go:152-171): the pod line, then one
        "fit failure on node (%s): Insufficient X" line per non-fitting node in node-list order."""
        lines = [f"fit failure on node ({self.nodes[j].name}): {L.REASON_TEXT[int(r)]}"
                 for j, r in enumerate(reasons) if r != L.REASON_FIT]
        return f"pod ({pod.name}) failed to fit in any node\n" + "\n".join(lines)

    def _explain_failures(self, idx):
        """Per-node reasons of every NO_FIT pod of the call just made, each against the state it saw at
        its own turn -- reconstructed on the device from the call's placements (ksched_explain_pod),
        no host replay and no state change."""
        return {i: self.engine.explain_pod(i)[1] for i, x in enumerate(idx) if x == L.NO_FIT}

    def bind(self, pod: Pod, node: Node) -> None:
        """POST Binding + Scheduled event (anchor/schedule.go:200-261), in memory."""
        pod.node_name = node.name
        self.events.append(dict(reason="Scheduled", message=f"Successfully assigned {pod.name} to {node.name}"))

    def schedule_pods(self, pending: Optional[List[Pod]] = None, selectors=None):
        """schedulePods (anchor/schedule.go:185-197): one engine call resolves every pending pod in order;
        binds follow in the same order.  Returns a list of (pod, node | Exception).  By default the
        pending set is getUnscheduledPods' (unbound pods annotated for this scheduler,
        anchor/schedule.go:175-177); pass `pending` to schedule any other list (the watch path)."""
        pending = self.unscheduled_pods() if pending is None else pending
        rc, rm, rp = pack_pods(pending)
        if selectors is None and self.use_labels:
            selectors = [self.selector_of(p) for p in pending]
        sel = None if not self.use_labels else np.asarray(selectors, dtype=np.uint64)
        idx, score, feas = self.engine.schedule(rc, rm, rp, sel)
        why = self._explain_failures(idx) if self.explain_failures else {}
        out = []
        for k, (pod, i) in enumerate(zip(pending, idx)):
            if i == L.NO_FIT:
                msg = (self.failed_scheduling_message(pod, why[k]) if k in why
                       else f"pod ({pod.name}) failed to fit in any node")
                self.events.append(dict(reason="FailedScheduling", message=msg, type="Warning",
                                        involved=pod.name))
                out.append((pod, FitError(f"Unable to schedule pod ({pod.name}) failed to fit in any node")))
            elif i == L.NO_POSITIVE_SCORE:
                out.append((pod, NilNodeError(pod.name)))
            else:
                node = self.nodes[int(i)]
                self.bind(pod, node)
                out.append((pod, node))
        return out

    def schedule_pod(self, pod: Pod, selector: Optional[int] = None):
        """schedulePod (anchor/schedule.go:68-89) for a single pod."""
        if selector is None:
            selector = self.selector_of(pod)
        res = self.schedule_pods([pod], selectors=[selector] if self.use_labels else None)[0][1]
        if isinstance(res, Exception):
            raise res
        return res
