"""Seeded synthetic clusters for the BASELINE.json configs.

The reference has no fake cluster: it reads nodes/pods from kube-apiserver over HTTP
(anchor/tools.go:53-108).  For parity tests and the bench we generate the same *packed* inputs the
engine consumes (node allocatable = capacity - used, anchor/predicate.go:56-67; pod request sums,
anchor/predicate.go:69-81), plus -- for small clusters -- the Kubernetes quantity strings they come
from, so the host packer (Go-exact parsing) is exercised too.

Node order is the array index (the reference iterates nodeList.Items in API order).
"""
from __future__ import annotations

import dataclasses
from typing import Optional

import numpy as np

# Decimal CPU strings used for ~5% of containers: they go through Go's
# strconv.ParseFloat(s, 32) -> float64(f32) * 1000 -> int64 truncation (anchor/predicate.go:18-20),
# e.g. "0.7" -> 699.  Values are computed by go_cpu_decimal() below and pinned by tests against
# the oracle's independent parser.
DECIMAL_CPU = ("0.1", "0.15", "0.2", "0.25", "0.3", "0.35", "0.4", "0.5", "0.6", "0.7",
               "0.75", "0.8", "0.9", "1.1", "1.2", "1.3", "1.5", "1.7", "2.3", "3.3")

HC_USED_LO, HC_USED_SPAN = 0.97, 0.027  # c5hc node usage (cpu and memory)
HC_POD_SCALE = 1                        # c5hc pod requests relative to the standard pods
HC_HOT_EVERY = 50                       # c5hc: one fresh large node per this many nodes

PRIORITY_RESOURCE = 0
PRIORITY_BEST_PRICE = 1
DOMAIN_ALL = 0
DOMAIN_FEASIBLE = 1


def go_cpu_decimal(s: str) -> int:
    """int64(float64(float32(s)) * 1000) for the short decimal literals above.

    Only valid for literals whose decimal->float32 rounding is not disturbed by the intermediate
    double (true for every entry of DECIMAL_CPU; tests/test_cluster.py checks each one against the
    oracle's correctly-rounded strtof path).
    """
    f32 = np.float32(float(s))
    return int(np.trunc(np.float64(f32) * np.float64(1000.0)))


DECIMAL_CPU_VALUES = np.array([go_cpu_decimal(s) for s in DECIMAL_CPU], dtype=np.int64)


@dataclasses.dataclass
class Cluster:
    """Packed cluster: node state (SoA, index = node order) and pending pods (in schedule order)."""
    name: str
    alloc_cpu: np.ndarray          # int64 millicores
    alloc_mem: np.ndarray          # int64 KiB
    alloc_pods: np.ndarray         # int64
    req_cpu: np.ndarray            # int64
    req_mem: np.ndarray            # int64
    req_pods: np.ndarray           # int64 (= number of containers, anchor/predicate.go:78)
    labels: Optional[np.ndarray] = None     # uint64 node label bitsets
    selector: Optional[np.ndarray] = None   # uint64 pod selector bitsets
    price: Optional[np.ndarray] = None      # float32 node price
    priority: int = PRIORITY_RESOURCE
    domain: int = DOMAIN_ALL
    use_labels: bool = False
    mode: str = "exact"
    # Optional Kubernetes-string form (small clusters only), consumed by the host packer:
    node_names: Optional[list] = None
    node_capacity: Optional[list] = None    # list of dict(cpu=, memory=, pods=) strings
    bound_pods: Optional[list] = None       # list of (node_name, [dict(cpu=, memory=)]) already bound
    pending_pods: Optional[list] = None     # list of [dict(cpu=, memory=)] per pending pod
    node_price_str: Optional[list] = None

    @property
    def n_nodes(self) -> int:
        return int(self.alloc_cpu.shape[0])

    @property
    def n_pods(self) -> int:
        return int(self.req_cpu.shape[0])

    def subset_pods(self, n: int) -> "Cluster":
        c = dataclasses.replace(self)
        c.req_cpu = self.req_cpu[:n].copy()
        c.req_mem = self.req_mem[:n].copy()
        c.req_pods = self.req_pods[:n].copy()
        if self.selector is not None:
            c.selector = self.selector[:n].copy()
        c.pending_pods = None if self.pending_pods is None else self.pending_pods[:n]
        return c

    def node_state(self):
        return self.alloc_cpu.copy(), self.alloc_mem.copy(), self.alloc_pods.copy()


CONFIGS = {
    # name: (nodes, pods, priority, domain, labels, mode)
    "c1": (6, 1, PRIORITY_BEST_PRICE, DOMAIN_FEASIBLE, False, "exact"),
    "c2": (5_000, 10_000, PRIORITY_BEST_PRICE, DOMAIN_FEASIBLE, False, "exact"),
    "c3": (50_000, 100_000, PRIORITY_RESOURCE, DOMAIN_ALL, False, "batched"),
    "c4": (100_000, 1_000_000, PRIORITY_RESOURCE, DOMAIN_ALL, False, "batched"),
    "c5": (200_000, 500_000, PRIORITY_RESOURCE, DOMAIN_FEASIBLE, True, "batched"),
    # c5 made genuinely high-conflict: nodes 97-99.7 % used except one fresh large
    # node in every 50, so every batch piles onto the same few fresh nodes -- placements re-touch
    # nodes of the batch, and most batches exhaust some pod's candidate list (truncation + re-score)
    "c5hc": (200_000, 500_000, PRIORITY_RESOURCE, DOMAIN_FEASIBLE, True, "batched"),
}
CONFIG_IDS = {"c1": 1, "c2": 2, "c3": 3, "c4": 4, "c5": 5, "c5hc": 6}
SEED_BASE = 20260915


def _pods_standard(rng: np.random.Generator, p: int):
    """1-3 containers; cpu "<50..2000 step 50>m" (5% decimal strings); mem "<64..4096>Mi";
    ~3% of pods carry no requests at all (tie stress)."""
    ncont = rng.integers(1, 4, size=p)
    cpu = np.zeros((p, 3), dtype=np.int64)
    mem = np.zeros((p, 3), dtype=np.int64)
    cpu_m = rng.integers(1, 41, size=(p, 3)) * 50
    use_dec = rng.random((p, 3)) < 0.05
    dec_i = rng.integers(0, len(DECIMAL_CPU), size=(p, 3))
    cpu_v = np.where(use_dec, DECIMAL_CPU_VALUES[dec_i], cpu_m)
    mem_mi = rng.integers(64, 4097, size=(p, 3))
    zero = rng.random(p) < 0.03
    mask = (np.arange(3)[None, :] < ncont[:, None]) & ~zero[:, None]
    cpu[mask] = cpu_v[mask]
    mem[mask] = mem_mi[mask] * 1024
    return cpu, mem, ncont.astype(np.int64), use_dec, dec_i, cpu_m, mem_mi, zero


def make_cluster(name: str, seed: Optional[int] = None, n_nodes: Optional[int] = None,
                 n_pods: Optional[int] = None, with_strings: bool = False) -> Cluster:
    """Build config `name` ("c1".."c5"); n_nodes / n_pods override the sizes (same distributions)."""
    if name not in CONFIGS:
        raise ValueError(f"unknown config {name}")
    nn, pp, prio, dom, lab, mode = CONFIGS[name]
    if name == "c1":
        return readme_demo()
    nn = nn if n_nodes is None else int(n_nodes)
    pp = pp if n_pods is None else int(n_pods)
    seed = SEED_BASE + CONFIG_IDS[name] if seed is None else seed
    rng = np.random.default_rng(seed)
    if name in ("c2", "c3", "c4"):
        cap_cpu = rng.choice(np.array([4, 8, 16, 32, 64], dtype=np.int64), size=nn) * 1000
        cap_mem = rng.choice(np.array([8, 16, 32, 64, 128, 256], dtype=np.int64), size=nn) * (1 << 20)
        cap_pods = np.full(nn, 110, dtype=np.int64)
        ucpu, umem, upod = rng.random(nn) * 0.5, rng.random(nn) * 0.5, rng.random(nn) * 0.5
    else:  # c5: heterogeneous 2-192 cores, near-full
        cores = rng.integers(2, 193, size=nn).astype(np.int64)
        cap_cpu = cores * 1000
        cap_mem = cores * rng.choice(np.array([2, 4, 8], dtype=np.int64), size=nn) * (1 << 20)
        cap_pods = rng.choice(np.array([110, 250], dtype=np.int64), size=nn)
        lo, span = (0.85, 0.13) if name == "c5" else (HC_USED_LO, HC_USED_SPAN)
        ucpu = lo + rng.random(nn) * span
        umem = lo + rng.random(nn) * span
        upod = 0.85 + rng.random(nn) * 0.13
        if name == "c5hc":  # every HC_HOT_EVERY-th node is a fresh (empty) large node
            hot = np.arange(nn) % HC_HOT_EVERY == HC_HOT_EVERY - 1
            cores[hot] = rng.integers(64, 193, size=int(hot.sum()))
            cap_cpu[hot] = cores[hot] * 1000
            cap_mem[hot] = cores[hot] * 8 * (1 << 20)
            ucpu[hot] = umem[hot] = upod[hot] = 0.0
    used_cpu = np.floor(ucpu * cap_cpu).astype(np.int64)
    used_mem = np.floor(umem * cap_mem).astype(np.int64)
    used_pod = np.floor(upod * cap_pods).astype(np.int64)
    cpu, mem, ncont, use_dec, dec_i, cpu_m, mem_mi, zero = _pods_standard(rng, pp)
    if name == "c5hc":  # large pods: every container's request scaled up
        cpu, mem, cpu_m, mem_mi = cpu * HC_POD_SCALE, mem * HC_POD_SCALE, cpu_m * HC_POD_SCALE, mem_mi * HC_POD_SCALE
        use_dec[:] = False
    c = Cluster(name=name,
                alloc_cpu=cap_cpu - used_cpu, alloc_mem=cap_mem - used_mem, alloc_pods=cap_pods - used_pod,
                req_cpu=cpu.sum(1), req_mem=mem.sum(1), req_pods=ncont,
                priority=prio, domain=dom, use_labels=lab, mode=mode)
    if prio == PRIORITY_BEST_PRICE:
        c.price = (rng.integers(1, 201, size=nn) / 100.0).astype(np.float32)
    if lab:
        bits = rng.random((nn, 64)) < 0.3
        c.labels = np.packbits(bits, axis=1, bitorder="little").view(np.uint64).reshape(nn)
        nsel = rng.integers(0, 4, size=pp)
        selbits = np.zeros((pp, 64), dtype=bool)
        picks = rng.integers(0, 64, size=(pp, 3))
        for k in range(3):
            on = nsel > k
            selbits[np.nonzero(on)[0], picks[on, k]] = True
        c.selector = np.packbits(selbits, axis=1, bitorder="little").view(np.uint64).reshape(pp)
    if with_strings:
        _attach_strings(c, cap_cpu, cap_mem, cap_pods, used_cpu, used_mem, used_pod,
                        ncont, use_dec, dec_i, cpu_m, mem_mi, zero)
    return c


def _attach_strings(c, cap_cpu, cap_mem, cap_pods, used_cpu, used_mem, used_pod,
                    ncont, use_dec, dec_i, cpu_m, mem_mi, zero):
    """Kubernetes-string form: node capacity as strings; `used` expressed as bound pods.

    Each node's used (cpu, mem, pods) becomes used_pod bound pods (pods count one each,
    anchor/predicate.go:102) whose containers carry the cpu/mem amounts (first pod takes all of it;
    with used_pod == 0 but cpu/mem > 0 we add one pod and bump nothing else -- so the generator keeps
    used_pod >= 1 whenever cpu or mem is used)."""
    n = c.n_nodes
    c.node_names = [f"node-{i:06d}" for i in range(n)]
    c.node_capacity = [dict(cpu=str(int(cap_cpu[i]) // 1000) if cap_cpu[i] % 1000 == 0 else f"{int(cap_cpu[i])}m",
                            memory=f"{int(cap_mem[i])}Ki", pods=str(int(cap_pods[i]))) for i in range(n)]
    bound = []
    for i in range(n):
        k = int(used_pod[i])
        if k == 0 and (used_cpu[i] or used_mem[i]):
            # express the used cpu/mem through one extra bound pod and compensate in the packed state
            k = 1
            c.alloc_pods[i] -= 1
        for j in range(k):
            if j == 0:
                bound.append((c.node_names[i], [dict(cpu=f"{int(used_cpu[i])}m", memory=f"{int(used_mem[i])}Ki")]))
            else:
                bound.append((c.node_names[i], [dict()]))
    c.bound_pods = bound
    pend = []
    for q in range(c.n_pods):
        conts = []
        for k in range(int(ncont[q])):
            if zero[q]:
                conts.append(dict())
                continue
            cs = DECIMAL_CPU[int(dec_i[q, k])] if use_dec[q, k] else f"{int(cpu_m[q, k])}m"
            conts.append(dict(cpu=cs, memory=f"{int(mem_mi[q, k])}Mi"))
        pend.append(conts)
    c.pending_pods = pend
    if c.price is not None:
        c.node_price_str = [f"{float(x):.2f}" for x in c.price]


def readme_demo() -> Cluster:
    """Config c1: the README demo (README.md:43-58): 6 GKE nodes with annotator prices, one nginx pod
    requesting cpu 200m (deployments/nginx.yaml:46-48); best-price picks ...-pxee (index 3).  Node
    capacity is not stated in the README; we use cpu "2", memory "7659876Ki", pods "110" on all six."""
    names = ["gke-k0-default-pool-728d327f-" + s for s in ("00lq", "3vzg", "nmz7", "pxee", "xm4i", "zynj")]
    prices = ["0.80", "0.40", "0.40", "0.05", "1.60", "0.40"]
    n = 6
    c = Cluster(name="c1",
                alloc_cpu=np.full(n, 2000, np.int64), alloc_mem=np.full(n, 7659876, np.int64),
                alloc_pods=np.full(n, 110, np.int64),
                req_cpu=np.array([200], np.int64), req_mem=np.array([0], np.int64), req_pods=np.array([1], np.int64),
                price=np.array([float(x) for x in prices], dtype=np.float32),
                priority=PRIORITY_BEST_PRICE, domain=DOMAIN_FEASIBLE, use_labels=False, mode="exact")
    c.node_names = names
    c.node_capacity = [dict(cpu="2", memory="7659876Ki", pods="110") for _ in range(n)]
    c.bound_pods = []
    c.pending_pods = [[dict(cpu="200m")]]
    c.node_price_str = prices
    return c


def random_small(seed: int, n_nodes: int = 64, n_pods: int = 256, priority: int = PRIORITY_RESOURCE,
                 domain: int = DOMAIN_ALL, use_labels: bool = False, edge: bool = True) -> Cluster:
    """Small adversarial clusters for parity tests: negative / zero allocatable, zero requests,
    exact fits, identical nodes (ties), huge values near the int64 / 2^53 edges when `edge`."""
    rng = np.random.default_rng(seed)
    cap_choice = np.array([0, 1, 2, 100, 500, 1000, 4000, 64000], dtype=np.int64)
    ac = rng.choice(cap_choice, size=n_nodes) - rng.integers(0, 3, size=n_nodes) * rng.integers(0, 200, size=n_nodes)
    am = rng.choice(np.array([0, 1024, 8 << 20, 64 << 20], dtype=np.int64), size=n_nodes) - rng.integers(0, 4096, size=n_nodes)
    ap = rng.choice(np.array([0, 1, 2, 3, 110], dtype=np.int64), size=n_nodes)
    # identical-node runs for tie coverage
    for s in range(0, n_nodes, 8):
        if rng.random() < 0.3:
            ac[s:s + 4] = ac[s]; am[s:s + 4] = am[s]; ap[s:s + 4] = ap[s]
    rc = rng.choice(np.array([0, 1, 50, 100, 200, 1000, 2000], dtype=np.int64), size=n_pods)
    rm = rng.choice(np.array([0, 1, 1024, 65536, 1 << 20], dtype=np.int64), size=n_pods)
    rp = rng.integers(0, 4, size=n_pods).astype(np.int64)
    if edge:
        k = max(1, n_pods // 32)
        idx = rng.integers(0, n_pods, size=k)
        rc[idx] = rng.choice(np.array([-5, (1 << 53) + 1, (1 << 62), -(1 << 62)], dtype=np.int64), size=k)
        kn = max(1, n_nodes // 16)
        nidx = rng.integers(0, n_nodes, size=kn)
        ac[nidx] = rng.choice(np.array([(1 << 53) + 3, (1 << 62) + 7, -(1 << 40), 9007199254740993], dtype=np.int64), size=kn)
    c = Cluster(name=f"small{seed}", alloc_cpu=ac.astype(np.int64), alloc_mem=am.astype(np.int64),
                alloc_pods=ap.astype(np.int64), req_cpu=rc, req_mem=rm, req_pods=rp,
                priority=priority, domain=domain, use_labels=use_labels, mode="exact")
    if priority == PRIORITY_BEST_PRICE:
        c.price = (rng.integers(1, 9, size=n_nodes) / 4.0).astype(np.float32)
    if use_labels:
        c.labels = rng.integers(0, 1 << 8, size=n_nodes, dtype=np.uint64) | (rng.integers(0, 2, size=n_nodes, dtype=np.uint64) << np.uint64(63))
        c.selector = rng.choice(np.array([0, 1, 2, 3, 1 << 7, (1 << 63) | 1], dtype=np.uint64), size=n_pods)
    return c
