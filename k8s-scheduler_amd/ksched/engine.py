"""Python front-end of the C-ABI engine (one context = one GPU = one node shard).

    eng = Engine(priority=PRIORITY_RESOURCE, mode=MODE_EXACT)
    eng.load_nodes(alloc_cpu, alloc_mem, alloc_pods, labels=None, price=None)
    idx, score, feasible = eng.schedule(req_cpu, req_mem, req_pods, selector=None)

`schedule` is the batched equivalent of the reference's schedulePods loop
(anchor/schedule.go:185-197): pods are resolved strictly in order and every placement is committed
before the next pod is evaluated.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _lib as L

# ksched_stats.pipeline (include/ksched.h KSCHED_PIPE_*)
PIPELINES = {0: "none", 1: "exact", 2: "stream", 3: "stream-sequential", 4: "persistent"}


def _i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


class Group:
    """In-process rank group (ksched_group): R contexts of this process on one device exchange their
    per-batch candidate lists through a shared device ring instead of RCCL.  Each rank's Engine calls
    set_group(); the ranks then run the same schedule calls concurrently (one thread each)."""

    def __init__(self, nranks: int, device: int = -1):
        h = C.c_void_p()
        L.check(L.lib().ksched_group_create(int(nranks), int(device), C.byref(h)), what="group_create")
        self._h = h
        self.nranks = nranks

    def close(self):
        if getattr(self, "_h", None):
            L.lib().ksched_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Engine:
    def __init__(self, mode: int = L.MODE_AUTO, priority: int = L.PRIORITY_RESOURCE, domain: int = L.DOMAIN_ALL,
                 use_labels: bool = False, batch: int = 0, topk: int = 0, device: int = -1,
                 rank: int = 0, nranks: int = 1, node_offset: int = 0, nodes_global: int = 0, exact_wgs: int = 0,
                 timing: bool = False, timing_every: int = 0, chunk_topk: int = 0,
                 commit_impl: int = 0, pipeline: int = L.PIPELINE_AUTO, pipe_wgs: int = 0):
        lb = L.lib()
        o = L.Opts()
        L.check(lb.ksched_default_opts(C.byref(o)), what="default_opts")
        o.mode, o.priority, o.domain, o.use_labels = mode, priority, domain, int(bool(use_labels))
        o.batch, o.topk, o.device = batch, topk, device
        o.rank, o.nranks, o.node_offset, o.nodes_global, o.exact_wgs = rank, nranks, node_offset, nodes_global, exact_wgs
        o.timing, o.timing_every, o.chunk_topk = int(bool(timing)), timing_every, chunk_topk
        o.commit_impl = commit_impl
        o.pipeline, o.pipe_wgs = pipeline, pipe_wgs
        ctx = L.CTX()
        L.check(lb.ksched_create(C.byref(o), C.byref(ctx)), what="create")
        self._ctx = ctx
        self.opts = o
        self.n = -1
        self.p = 0

    # -- lifecycle ---------------------------------------------------------------------------
    def close(self):
        if getattr(self, "_ctx", None):
            L.lib().ksched_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _chk(self, rc, what):
        L.check(rc, self._ctx, what)

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        L.check(L.lib().ksched_get_unique_id(buf), what="get_unique_id")
        return buf.raw

    def set_comm(self, uid: bytes):
        assert len(uid) == 128
        self._chk(L.lib().ksched_set_comm(self._ctx, uid), "set_comm")

    def xchg_export(self) -> bytes:
        """Allocate this rank's receive ring of the device-side exchange; returns its IPC handle."""
        buf = C.create_string_buffer(L.XCHG_HANDLE_BYTES)
        self._chk(L.lib().ksched_xchg_export(self._ctx, buf), "xchg_export")
        return buf.raw

    def xchg_import(self, handles):
        """Map every rank's ring (handles in rank order, as xchg_export returned them)."""
        blob = b"".join(handles)
        assert len(blob) == L.XCHG_HANDLE_BYTES * self.opts.nranks
        self._chk(L.lib().ksched_xchg_import(self._ctx, blob), "xchg_import")

    def xchg_close(self):
        """Turn the device exchange off on this rank (the ranks must agree on the transport)."""
        self._chk(L.lib().ksched_xchg_close(self._ctx), "xchg_close")

    @staticmethod
    def xchg_join_local(engines, rings: str = "plain"):
        """Ranks as threads of this process on one device (engines[r] = rank r): the device exchange, the ranks'
        persistent kernels as ONE cooperative launch (ksched_xchg_join_local_ex).  rings: "plain" device memory,
        "uncached" (allocated, zeroed and tagged exactly as xchg_export's) or "ipc" (uncached, and every peer's
        ring mapped from its IPC handle as xchg_import does)."""
        flags = {"plain": 0, "uncached": L.XCHG_RINGS_UNCACHED, "ipc": L.XCHG_RINGS_IPC}[rings]
        arr = (L.CTX * len(engines))(*[e._ctx for e in engines])
        L.check(L.lib().ksched_xchg_join_local_ex(arr, len(engines), flags), engines[0]._ctx, "xchg_join_local")

    @staticmethod
    def close_group(engines):
        """Close the ranks of a local group: every rank's peer maps first (xchg_close), then the contexts."""
        for e in engines:
            if e._ctx:
                L.lib().ksched_xchg_close(e._ctx)
        for e in engines:
            e.close()

    @property
    def xchg_ready(self) -> bool:
        return bool(L.lib().ksched_xchg_ready(self._ctx))

    def set_group(self, group: "Group"):
        self._chk(L.lib().ksched_set_group(self._ctx, group._h), "set_group")
        self._group = group  # keep the group alive as long as this context

    # -- nodes ---------------------------------------------------------------------------------
    def load_nodes(self, alloc_cpu, alloc_mem, alloc_pods, labels=None, price=None):
        ac, am, ap = _i64(alloc_cpu), _i64(alloc_mem), _i64(alloc_pods)
        n = ac.shape[0]
        assert am.shape[0] == n and ap.shape[0] == n
        lab = None if labels is None else np.ascontiguousarray(labels, dtype=np.uint64)
        pr = None if price is None else np.ascontiguousarray(price, dtype=np.float32)
        self._chk(L.lib().ksched_load_nodes(self._ctx, n, L.ptr(ac, C.c_int64), L.ptr(am, C.c_int64),
                                            L.ptr(ap, C.c_int64), L.ptr(lab, C.c_uint64), L.ptr(pr, C.c_float)),
                  "load_nodes")
        self.n = n

    def apply_delta(self, node_idx, d_cpu, d_mem, d_pods):
        ix = np.ascontiguousarray(node_idx, dtype=np.int32)
        dc, dm, dp = _i64(d_cpu), _i64(d_mem), _i64(d_pods)
        self._chk(L.lib().ksched_apply_delta(self._ctx, ix.shape[0], L.ptr(ix, C.c_int32), L.ptr(dc, C.c_int64),
                                             L.ptr(dm, C.c_int64), L.ptr(dp, C.c_int64)), "apply_delta")

    def explain(self, req_cpu: int, req_mem: int, req_pods: int, selector: int = 0, per_node: bool = True):
        """Predicate outcome of ONE pod against the current node state (anchor/predicate.go:127-157).
        Returns (counts int64[NUM_REASONS], reasons uint8[n] | None)."""
        cnt = np.zeros(L.NUM_REASONS, np.int64)
        rs = np.empty(max(self.n, 0), np.uint8) if per_node else None
        self._chk(L.lib().ksched_explain(self._ctx, int(req_cpu), int(req_mem), int(req_pods), int(selector),
                                         L.ptr(cnt, C.c_int64), L.ptr(rs, C.c_uint8)), "explain")
        return cnt, rs

    def explain_batch(self):
        """Reason counts (int64[p, NUM_REASONS]) of every NO_FIT pod of the last schedule call at its
        own turn, computed on the device; rows of other pods are zero.  Returns (counts, n_nofit)."""
        cnt = np.zeros((self.p, L.NUM_REASONS), np.int64)
        nf = C.c_int64(0)
        self._chk(L.lib().ksched_explain_batch(self._ctx, self.p, L.ptr(cnt, C.c_int64), C.byref(nf)),
                  "explain_batch")
        return cnt, nf.value

    def explain_pod(self, pod: int, per_node: bool = True):
        """Per-node reasons of pod `pod` of the last schedule call against the state it saw at its turn.
        Returns (counts int64[NUM_REASONS], reasons uint8[n] | None)."""
        cnt = np.zeros(L.NUM_REASONS, np.int64)
        rs = np.empty(max(self.n, 0), np.uint8) if per_node else None
        self._chk(L.lib().ksched_explain_pod(self._ctx, int(pod), L.ptr(cnt, C.c_int64), L.ptr(rs, C.c_uint8)),
                  "explain_pod")
        return cnt, rs

    def read_nodes(self):
        ac = np.empty(self.n, np.int64); am = np.empty(self.n, np.int64); ap = np.empty(self.n, np.int64)
        self._chk(L.lib().ksched_read_nodes(self._ctx, self.n, L.ptr(ac, C.c_int64), L.ptr(am, C.c_int64),
                                            L.ptr(ap, C.c_int64)), "read_nodes")
        return ac, am, ap

    def save_state(self):
        self._chk(L.lib().ksched_save_state(self._ctx), "save_state")

    def restore_state(self):
        self._chk(L.lib().ksched_restore_state(self._ctx), "restore_state")

    # -- pods ----------------------------------------------------------------------------------
    def upload_pods(self, req_cpu, req_mem, req_pods, selector=None):
        rc, rm, rp = _i64(req_cpu), _i64(req_mem), _i64(req_pods)
        p = rc.shape[0]
        sel = None if selector is None else np.ascontiguousarray(selector, dtype=np.uint64)
        self._keep = (rc, rm, rp, sel)
        self._chk(L.lib().ksched_upload_pods(self._ctx, p, L.ptr(rc, C.c_int64), L.ptr(rm, C.c_int64),
                                             L.ptr(rp, C.c_int64), L.ptr(sel, C.c_uint64)), "upload_pods")
        self.p = p

    def run(self):
        self._chk(L.lib().ksched_run(self._ctx), "run")

    def sync(self):
        self._chk(L.lib().ksched_sync(self._ctx), "sync")

    def results(self):
        oi = np.empty(self.p, np.int32); os_ = np.empty(self.p, np.float64); of = np.empty(self.p, np.int32)
        self._chk(L.lib().ksched_download_results(self._ctx, self.p, L.ptr(oi, C.c_int32), L.ptr(os_, C.c_double),
                                                  L.ptr(of, C.c_int32)), "download_results")
        return oi, os_, of

    def stats(self) -> dict:
        s = L.Stats()
        self._chk(L.lib().ksched_get_stats(self._ctx, C.byref(s)), "get_stats")
        return dict(pods=s.pods, placed=s.placed, batches=s.batches, truncations=s.truncations,
                    pair_evals=s.pair_evals, device_ms=s.device_ms, kernel_ms=list(s.kernel_ms),
                    kernel_launches=list(s.kernel_launches), kernel_pairs=list(s.kernel_pairs),
                    pipeline=PIPELINES.get(int(s.pipeline), str(int(s.pipeline))), rescues=s.rescues,
                    exact_rows=s.exact_rows, scan_rows=s.scan_rows)

    def set_timing(self, on: bool, every: int = 0):
        """Sampled per-kernel HIP-event timing for the following calls (every: one batch in N)."""
        self._chk(L.lib().ksched_set_timing(self._ctx, int(bool(on)), int(every)), "set_timing")

    def set_timeout(self, ms: int):
        """Bound (ms) of every device-side wait of the persistent pipeline (ksched_set_timeout)."""
        self._chk(L.lib().ksched_set_timeout(self._ctx, int(ms)), "set_timeout")

    def schedule(self, req_cpu, req_mem, req_pods, selector=None):
        """schedulePods over the given pending pods (in order).  Returns (idx, score, feasible)."""
        self.upload_pods(req_cpu, req_mem, req_pods, selector)
        self.run()
        self.sync()
        return self.results()


def engine_for(cl, mode: Optional[int] = None, **kw) -> Engine:
    """Engine configured for a ksched.cluster.Cluster and loaded with its nodes."""
    if mode is None:
        mode = L.MODE_EXACT if cl.mode == "exact" else L.MODE_BATCHED
    e = Engine(mode=mode, priority=cl.priority, domain=cl.domain, use_labels=cl.use_labels, **kw)
    e.load_nodes(cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods, labels=cl.labels, price=cl.price)
    return e
