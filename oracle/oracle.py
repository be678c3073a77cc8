"""ctypes front-end of the C oracle (oracle/cpu_ref.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg as the checker.  The product never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libksched_oracle.so")
_lib = None

NO_FIT = -1
NO_POSITIVE_SCORE = -2


class Opts(C.Structure):
    _fields_ = [("priority", C.c_int32), ("domain", C.c_int32), ("use_labels", C.c_int32), ("pad", C.c_int32)]


REC_DTYPE = np.dtype([("key", "<f8"), ("idx", "<i4"), ("valid", "<i4"), ("a_cpu", "<i8"), ("a_mem", "<i8"),
                      ("a_pods", "<i8"), ("labels", "<u8"), ("price", "<f4"), ("pad", "<i4")])
TOUCHED_DTYPE = np.dtype([("idx", "<i4"), ("pad", "<i4"), ("s0", "<i8", 3), ("cur", "<i8", 3), ("labels", "<u8"),
                          ("price", "<f4"), ("pad2", "<i4")])


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = C.CDLL(_LIB_PATH)
        _lib.or_score.restype = C.c_double
        _lib.or_score.argtypes = [C.c_int64] * 6
        for fn in ("or_parse_cpu", "or_parse_memory", "or_parse_pods"):
            getattr(_lib, fn).argtypes = [C.c_char_p, C.POINTER(C.c_int64)]
            getattr(_lib, fn).restype = C.c_int
        _lib.or_commit_batch.restype = C.c_int64
        assert _lib.or_rec_size() == REC_DTYPE.itemsize
        assert _lib.or_touched_size() == TOUCHED_DTYPE.itemsize
    return _lib


def _p(a, t):
    return None if a is None else a.ctypes.data_as(C.POINTER(t))


def parse(kind: str, s):
    """Go-semantics quantity parse.  Returns the int64 value, or raises ValueError on the
    reference's errFatal paths."""
    out = C.c_int64(0)
    fn = {"cpu": lib().or_parse_cpu, "memory": lib().or_parse_memory, "pods": lib().or_parse_pods}[kind]
    rc = fn(None if s is None else s.encode(), C.byref(out))
    if rc != 0:
        raise ValueError(f"fatal parse of {kind}={s!r}")
    return out.value


def score(rc, rm, rp, ac, am, ap) -> float:
    return lib().or_score(int(rc), int(rm), int(rp), int(ac), int(am), int(ap))


def _opts(priority, domain, use_labels):
    return Opts(int(priority), int(domain), int(bool(use_labels)), 0)


def schedule(cl, nthreads: int = 1, n_pods=None):
    """Sequential reference semantics over a ksched.cluster.Cluster-like object.  Returns
    (idx int32[P], score f64[P], feasible int32[P], final (cpu, mem, pods))."""
    ac, am, ap = (np.ascontiguousarray(x, dtype=np.int64).copy() for x in (cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods))
    p = cl.n_pods if n_pods is None else int(n_pods)
    rc, rm, rp = (np.ascontiguousarray(x[:p], dtype=np.int64) for x in (cl.req_cpu, cl.req_mem, cl.req_pods))
    lab = None if cl.labels is None else np.ascontiguousarray(cl.labels, dtype=np.uint64)
    sel = None if cl.selector is None else np.ascontiguousarray(cl.selector[:p], dtype=np.uint64)
    pr = None if cl.price is None else np.ascontiguousarray(cl.price, dtype=np.float32)
    oi = np.empty(p, np.int32); os_ = np.empty(p, np.float64); of = np.empty(p, np.int32)
    o = _opts(cl.priority, cl.domain, cl.use_labels)
    r = lib().or_schedule(C.byref(o), C.c_int64(ac.shape[0]), _p(ac, C.c_int64), _p(am, C.c_int64), _p(ap, C.c_int64),
                          _p(lab, C.c_uint64), _p(pr, C.c_float), C.c_int64(p),
                          _p(rc, C.c_int64), _p(rm, C.c_int64), _p(rp, C.c_int64), _p(sel, C.c_uint64),
                          _p(oi, C.c_int32), _p(os_, C.c_double), _p(of, C.c_int32), C.c_int(nthreads))
    if r != 0:
        raise RuntimeError(f"or_schedule failed: {r}")
    return oi, os_, of, (ac, am, ap)


def node_reasons(cl, state, rc, rm, rp, sel=0):
    """Per-node first failing check of one pod against `state` = (cpu, mem, pods) arrays
    (anchor/predicate.go:134-148).  Returns (counts int64[5], reason uint8[n])."""
    ac, am, ap = (np.ascontiguousarray(x, dtype=np.int64) for x in state)
    lab = None if cl.labels is None else np.ascontiguousarray(cl.labels, dtype=np.uint64)
    reason = np.empty(ac.shape[0], np.uint8)
    counts = np.zeros(5, np.int64)
    o = _opts(cl.priority, cl.domain, cl.use_labels)
    lib().or_node_reasons(C.byref(o), C.c_int64(ac.shape[0]), _p(ac, C.c_int64), _p(am, C.c_int64), _p(ap, C.c_int64),
                          _p(lab, C.c_uint64), C.c_int64(int(rc)), C.c_int64(int(rm)), C.c_int64(int(rp)),
                          C.c_uint64(int(sel)), _p(reason, C.c_uint8), _p(counts, C.c_int64))
    return counts, reason


def schedule_reasons(cl, n_pods=None):
    """Sequential schedule plus every pod's reason counts at its turn.  Returns
    (idx, score, feasible, counts int64[P, 5], final state)."""
    ac, am, ap = (np.ascontiguousarray(x, dtype=np.int64).copy() for x in (cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods))
    p = cl.n_pods if n_pods is None else int(n_pods)
    rc, rm, rp = (np.ascontiguousarray(x[:p], dtype=np.int64) for x in (cl.req_cpu, cl.req_mem, cl.req_pods))
    lab = None if cl.labels is None else np.ascontiguousarray(cl.labels, dtype=np.uint64)
    sel = None if cl.selector is None else np.ascontiguousarray(cl.selector[:p], dtype=np.uint64)
    pr = None if cl.price is None else np.ascontiguousarray(cl.price, dtype=np.float32)
    oi = np.empty(p, np.int32); os_ = np.empty(p, np.float64); of = np.empty(p, np.int32)
    counts = np.zeros((p, 5), np.int64)
    o = _opts(cl.priority, cl.domain, cl.use_labels)
    r = lib().or_schedule_reasons(C.byref(o), C.c_int64(ac.shape[0]), _p(ac, C.c_int64), _p(am, C.c_int64),
                                  _p(ap, C.c_int64), _p(lab, C.c_uint64), _p(pr, C.c_float), C.c_int64(p),
                                  _p(rc, C.c_int64), _p(rm, C.c_int64), _p(rp, C.c_int64), _p(sel, C.c_uint64),
                                  _p(oi, C.c_int32), _p(os_, C.c_double), _p(of, C.c_int32), _p(counts, C.c_int64))
    if r != 0:
        raise RuntimeError(f"or_schedule_reasons failed: {r}")
    return oi, os_, of, counts, (ac, am, ap)


def schedule_batched(cl, K: int, B: int, n_pods=None):
    ac, am, ap = (np.ascontiguousarray(x, dtype=np.int64).copy() for x in (cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods))
    p = cl.n_pods if n_pods is None else int(n_pods)
    rc, rm, rp = (np.ascontiguousarray(x[:p], dtype=np.int64) for x in (cl.req_cpu, cl.req_mem, cl.req_pods))
    lab = None if cl.labels is None else np.ascontiguousarray(cl.labels, dtype=np.uint64)
    sel = None if cl.selector is None else np.ascontiguousarray(cl.selector[:p], dtype=np.uint64)
    pr = None if cl.price is None else np.ascontiguousarray(cl.price, dtype=np.float32)
    oi = np.empty(p, np.int32); os_ = np.empty(p, np.float64); of = np.empty(p, np.int32)
    st = np.zeros(3, np.int64)
    o = _opts(cl.priority, cl.domain, cl.use_labels)
    r = lib().or_schedule_batched(C.byref(o), C.c_int32(K), C.c_int32(B), C.c_int64(ac.shape[0]),
                                  _p(ac, C.c_int64), _p(am, C.c_int64), _p(ap, C.c_int64),
                                  _p(lab, C.c_uint64), _p(pr, C.c_float), C.c_int64(p),
                                  _p(rc, C.c_int64), _p(rm, C.c_int64), _p(rp, C.c_int64), _p(sel, C.c_uint64),
                                  _p(oi, C.c_int32), _p(os_, C.c_double), _p(of, C.c_int32), _p(st, C.c_int64))
    if r != 0:
        raise RuntimeError(f"or_schedule_batched failed: {r}")
    return oi, os_, of, (ac, am, ap), dict(batches=int(st[0]), truncations=int(st[1]), pairs=int(st[2]))


def schedule_pipelined(cl, K: int, B: int, n_pods=None):
    """CPU model of the GPU batched pipeline (lag-one snapshot, speculative plan, skip + resync)."""
    ac, am, ap = (np.ascontiguousarray(x, dtype=np.int64).copy() for x in (cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods))
    p = cl.n_pods if n_pods is None else int(n_pods)
    rc, rm, rp = (np.ascontiguousarray(x[:p], dtype=np.int64) for x in (cl.req_cpu, cl.req_mem, cl.req_pods))
    lab = None if cl.labels is None else np.ascontiguousarray(cl.labels, dtype=np.uint64)
    sel = None if cl.selector is None else np.ascontiguousarray(cl.selector[:p], dtype=np.uint64)
    pr = None if cl.price is None else np.ascontiguousarray(cl.price, dtype=np.float32)
    oi = np.empty(p, np.int32); os_ = np.empty(p, np.float64); of = np.empty(p, np.int32)
    st = np.zeros(3, np.int64)
    o = _opts(cl.priority, cl.domain, cl.use_labels)
    r = lib().or_schedule_pipelined(C.byref(o), C.c_int32(K), C.c_int32(B), C.c_int64(ac.shape[0]),
                                    _p(ac, C.c_int64), _p(am, C.c_int64), _p(ap, C.c_int64),
                                    _p(lab, C.c_uint64), _p(pr, C.c_float), C.c_int64(p),
                                    _p(rc, C.c_int64), _p(rm, C.c_int64), _p(rp, C.c_int64), _p(sel, C.c_uint64),
                                    _p(oi, C.c_int32), _p(os_, C.c_double), _p(of, C.c_int32), _p(st, C.c_int64))
    if r != 0:
        raise RuntimeError(f"or_schedule_pipelined failed: {r}")
    return oi, os_, of, (ac, am, ap), dict(batches=int(st[0]), truncations=int(st[1]), skipped=int(st[2]))


def schedule_lagged(cl, K: int, B: int, lag: int, n_pods=None, rescue: bool = False, rescue_max=None,
                    shards: int = 1):
    """CPU model of the persistent pipeline at lag `lag` (the device runs 3): cpu_ref.c or_schedule_lagged_rescue2;
    rescue=True resolves an exhausted candidate list by a full scan of the untouched nodes (the device's commit)
    instead of truncating the batch -- at most rescue_max per batch (None: no limit; the device's
    KSCHED_RESCUE_MAX), the scan split over `shards` contiguous node shards whose bests are folded (the
    node-sharded ranks' rescue)."""
    rmax = (-1 if rescue_max is None else int(rescue_max)) if rescue else 0
    ac, am, ap = (np.ascontiguousarray(x, dtype=np.int64).copy() for x in (cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods))
    p = cl.n_pods if n_pods is None else int(n_pods)
    rc, rm, rp = (np.ascontiguousarray(x[:p], dtype=np.int64) for x in (cl.req_cpu, cl.req_mem, cl.req_pods))
    lab = None if cl.labels is None else np.ascontiguousarray(cl.labels, dtype=np.uint64)
    sel = None if cl.selector is None else np.ascontiguousarray(cl.selector[:p], dtype=np.uint64)
    pr = None if cl.price is None else np.ascontiguousarray(cl.price, dtype=np.float32)
    oi = np.empty(p, np.int32); os_ = np.empty(p, np.float64); of = np.empty(p, np.int32)
    st = np.zeros(4, np.int64)
    o = _opts(cl.priority, cl.domain, cl.use_labels)
    r = lib().or_schedule_lagged_rescue2(C.byref(o), C.c_int32(K), C.c_int32(B), C.c_int32(lag), C.c_int32(rmax),
                                         C.c_int32(int(shards)), C.c_int64(ac.shape[0]),
                                 _p(ac, C.c_int64), _p(am, C.c_int64), _p(ap, C.c_int64),
                                 _p(lab, C.c_uint64), _p(pr, C.c_float), C.c_int64(p),
                                 _p(rc, C.c_int64), _p(rm, C.c_int64), _p(rp, C.c_int64), _p(sel, C.c_uint64),
                                 _p(oi, C.c_int32), _p(os_, C.c_double), _p(of, C.c_int32), _p(st, C.c_int64))
    if r != 0:
        raise RuntimeError(f"or_schedule_lagged failed: {r}")
    return oi, os_, of, (ac, am, ap), dict(batches=int(st[0]), truncations=int(st[1]), skipped=int(st[2]),
                                           rescues=int(st[3]))


def local_topk(opts, K, offset, ac, am, ap, labels, price, rc, rm, rp, sel):
    nb = rc.shape[0]
    recs = np.zeros(nb * K, REC_DTYPE)
    fc = np.zeros(nb, np.int64)
    o = _opts(*opts)
    lib().or_local_topk(C.byref(o), C.c_int32(K), C.c_int64(offset), C.c_int64(ac.shape[0]),
                        _p(ac, C.c_int64), _p(am, C.c_int64), _p(ap, C.c_int64), _p(labels, C.c_uint64),
                        _p(price, C.c_float), C.c_int64(nb), _p(rc, C.c_int64), _p(rm, C.c_int64),
                        _p(rp, C.c_int64), _p(sel, C.c_uint64), recs.ctypes.data_as(C.c_void_p), _p(fc, C.c_int64))
    return recs, fc


def merge_topk(K, R, nb, recs_all, fc_all):
    out = np.zeros(nb * K, REC_DTYPE)
    fc = np.zeros(nb, np.int64)
    recs_all = np.ascontiguousarray(recs_all)
    fc_all = np.ascontiguousarray(fc_all, dtype=np.int64)
    lib().or_merge_topk(C.c_int32(K), C.c_int32(R), C.c_int64(nb), recs_all.ctypes.data_as(C.c_void_p),
                        _p(fc_all, C.c_int64), out.ctypes.data_as(C.c_void_p), _p(fc, C.c_int64))
    return out, fc


def commit_batch(opts, K, rc, rm, rp, sel, lists, fc0, max_touched):
    nb = rc.shape[0]
    touched = np.zeros(max_touched, TOUCHED_DTYPE)
    nt = C.c_int32(0)
    oi = np.empty(nb, np.int32); os_ = np.empty(nb, np.float64); of = np.empty(nb, np.int32)
    o = _opts(*opts)
    done = lib().or_commit_batch(C.byref(o), C.c_int32(K), C.c_int64(nb), _p(rc, C.c_int64), _p(rm, C.c_int64),
                                 _p(rp, C.c_int64), _p(sel, C.c_uint64), lists.ctypes.data_as(C.c_void_p),
                                 _p(np.ascontiguousarray(fc0, dtype=np.int64), C.c_int64),
                                 touched.ctypes.data_as(C.c_void_p), C.byref(nt), C.c_int32(max_touched),
                                 _p(oi, C.c_int32), _p(os_, C.c_double), _p(of, C.c_int32))
    return int(done), touched[:nt.value], oi, os_, of
