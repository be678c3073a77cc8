"""ctypes binding of libksched.so (include/ksched.h).

The library is built in-tree (k8s-scheduler_amd/libksched.so, `make -C k8s-scheduler_amd`).  There is
no fallback: if the library is missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# KSCHED_LIB: an alternative in-tree build of the same ABI (A/B measurements of kernel variants)
LIB_PATH = os.environ.get("KSCHED_LIB") or os.path.join(PKG_ROOT, "libksched.so")
HEADER_PATH = os.path.join(os.path.dirname(PKG_ROOT), "include", "ksched.h")

OK = 0
E_INVALID = -1
E_DEVICE = -2
E_PARSE = -3
E_STATE = -4
E_NOMEM = -5
E_UNKNOWN_NODE = -6
NO_FIT = -1
NO_POSITIVE_SCORE = -2

ABI_VERSION = 6
XCHG_RINGS_UNCACHED, XCHG_RINGS_IPC = 1, 2
MODE_EXACT, MODE_BATCHED, MODE_AUTO = 0, 1, 2
PIPELINE_AUTO, PIPELINE_STREAM = 0, 1
PRIORITY_RESOURCE, PRIORITY_BEST_PRICE = 0, 1
DOMAIN_ALL, DOMAIN_FEASIBLE = 0, 1
REASON_FIT, REASON_CPU, REASON_MEMORY, REASON_POD, REASON_LABELS = 0, 1, 2, 3, 4
NUM_REASONS = 5
XCHG_HANDLE_BYTES = 128
# the reference's per-node failure text (anchor/predicate.go:135,140,145)
REASON_TEXT = {REASON_CPU: "Insufficient CPU", REASON_MEMORY: "Insufficient Memory", REASON_POD: "Insufficient Pod",
               REASON_LABELS: "node labels do not match the pod's selector"}

_ERRNAMES = {E_INVALID: "E_INVALID", E_DEVICE: "E_DEVICE", E_PARSE: "E_PARSE", E_STATE: "E_STATE",
             E_NOMEM: "E_NOMEM", E_UNKNOWN_NODE: "E_UNKNOWN_NODE"}


class Opts(C.Structure):
    _fields_ = [("struct_size", C.c_int32), ("mode", C.c_int32), ("priority", C.c_int32),
                ("domain", C.c_int32), ("use_labels", C.c_int32), ("batch", C.c_int32), ("topk", C.c_int32),
                ("device", C.c_int32), ("rank", C.c_int32), ("nranks", C.c_int32),
                ("node_offset", C.c_int64), ("nodes_global", C.c_int64), ("exact_wgs", C.c_int32),
                ("timing", C.c_int32), ("timing_every", C.c_int32), ("chunk_topk", C.c_int32),
                ("commit_impl", C.c_int32), ("pipeline", C.c_int32), ("pipe_wgs", C.c_int32),
                ("reserved", C.c_int32 * 1)]


class Stats(C.Structure):
    _fields_ = [("pods", C.c_int64), ("placed", C.c_int64), ("batches", C.c_int64), ("truncations", C.c_int64),
                ("pair_evals", C.c_int64), ("device_ms", C.c_double), ("kernel_ms", C.c_double * 4),
                ("kernel_launches", C.c_int64 * 4), ("kernel_pairs", C.c_int64 * 4),
                ("pipeline", C.c_int64), ("rescues", C.c_int64), ("exact_rows", C.c_int64), ("scan_rows", C.c_int64)]


class KschedError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        super().__init__(f"{_ERRNAMES.get(code, code)}: {msg}")
        self.code = code


_lib = None

I64P = C.POINTER(C.c_int64)
U64P = C.POINTER(C.c_uint64)
I32P = C.POINTER(C.c_int32)
F64P = C.POINTER(C.c_double)
F32P = C.POINTER(C.c_float)
CTX = C.c_void_p
STRV = C.POINTER(C.c_char_p)

# (name, restype, argtypes) -- every symbol declared in include/ksched.h
SIGNATURES = [
    ("ksched_abi_version", C.c_int, []),
    ("ksched_default_opts", C.c_int, [C.POINTER(Opts)]),
    ("ksched_create", C.c_int, [C.POINTER(Opts), C.POINTER(CTX)]),
    ("ksched_destroy", C.c_int, [CTX]),
    ("ksched_last_error", C.c_char_p, [CTX]),
    ("ksched_get_unique_id", C.c_int, [C.c_char_p]),
    ("ksched_set_comm", C.c_int, [CTX, C.c_char_p]),
    ("ksched_group_create", C.c_int, [C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    ("ksched_group_destroy", C.c_int, [C.c_void_p]),
    ("ksched_set_group", C.c_int, [CTX, C.c_void_p]),
    ("ksched_xchg_export", C.c_int, [CTX, C.c_char_p]),
    ("ksched_xchg_import", C.c_int, [CTX, C.c_char_p]),
    ("ksched_xchg_ready", C.c_int, [CTX]),
    ("ksched_xchg_close", C.c_int, [CTX]),
    ("ksched_xchg_join_local", C.c_int, [C.POINTER(CTX), C.c_int32]),
    ("ksched_xchg_join_local_ex", C.c_int, [C.POINTER(CTX), C.c_int32, C.c_int32]),
    ("ksched_load_nodes", C.c_int, [CTX, C.c_int64, I64P, I64P, I64P, U64P, F32P]),
    ("ksched_apply_delta", C.c_int, [CTX, C.c_int64, I32P, I64P, I64P, I64P]),
    ("ksched_explain", C.c_int, [CTX, C.c_int64, C.c_int64, C.c_int64, C.c_uint64, I64P, C.POINTER(C.c_uint8)]),
    ("ksched_explain_batch", C.c_int, [CTX, C.c_int64, I64P, I64P]),
    ("ksched_explain_pod", C.c_int, [CTX, C.c_int64, I64P, C.POINTER(C.c_uint8)]),
    ("ksched_read_nodes", C.c_int, [CTX, C.c_int64, I64P, I64P, I64P]),
    ("ksched_save_state", C.c_int, [CTX]),
    ("ksched_restore_state", C.c_int, [CTX]),
    ("ksched_schedule", C.c_int, [CTX, C.c_int64, I64P, I64P, I64P, U64P, I32P, F64P, I32P]),
    ("ksched_upload_pods", C.c_int, [CTX, C.c_int64, I64P, I64P, I64P, U64P]),
    ("ksched_run", C.c_int, [CTX]),
    ("ksched_sync", C.c_int, [CTX]),
    ("ksched_download_results", C.c_int, [CTX, C.c_int64, I32P, F64P, I32P]),
    ("ksched_get_stats", C.c_int, [CTX, C.POINTER(Stats)]),
    ("ksched_set_timing", C.c_int, [CTX, C.c_int32, C.c_int32]),
    ("ksched_set_timeout", C.c_int, [CTX, C.c_int32]),
    ("ksched_selftest_fastdiv", C.c_int, [CTX, C.c_int64, F64P, F64P, F64P, F64P]),
    ("ksched_parse_cpu", C.c_int, [C.c_char_p, I64P]),
    ("ksched_parse_memory", C.c_int, [C.c_char_p, I64P]),
    ("ksched_parse_pods", C.c_int, [C.c_char_p, I64P]),
    ("ksched_parse_price", C.c_int, [C.c_char_p, F32P]),
    ("ksched_pack_nodes", C.c_int, [C.c_int64, STRV, STRV, STRV, STRV, C.c_int64, STRV, I64P, STRV, STRV,
                                    I64P, I64P, I64P]),
    ("ksched_pack_pods", C.c_int, [C.c_int64, I64P, STRV, STRV, I64P, I64P, I64P]),
]


def lib():
    """Load libksched.so (raises if it has not been built: there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make -C {PKG_ROOT}` (no CPU fallback exists)")
        lb = C.CDLL(LIB_PATH)
        # KSCHED_LIB (a same-box A/B against an older build, tools/build_base.sh) admits the previous ABI: entry
        # points it lacks stay unbound (calling one raises AttributeError)
        ab = bool(os.environ.get("KSCHED_LIB"))
        for name, res, args in SIGNATURES:
            if ab and not hasattr(lb, name):
                continue
            fn = getattr(lb, name)
            fn.restype = res
            fn.argtypes = args
        if lb.ksched_abi_version() != ABI_VERSION and not (ab and lb.ksched_abi_version() >= ABI_VERSION - 1):
            raise ImportError("libksched ABI version mismatch")
        _lib = lb
    return _lib


def check(rc: int, ctx=None, what: str = "") -> None:
    if rc != OK:
        msg = ""
        if ctx:
            m = lib().ksched_last_error(ctx)
            msg = m.decode() if m else ""
        raise KschedError(rc, f"{what}: {msg}")


def ptr(a, t):
    return None if a is None else a.ctypes.data_as(C.POINTER(t))
