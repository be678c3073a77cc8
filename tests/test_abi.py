"""CPU tests of the C-ABI library: it loads without a GPU, exports every symbol include/ksched.h
declares, and its host-side packer reproduces the reference's Go parsing and accounting."""
import json
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN, ROOT


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "ksched.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ksched_[a-z_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from ksched import _lib as L
    lb = L.lib()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lb, s), s
    # and the ctypes binding covers the whole header
    assert sorted(n for n, _, _ in L.SIGNATURES) == syms


def test_abi_version_and_defaults():
    import ctypes as C
    from ksched import _lib as L
    lb = L.lib()
    assert lb.ksched_abi_version() == L.ABI_VERSION == 6
    o = L.Opts()
    assert lb.ksched_default_opts(C.byref(o)) == 0
    assert o.struct_size == C.sizeof(L.Opts) and o.nranks == 1 and o.mode == L.MODE_AUTO


def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ksched import Engine, KschedError
    with pytest.raises(KschedError):
        Engine()


def test_product_parser_matches_golden_vectors():
    import ctypes as C
    from ksched import _lib as L
    fns = {"cpu": L.lib().ksched_parse_cpu, "memory": L.lib().ksched_parse_memory, "pods": L.lib().ksched_parse_pods}
    for v in json.load(open(os.path.join(GOLDEN, "parse_vectors.json"))):
        out = C.c_int64(0)
        rc = fns[v["kind"]](None if v["s"] is None else v["s"].encode(), C.byref(out))
        got = "fatal" if rc == L.E_PARSE else out.value
        assert rc in (L.OK, L.E_PARSE)
        assert got == v["value"], v


def test_product_parser_matches_oracle_random(oracle_mod):
    import ctypes as C
    from ksched import _lib as L
    rng = np.random.default_rng(5)
    alphabet = list("0123456789.eE+-_mxXpPiInNfFaKM ")
    for _ in range(4000):
        s = "".join(rng.choice(alphabet, size=int(rng.integers(0, 9))))
        for kind in ("cpu", "memory", "pods"):
            out = C.c_int64(0)
            rc = getattr(L.lib(), f"ksched_parse_{kind}")(s.encode(), C.byref(out))
            try:
                want = oracle_mod.parse(kind, s)
                assert rc == L.OK and out.value == want, (kind, s)
            except ValueError:
                assert rc == L.E_PARSE, (kind, s)


def test_product_parser_matches_independent_python_random():
    """The product parser (csrc/packer.cpp) against the pure-Python restatement of Go's strconv
    (oracle/ref_py.py: its own ParseFloat32 with hex literals and digit separators, written from the Go
    spec rather than from the C code) on random strings of the literal grammar's alphabet."""
    import ctypes as C
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ref_py as R
    from ksched import _lib as L
    rng = np.random.default_rng(11)
    pieces = ["0", "1", "7", "9", "0x", "0X", ".", "e", "E", "p", "P", "+", "-", "_", "a", "f", "F", "inf", "nan",
              "Infinity", "m", "Ki", "Mi", "5", "3"]
    pyf = {"cpu": R.parse_cpu, "memory": R.parse_memory, "pods": R.parse_pods}
    for _ in range(6000):
        s = "".join(rng.choice(pieces, size=int(rng.integers(1, 7))))
        for kind in ("cpu", "memory", "pods"):
            out = C.c_int64(0)
            rc = getattr(L.lib(), f"ksched_parse_{kind}")(s.encode(), C.byref(out))
            try:
                want = pyf[kind](s)
                assert rc == L.OK and out.value == want, (kind, s, out.value, want)
            except R.Fatal:
                assert rc == L.E_PARSE, (kind, s)


def test_price_parse():
    from ksched.host import FatalParse, parse_price
    assert parse_price("0.05") == np.float32(0.05)
    assert parse_price("1.60") == np.float32(1.6)
    for bad in ("", "abc", "inf", "nan", "3.5e38"):
        with pytest.raises(FatalParse):
            parse_price(bad)


def test_packer_matches_generator():
    """Kubernetes-string form -> packer -> SoA equals the generator's packed arrays."""
    from ksched import cluster
    from ksched.host import Container, Node, Pod, pack_nodes, pack_pods
    for name in ("c2", "c3", "c5"):
        cl = cluster.make_cluster(name, n_nodes=300, n_pods=500, with_strings=True)
        nodes = [Node(nm, cap) for nm, cap in zip(cl.node_names, cl.node_capacity)]
        bound = [Pod(f"b{i}", [Container(requests=r) for r in conts], node_name=nm)
                 for i, (nm, conts) in enumerate(cl.bound_pods)]
        ac, am, ap = pack_nodes(nodes, bound)
        assert np.array_equal(ac, cl.alloc_cpu) and np.array_equal(am, cl.alloc_mem)
        assert np.array_equal(ap, cl.alloc_pods)
        pend = [Pod(f"p{i}", [Container(requests=r) for r in conts]) for i, conts in enumerate(cl.pending_pods)]
        rc, rm, rp = pack_pods(pend)
        assert np.array_equal(rc, cl.req_cpu) and np.array_equal(rm, cl.req_mem) and np.array_equal(rp, cl.req_pods)


def test_packer_errors():
    from ksched.host import Container, FatalParse, Node, Pod, pack_nodes, pack_pods
    nodes = [Node("a", dict(cpu="2", memory="1Ki", pods="3"))]
    with pytest.raises(KeyError):  # reference: nil deref in usedResource (anchor/predicate.go:94-99)
        pack_nodes(nodes, [Pod("x", [Container(requests=dict(cpu="1m"))], node_name="ghost")])
    with pytest.raises(FatalParse):  # errFatal (anchor/predicate.go:15)
        pack_pods([Pod("x", [Container(requests=dict(cpu="1.5m"))])])
    with pytest.raises(FatalParse):  # errFatal (anchor/predicate.go:49)
        pack_nodes([Node("a", dict(cpu="2", memory="1Ki", pods="x"))], [])
    # a pod with no containers requests nothing and counts zero pods (anchor/predicate.go:72-79)
    rc, rm, rp = pack_pods([Pod("e", [])])
    assert rc.tolist() == [0] and rm.tolist() == [0] and rp.tolist() == [0]
    # used counts ONE pod per bound pod whatever its container count (anchor/predicate.go:102)
    ac, am, ap = pack_nodes(nodes, [Pod("b", [Container(requests=dict(cpu="100m", memory="1Mi"))] * 3,
                                        node_name="a")])
    assert ac.tolist() == [1700] and am.tolist() == [1 - 3072] and ap.tolist() == [2]


def test_generator_decimal_table(oracle_mod):
    from ksched import cluster
    for s, v in zip(cluster.DECIMAL_CPU, cluster.DECIMAL_CPU_VALUES):
        assert oracle_mod.parse("cpu", s) == int(v), s


def test_shard_ranges():
    from ksched.dist import shard_range
    for n in (0, 1, 5, 100, 100001):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1
