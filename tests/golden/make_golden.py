"""Generates the committed golden fixtures under tests/golden/.

The reference (Go, no go.mod, no tests) cannot run in this image, so the expected values come from the
two independent CPU restatements (oracle/cpu_ref.c and oracle/ref_py.py), which must agree bit for
bit before anything is written.  The hand-derived values of SURVEY.md section 8c and the README demo
(README.md:43-58) are recorded as known-answer tests alongside.

Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "k8s-scheduler_amd"))

import oracle as O  # noqa: E402
import ref_py as R  # noqa: E402
from ksched import cluster  # noqa: E402

PARSE_CPU = ["0.7", "2.3", "3.3", "0.35", "0.1", "0.0015", "200m", "2", "4", "64", "0.5", "1.5", "-0.5", "+1.25",
             "1e3", "1.5e-3", "3.4e38", "3.5e38", "1e-50", "inf", "-Inf", "infinity", "nan", "NaN", "", "m", "abc",
             ".5", "5.", ".", "1e", "1e+", "0x1p-2", "0x1.8p1", "0x10", "1_000", "1__0", "_1", "1_", "0x_1p0",
             "1000000000000000000000", "9223372036854775807m", "9223372036854775808m", "-9223372036854775808m",
             "100.5m", " 1", "1 ", "+", "-", "1.1", "0.15", "0.25", "0.75", "1.7", "0.9", "2.5m",
             # Go literal forms strconv.ParseFloat accepts (hex mantissa + binary exponent, digit separators)
             "0X1P-2", "0x.8p1", "0x1p", "0x1", "0x1.fffffep127", "0x1.ffffffp127", "0x1p-149", "1_0.5",
             "1_0.5e1_0", "0x1_0p0", "1e1_0", "1_e5", "0_x1p0", "+_1", "-0x1p0", "+Inf", "+infinity", "infinit",
             "infx", "-nan", "nAn", "1.5E3", "1e-3_0", "1.5_", "0x1p1_", "0x1.p0", "0x.p0", "0x1p+_1", "1e_1",
             "0.000_1", "-0", "-0.0", "+.5e1", "1e99999", "0e99999", "0x1p99999", "0x1.8p-1", "0x0.4p4",
             "123456789012345678901234567890", "0.0005", "0.0015e0", "2.3e0", "0x1.26666p1"]
PARSE_MEM = ["7659876Ki", "64Mi", "4096Mi", "1Gi", "1024", "1G", "Ki", "Mi", "-5Ki", "+5Mi", "9007199254740993Mi",
             "9223372036854775807Ki", "9223372036854775808Ki", "1.5Mi", "0Ki", "12KI", "12ki"]
PARSE_PODS = ["110", "0", "-1", "+3", "1.0", "", "abc", "9223372036854775807", "9223372036854775808"]

# SURVEY.md 8c example values (capacities cpu 4000 m, mem 8388608 Ki, pods 110)
SCORE_KATS = [
    dict(req=[200, 0, 1], alloc=[4000, 8388608, 110], score=9.89915059687787, feasible=True),
    dict(req=[0, 0, 1], alloc=[4000, 8388608, 110], score=9.98475665748393, feasible=True),
    dict(req=[1000, 1024, 1], alloc=[1000, 1024, 1], score=0.0, feasible=True),
    dict(req=[1000, 1024, 1], alloc=[500, 8388608, 110], score=3.3179783676609844, feasible=False),
    dict(req=[100, 1024, 1], alloc=[-100, 8388608, 110], score=7.196540001880367, feasible=False),
]


def parse_vectors():
    out = []
    for kind, cases, pyf in (("cpu", PARSE_CPU, R.parse_cpu), ("memory", PARSE_MEM, R.parse_memory),
                             ("pods", PARSE_PODS, R.parse_pods)):
        for s in cases + [None]:
            try:
                c = O.parse(kind, s)
            except ValueError:
                c = "fatal"
            try:
                p = pyf(s)
            except R.Fatal:
                p = "fatal"
            if c != p:
                raise SystemExit(f"restatements disagree on {kind}={s!r}: C={c} py={p}")
            out.append(dict(kind=kind, s=s, value=c))
    return out


def score_kats():
    for k in SCORE_KATS:
        c = O.score(*k["req"], *k["alloc"])
        p = R.score(*k["req"], *k["alloc"])
        if c != p or abs(c - k["score"]) > 1e-12 * max(1, abs(k["score"])):
            raise SystemExit(f"score KAT mismatch {k}: C={c!r} py={p!r}")
        k["score_hex"] = float(c).hex()
    return SCORE_KATS


def run_small(cl):
    oi, os_, of, st = O.schedule(cl)
    pi, ps, pf, pst = R.schedule(np.stack([cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods], 1).tolist(),
                                 np.stack([cl.req_cpu, cl.req_mem, cl.req_pods], 1).tolist(),
                                 priority=cl.priority, domain=cl.domain, use_labels=cl.use_labels,
                                 labels=cl.labels, selector=cl.selector, price=cl.price)
    assert list(oi) == pi and list(of) == pf, cl.name
    assert [float(x).hex() for x in os_] == [float(x).hex() for x in ps], cl.name
    assert np.array_equal(np.stack(st, 1), np.array(pst, dtype=np.int64)), cl.name
    return oi, os_, of, st


def cluster_fixture(cl, oi, os_, of, st):
    d = dict(name=cl.name, priority=cl.priority, domain=cl.domain, use_labels=bool(cl.use_labels),
             alloc_cpu=cl.alloc_cpu.tolist(), alloc_mem=cl.alloc_mem.tolist(), alloc_pods=cl.alloc_pods.tolist(),
             req_cpu=cl.req_cpu.tolist(), req_mem=cl.req_mem.tolist(), req_pods=cl.req_pods.tolist(),
             labels=None if cl.labels is None else [int(x) for x in cl.labels],
             selector=None if cl.selector is None else [int(x) for x in cl.selector],
             price=None if cl.price is None else [float(x) for x in cl.price],
             expect_idx=[int(x) for x in oi], expect_score_hex=[float(x).hex() for x in os_],
             expect_feasible=[int(x) for x in of],
             expect_final=[st[0].tolist(), st[1].tolist(), st[2].tolist()])
    return d


def main():
    with open(os.path.join(HERE, "parse_vectors.json"), "w") as f:
        json.dump(parse_vectors(), f, indent=0)
    with open(os.path.join(HERE, "score_kats.json"), "w") as f:
        json.dump(score_kats(), f, indent=1)
    fixtures = []
    c1 = cluster.readme_demo()
    res = run_small(c1)
    assert int(res[0][0]) == 3, "README KAT: best price must pick ...-pxee (index 3)"
    fixtures.append(cluster_fixture(c1, *res))
    combos = [(0, 0, False), (0, 1, False), (1, 1, False), (0, 1, True), (1, 1, True), (0, 0, True)]
    for s in range(12):
        pr, dm, lb = combos[s % len(combos)]
        cl = cluster.random_small(1000 + s, n_nodes=48 + 7 * s, n_pods=160, priority=pr, domain=dm, use_labels=lb)
        fixtures.append(cluster_fixture(cl, *run_small(cl)))
    for name, nn, pp in (("c2", 300, 400), ("c3", 400, 400), ("c5", 500, 300)):
        cl = cluster.make_cluster(name, n_nodes=nn, n_pods=pp)
        cl.name = f"{name}_mini"
        fixtures.append(cluster_fixture(cl, *run_small(cl)))
    with open(os.path.join(HERE, "clusters.json"), "w") as f:
        json.dump(fixtures, f)
    print(f"wrote {len(fixtures)} cluster fixtures")


if __name__ == "__main__":
    main()
