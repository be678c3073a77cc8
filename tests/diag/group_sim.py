#!/usr/bin/env python3
"""CPU simulation of the score workgroups' row-group pruning ("group bounds").

  python tests/diag/group_sim.py [cfg=c4] [t0,t1,...] [sort=savg|morton|cpu|none] [gsize=4]

Each score workgroup sorts its rows once (at load, by the state then) and cuts them into groups of `gsize`; per
batch it keeps every group's per-resource [min, max] box of the allocatables.  For each pod of a batch the box
gives an upper bound U of every row's key and, when every row of the group surely fits with fractions < 0.999,
a lower bound Lo; L_box = the KC-th largest of min(KC, rows) copies of each group's Lo.  A group is skipped by
pass 1 when no pod's U reaches L_box.  Reports the fraction of rows pass 1 still scans, against the rows pass 2
scores exactly (the union over pods of the rows whose key reaches the KC-th best).  The node states are the
sequential schedule's (oracle, cached in /tmp/screen_sim_<cfg>_idx.npy as tests/diag/screen_sim.py makes it).
Exploration tool; f64 keys (anchor/priorities.go:5-23,45-50).
"""
import os
import sys

import numpy as np

sys.path[:0] = [os.path.dirname(os.path.abspath(__file__))]
from screen_sim import ROOT, keys, state_at  # noqa: E402

sys.path[:0] = [os.path.join(ROOT, "k8s-scheduler_amd"), os.path.join(ROOT, "oracle")]


def sort_order(kind, ac, am, ap, rows):
    a = np.stack([ac[rows], am[rows], ap[rows]], 1).astype(np.float64)
    if kind == "none":
        return np.arange(len(rows))
    if kind == "savg":
        return np.argsort(1000.0 / a[:, 0] + 4e6 / a[:, 1] + 2.0 / a[:, 2], kind="stable")
    if kind == "cpu":
        return np.lexsort((a[:, 1], a[:, 0]))
    if kind == "morton":
        q = np.clip(np.log2(np.maximum(a, 1.0)) * 16, 0, 1023).astype(np.int64)
        code = np.zeros(len(rows), np.int64)
        for bit in range(10):
            for d in range(3):
                code |= ((q[:, d] >> bit) & 1) << (3 * bit + d)
        return np.argsort(code, kind="stable")
    raise ValueError(kind)


def main():
    from ksched import cluster
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
    ts = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0]
    kinds = sys.argv[3].split(",") if len(sys.argv) > 3 else ["savg", "morton", "cpu", "none"]
    fresh = os.environ.get("FRESH", "0") == "1"  # sort by the state at t (regrouped) instead of at load
    gs = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    KC, G, eps, marg = 4, 232, 4e-5, 1e-4
    cl = cluster.make_cluster(cfg)
    n = cl.n_nodes
    idx = np.load(f"/tmp/screen_sim_{cfg}_idx.npy") if max(ts) > 0 else None
    a0 = cl.node_state()
    wgs = list(range(0, G, 29))
    for kind in kinds:
        for t in ts:
            ac, am, ap = state_at(cl, idx, t)
            sl = slice(t, t + 64)
            rc, rm, rp = (x[sl].astype(np.float64)[:, None] for x in (cl.req_cpu, cl.req_mem, cl.req_pods))
            scanned = exact = tot = ideal = 0
            gapL = 0.0
            for g in wgs:
                rows = np.arange(g, n, G)
                order = rows[sort_order(kind, *((ac, am, ap) if fresh else a0), rows)]
                ng = (len(order) + gs - 1) // gs
                pad = np.concatenate([order, np.full(ng * gs - len(order), order[-1])]).reshape(ng, gs)
                A = [x[pad].astype(np.float64) for x in (ac, am, ap)]  # [group][row]
                lo = [x.min(1)[None, :] for x in A]
                hi = [x.max(1)[None, :] for x in A]
                R = [rc, rm, rp]
                fl = [R[k] / hi[k] for k in range(3)]   # fraction lower bounds
                fh = [R[k] / lo[k] for k in range(3)]   # fraction upper bounds
                S_lo = fl[0] + fl[1] + fl[2]
                S_hi = fh[0] + fh[1] + fh[2]
                gap = np.maximum(0, np.maximum(np.maximum(fl[0], fl[1]), fl[2]) - np.minimum(np.minimum(fh[0], fh[1]), fh[2]))
                U_poly = 10 - 5 / 3 * S_lo - 5 * gap ** 2 / 6
                U_nf = 5 / 3 * ((1 - fl[0]) + (1 - fl[1]) + (1 - fl[2]))
                allfit = (R[0] <= lo[0]) & (R[1] <= lo[1]) & (R[2] <= lo[2])
                nonefit = (R[0] > hi[0]) | (R[1] > hi[1]) | (R[2] > hi[2])
                U = np.where(nonefit, U_nf, np.where(allfit, U_poly, np.maximum(U_poly, U_nf))) + marg
                D = np.maximum(np.maximum(fh[0], fh[1]), fh[2]) - np.minimum(np.minimum(fl[0], fl[1]), fl[2])
                Lo = np.where(allfit & (np.maximum(np.maximum(fh[0], fh[1]), fh[2]) < 0.999),
                              10 - 5 / 3 * S_hi - 5 * D ** 2 / 4 - marg, -np.inf)
                cop = np.repeat(Lo, min(KC, gs), axis=1)
                L_box = -np.sort(-cop, axis=1)[:, KC - 1]
                need = (U >= L_box[:, None]).any(0)
                scanned += need.sum() * gs
                K = keys(cl, sl, ac, am, ap)[:, rows]
                L_ex = -np.sort(-K, axis=1)[:, KC - 1] - eps
                ideal += (U >= L_ex[:, None]).any(0).sum() * gs
                gapL += (L_ex - L_box).mean()
                exact += ((K + eps) >= L_ex[:, None]).any(0).sum()
                tot += len(rows)
            print(f"{cfg} sort={kind} gsize={gs} t={t}: pass-1 rows {scanned / tot:.3f}, exact rows {exact / tot:.3f}, with the exact L {ideal / tot:.3f}, L gap {gapL / len(wgs):.4f}")


if __name__ == "__main__":
    main()
