#!/usr/bin/env python3
"""CPU simulation of the screened scan's row counts on the real states of a run.

  python tests/diag/screen_sim.py c4 [G=255] [eps=1e-4] [t0,t1,...]

The node state before pod t is the initial state minus every placement of pods < t (the sequential
schedule, from the CPU oracle -- cached in /tmp/screen_sim_<cfg>_idx.npy; the full c4 run takes ~6 min
on 8 threads).  For the batch of pods [t, t+64), with workgroup g owning rows j = g (mod G) and wave w
scanning rows r = w (mod 8) of them, it reports how many of a wave's rows pass 2 scores exactly: the union
over the 64 pods of the rows whose key + eps reaches the pod's bound L (the workgroup's KC-th best key
- eps), and, for comparison, the bound taken as the max over waves of each wave's own KC-th best.
Exploration tool; the keys are the reference formula in numpy f64 (anchor/priorities.go:5-23,45-50).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "k8s-scheduler_amd"), os.path.join(ROOT, "oracle")]


def state_at(cl, idx, t):
    ac, am, ap = cl.alloc_cpu.copy(), cl.alloc_mem.copy(), cl.alloc_pods.copy()
    if t == 0:
        return ac, am, ap
    pl = idx[:t]
    ok = pl >= 0
    np.subtract.at(ac, pl[ok], cl.req_cpu[:t][ok])
    np.subtract.at(am, pl[ok], cl.req_mem[:t][ok])
    np.subtract.at(ap, pl[ok], 1)
    return ac, am, ap


def keys(cl, sl, ac, am, ap):
    rc = cl.req_cpu[sl][:, None].astype(float)
    rm = cl.req_mem[sl][:, None].astype(float)
    rp = cl.req_pods[sl][:, None].astype(float)
    acf, amf, apf = (x[None, :].astype(float) for x in (ac, am, ap))
    with np.errstate(all="ignore"):
        c = np.where(acf == 0, 1.0, rc / acf)
        m = np.where(amf == 0, 1.0, rm / amf)
        p = np.where(apf == 0, 1.0, rp / apf)
        mean = ((c + m) + p) / 3.0
        var = (((c - mean) ** 2 + (m - mean) ** 2) + (p - mean) ** 2) / 3.0
        b = np.where((c >= 1) | (m >= 1) | (p >= 1), 0.0, (1 - var) * 10)
        lc = np.where((acf == 0) | (rc > acf), 0.0, (acf - rc) * 10 / acf)
        lm = np.where((amf == 0) | (rm > amf), 0.0, (amf - rm) * 10 / amf)
        lp = np.where((apf == 0) | (rp > apf), 0.0, (apf - rp) * 10 / apf)
        s = (b + ((lc + lm) + lp) / 3.0) / 2
    fit = (acf >= rc) & (amf >= rm) & (apf >= rp)
    if cl.use_labels:
        fit &= (cl.labels[None, :] & cl.selector[sl][:, None]) == cl.selector[sl][:, None]
    el = s > 0
    if cl.domain == 1:
        el &= fit
    return np.where(el, s, -np.inf)


def main():
    from ksched import cluster
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 255
    eps = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-4
    ts = [int(x) for x in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0]
    KC, W = 4, 12
    cl = cluster.make_cluster(cfg)
    idx = None
    if max(ts) > 0:
        cache = f"/tmp/screen_sim_{cfg}_idx.npy"
        if not os.path.exists(cache):
            import oracle as O
            np.save(cache, O.schedule(cl, nthreads=os.cpu_count() or 8, n_pods=max(ts))[0])
        idx = np.load(cache)
    n = cl.n_nodes
    for t in ts:
        ac, am, ap = state_at(cl, idx, t)
        K = keys(cl, slice(t, t + 64), ac, am, ap)
        R = (n + G - 1) // G
        Kp = np.full((K.shape[0], G * R), -np.inf)
        Kp[:, :n] = K
        Kw = Kp.reshape(K.shape[0], R, G)  # [pod, row, workgroup]
        L_wg = -np.sort(-Kw, axis=1)[:, KC - 1, :] - eps
        L_wv = np.max(np.stack([-np.sort(-Kw[:, w::W, :], axis=1)[:, KC - 1, :] for w in range(W)]), axis=0) - eps
        # KC-th best of the per-(wave, unroll slot) maxima: wave w's row r = w + k W sits in slot (k % SPU)
        SPU = 4
        sub = [Kw[:, w::W, :][:, u::SPU, :].max(axis=1) for w in range(W) for u in range(SPU)]
        L_sub = -np.sort(-np.stack(sub, axis=1), axis=1)[:, KC - 1, :] - eps
        for name, L in (("workgroup KC-th", L_wg), ("max of wave KC-th", L_wv), ("KC-th of slot maxima", L_sub)):
            need = Kw + eps >= L[:, None, :]
            union = np.array([need[:, w::W, :].any(0).sum(0) for w in range(W)])
            lane_max = np.array([need[:, w::W, :].sum(1).max(0) for w in range(W)])
            print(f"{cfg} t={t} bound={name}: rows/wave {Kw[:, 0::W, :].shape[1]}, exact rows/wave (union over pods) "
                  f"mean {union.mean():.2f} max {union.max()}, per-pod max {lane_max.mean():.2f}, "
                  f"needed per pod per workgroup {need.sum(1).mean():.2f}")


if __name__ == "__main__":
    main()
