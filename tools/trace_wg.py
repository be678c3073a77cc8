#!/usr/bin/env python3
"""Per-workgroup score timing of one persistent call (KSCHED_TRACE_WG=<file>, optionally with
KSCHED_PERSIST_TRACE=1 KSCHED_TRACE_DUMP=<file> for the commit stamps).

  python tools/trace_wg.py WG.bin [TRACE.bin]

For every batch: each score workgroup's scan start and arrival (100 MHz wall clock, low 32 bits).  Reports
what makes the last arrival late: the last workgroup's start lag behind the first start, its own scan time
against the batch's median, and whether it started late because it was still busy with the previous batch
(start - its previous arrival small) or because it saw commit(b - 3) late.
"""
import sys

import numpy as np

COLS = 54
LAG = 3


def main():
    raw = np.fromfile(sys.argv[1], dtype=np.uint64)
    G, cap = int(raw[0]), int(raw[1])
    t = raw[2:2 + G * cap].reshape(cap, G)
    ok = (t != 0).all(axis=1)
    st = (t & 0xffffffff).astype(np.int64)
    ar = (t >> 32).astype(np.int64)
    bs = np.nonzero(ok)[0]
    bs = bs[bs >= LAG + 1]
    base = st[bs].min(axis=1, keepdims=True)
    s = (st[bs] - base) / 100.0  # us after the batch's first start
    a = (ar[bs] - base) / 100.0
    d = a - s
    last = a.argmax(axis=1)
    rows = np.arange(len(bs))
    print(f"{len(bs)} batches, G = {G}")

    def pct(x, name):
        q = np.percentile(x, [10, 50, 90, 99])
        print(f"  {name:58s} mean {x.mean():6.2f}  p10 {q[0]:6.2f}  p50 {q[1]:6.2f}  p90 {q[2]:6.2f}  p99 {q[3]:6.2f}")

    pct(a.max(axis=1), "first start -> last arrival")
    pct(s.max(axis=1), "first start -> last start")
    pct(np.median(s, axis=1), "first start -> median start")
    pct(np.median(d, axis=1), "median scan (start -> arrival)")
    pct(d.max(axis=1), "longest scan")
    pct(s[rows, last], "last arriver: its start lag")
    pct(d[rows, last], "last arriver: its scan")
    pct(d[rows, last] - np.median(d, axis=1), "last arriver: scan - median scan")
    # busy-bound starts: a workgroup that arrived for b-1 less than 1 us before its start of b was still busy
    prev_ar = ar[bs - 1]
    gap = (st[bs] - prev_ar) / 100.0
    pct(gap[rows, last], "last arriver: its start - its previous arrival")
    print(f"  share of (batch, wg) starts within 1 us of the previous arrival: {(gap < 1.0).mean():.3f}")
    print(f"  ... for the last arrivers: {(gap[rows, last] < 1.0).mean():.3f}")
    if len(sys.argv) > 2:
        tr = np.fromfile(sys.argv[2], dtype=np.uint64).reshape(-1, COLS)
        cend = (tr[:, 4] & 0xffffffff).astype(np.int64)
        good = tr[bs - LAG, 4] != 0
        w = (st[bs][good] - cend[bs - LAG][good][:, None]) / 100.0  # start - commit(b-3) end, per wg
        wl = w[np.arange(good.sum()), last[good]]
        pct(w.min(axis=1), "commit(b-3) end -> first start")
        pct(np.median(w, axis=1), "commit(b-3) end -> median start")
        pct(wl, "commit(b-3) end -> last arriver's start")
    # per workgroup over the call
    md = d.mean(axis=0)
    ms = s.mean(axis=0)
    nl = np.bincount(last, minlength=G)
    order = np.argsort(-nl)[:12]
    print("  most often last:", " ".join(f"#{g}({nl[g]}x scan {md[g]:.2f} lag {ms[g]:.2f})" for g in order))
    print(f"  per-wg mean scan: min {md.min():.2f} median {np.median(md):.2f} max {md.max():.2f} us;"
          f" mean start lag: min {ms.min():.2f} median {np.median(ms):.2f} max {ms.max():.2f} us")
    print("  mean scan by g % 8:", " ".join(f"{k}:{md[k::8].mean():.2f}" for k in range(8)))
    print("  mean start lag by g % 8:", " ".join(f"{k}:{ms[k::8].mean():.2f}" for k in range(8)))


if __name__ == "__main__":
    main()
