#!/usr/bin/env python3
"""Per-batch distributions of the persistent pipeline's phase stamps (KSCHED_TRACE_DUMP raw file: [cap][16]
u64: wall-clock stamps at 100 MHz and the commit's counters in column 16, the columns of print_persist_trace in ksched_engine.hip).  The stderr summary
gives means; a mean can hide a few long stalls, so this prints percentiles and the stalls.

  python tools/trace_dist.py gpurun_out/trace_c4.bin [lag=3]
"""
import sys

import numpy as np

COLS = 54


def main():
    t = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, COLS).astype(np.int64)
    lag = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    n = t.shape[0]
    b = np.arange(lag, n)
    ok = (t[b, 0] > 0) & (t[b, 1] > 0) & (t[b, 2] > 0) & (t[b, 3] > 0) & (t[b, 4] > 0) & (t[b - lag, 4] > 0)
    b = b[ok]
    us = lambda x: x * 0.01  # noqa: E731  100 MHz ticks -> us
    ph = {
        "to-score (commit(b-L) end -> WG0 score start)": t[b, 0] - t[b - lag, 4],
        "score (WG0 start -> last arrival)": t[b, 1] - t[b, 0],
        "merge (last arrival -> last merge)": t[b, 2] - t[b, 1],
        "to-commit (last merge -> commit past wait)": t[b, 3] - t[b, 2],
        "commit (past wait -> end)": t[b, 4] - t[b, 3],
        "commit gap (commit(b-1) end -> past wait)": t[b, 3] - t[b - 1, 4],
        "period (commit(b-1) end -> commit(b) end)": t[b, 4] - t[b - 1, 4],
        "wg0 score busy (start -> its arrival)": t[b, 5] - t[b, 0],
        "loop top -> past wait": t[b, 3] - t[b, 15],
    }
    if (t[b, 22] > 0).all():  # two commit workgroups: P1, the hand-off, the rest
        ph["P1: past merges' wait -> past the hand-off"] = t[b, 22] - t[b, 3]
        ph["commit(b-1) end -> past the hand-off"] = t[b, 22] - t[b - 1, 4]
        ph["past the hand-off -> commit end"] = t[b, 4] - t[b, 22]
    sub = {}
    bs = b[(t[b, 22] > 0) & (t[b, 23] > 0) & (t[b, 24] > 0) & (t[b, 25] > 0) & (t[b, 49] > 0) & (t[b, 53] > 0)
           & (t[b - 1, 53] > 0) & ((t[b, 16] & 0xffff) == 1)]
    if len(bs):  # single-round batches: the chain from commit(b-1)'s record to commit(b)'s
        sub = {
            "record(b-1) issued -> past the hand-off": t[bs, 22] - t[bs - 1, 53],
            "  hand-off -> export(b-1) in slots": t[bs, 23] - t[bs, 22],
            "  -> its keys": t[bs, 24] - t[bs, 23],
            "  -> rounds start (wave-0 state)": t[bs, 25] - t[bs, 24],
            "  -> guess done": t[bs, 49] - t[bs, 25],
            "  -> evaluation done": t[bs, 50] - t[bs, 49],
            "  -> check done": t[bs, 51] - t[bs, 50],
            "  -> wave 0 past the rounds": t[bs, 52] - t[bs, 51],
            "  -> record issued (export, plan)": t[bs, 53] - t[bs, 52],
            "record(b-1) -> record(b)": t[bs, 53] - t[bs - 1, 53],
            "record(b) -> commit end (publish, outputs)": t[bs, 4] - t[bs, 53],
        }
    print(f"{len(b)} batches (lag {lag})")
    print(f"{'phase':48s} {'mean':>7s} {'p10':>7s} {'p50':>7s} {'p90':>7s} {'p99':>7s} {'max':>9s}  (us)")
    for k, v in ph.items():
        v = us(v.astype(np.float64))
        q = np.percentile(v, [10, 50, 90, 99])
        print(f"{k:48s} {v.mean():7.2f} {q[0]:7.2f} {q[1]:7.2f} {q[2]:7.2f} {q[3]:7.2f} {v.max():9.1f}")
    if sub:
        print(f"single-round batches ({len(bs)}), the commit chain:")
        for k, v in sub.items():
            v = us(v.astype(np.float64))
            q = np.percentile(v, [10, 50, 90, 99])
            print(f"{k:48s} {v.mean():7.2f} {q[0]:7.2f} {q[1]:7.2f} {q[2]:7.2f} {q[3]:7.2f} {v.max():9.1f}")
    per = us((t[b, 4] - t[b - 1, 4]).astype(np.float64))
    med = np.median(per)
    slow = per > 3 * med
    print(f"stalls (period > 3 x median {med:.1f} us): {slow.sum()} batches, {per[slow].sum() / 1e3:.2f} ms of "
          f"{per.sum() / 1e3:.2f} ms")
    order = np.argsort(-per)[:8]
    for i in order:
        bb = b[i]
        c = int(t[bb, 16])
        print(f"  batch {bb}: period {per[i]:.1f} us | score {us(t[bb, 1] - t[bb, 0]):.1f} merge {us(t[bb, 2] - t[bb, 1]):.1f}"
              f" to-commit {us(t[bb, 3] - t[bb, 2]):.1f} commit {us(t[bb, 4] - t[bb, 3]):.1f} | rounds {c & 0xffff}"
              f" rescues {(c >> 16) & 0xff} (waited {us(t[bb, 17]):.1f} us) done {(c >> 24) & 0xff} failed {(c >> 32) & 0xffff}"
              f" one-by-one {c >> 48} | kcycles pro {t[bb, 18] / 1e3:.1f} guess {t[bb, 19] / 1e3:.1f} eval {t[bb, 20] / 1e3:.1f}"
              f" check {t[bb, 21] / 1e3:.1f}")
    cc = t[b, 16]
    rounds, resc, done = cc & 0xffff, (cc >> 16) & 0xff, (cc >> 24) & 0xff
    seq = cc >> 48
    print(f"pods resolved one by one: {seq.sum()} ({seq.sum() / max(len(b), 1):.2f} per batch)")
    cm = us((t[b, 4] - t[b, 3]).astype(np.float64))
    rw = us(t[b, 17].astype(np.float64))
    print(f"rescue waits: {rw.sum() / 1e3:.2f} ms in total, {us(float(t[b, 17].sum())) / max(int(resc.sum()), 1):.1f} us per rescue")
    print("commit time by rescues in the batch:")
    for r in range(int(resc.max()) + 1 if len(resc) else 0):
        s = resc == r
        if s.any():
            print(f"  {r} rescues: {s.sum()} batches, commit mean {cm[s].mean():.1f} p50 {np.median(cm[s]):.1f} max {cm[s].max():.1f} us,"
                  f" rounds mean {rounds[s].mean():.2f}, resolved {done[s].mean():.1f}")
    print("commit time by rounds (kcycles per batch: prologue / guess / evaluate / check):")
    for lo, hi in ((0, 1), (1, 2), (2, 3), (3, 5), (5, 10), (10, 1 << 16)):
        s = (rounds >= lo) & (rounds < hi)
        if s.any():
            kc = [t[b[s], c].mean() / 1e3 for c in (18, 19, 20, 21, 26, 27, 28, 29, 30, 31, 32)]
            print(f"  rounds [{lo},{hi}): {s.sum()} batches, commit mean {cm[s].mean():.1f} max {cm[s].max():.1f} us, total"
                  f" {cm[s].sum() / 1e3:.2f} ms | {kc[0]:.1f} / {kc[1]:.1f} / {kc[2]:.1f} / {kc[3]:.1f}"
                  f" (guess: set-up {kc[9]:.1f} fixpoint {kc[10]:.1f}; check: update {kc[4]:.1f} probe {kc[5]:.1f}"
                  f" commit {kc[6]:.1f} [state load {kc[8]:.1f}] rescan {kc[7]:.1f})")
    # which phase of the chain is the long one when the period is long
    chain = us((t[b, 4] - t[b - lag, 4]).astype(np.float64))
    print(f"chain (commit(b-L) end -> commit(b) end): mean {chain.mean():.1f} p50 {np.median(chain):.1f} us = "
          f"{lag} x {chain.mean() / lag:.2f}")


if __name__ == "__main__":
    main()
