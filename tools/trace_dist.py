#!/usr/bin/env python3
"""Per-batch distributions of the persistent pipeline's phase stamps (KSCHED_TRACE_DUMP raw file: [cap][16]
u64 wall-clock stamps at 100 MHz, the columns of print_persist_trace in ksched_engine.hip).  The stderr summary
gives means; a mean can hide a few long stalls, so this prints percentiles and the stalls.

  python tools/trace_dist.py gpurun_out/trace_c4.bin [lag=3]
"""
import sys

import numpy as np

COLS = 16


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
    print(f"{len(b)} batches (lag {lag})")
    print(f"{'phase':48s} {'mean':>7s} {'p10':>7s} {'p50':>7s} {'p90':>7s} {'p99':>7s} {'max':>9s}  (us)")
    for k, v in ph.items():
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
        print(f"  batch {bb}: period {per[i]:.1f} us | score {us(t[bb, 1] - t[bb, 0]):.1f} merge {us(t[bb, 2] - t[bb, 1]):.1f}"
              f" to-commit {us(t[bb, 3] - t[bb, 2]):.1f} commit {us(t[bb, 4] - t[bb, 3]):.1f}")
    # which phase of the chain is the long one when the period is long
    chain = us((t[b, 4] - t[b - lag, 4]).astype(np.float64))
    print(f"chain (commit(b-L) end -> commit(b) end): mean {chain.mean():.1f} p50 {np.median(chain):.1f} us = "
          f"{lag} x {chain.mean() / lag:.2f}")


if __name__ == "__main__":
    main()
