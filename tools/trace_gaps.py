"""Pipeline gap analysis of a rocprofv3 kernel trace (CSV) of a batched run.

Per batch i the pipeline runs score(i) on stream S, merge(i) on M and commit(i) on C, with
score(i) after commit(i-2), merge(i) after score(i), commit(i) after merge(i).  For every kernel this
prints the distribution of its start minus the end of the dependency that released it last, and of
its duration, so the cost of the cross-stream hand-offs can be read off directly.

usage: python tools/trace_gaps.py <kernel_trace.csv> [lag=2]
"""
import csv
import sys

import numpy as np


def main():
    path = sys.argv[1]
    lag = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    fam = {"score": [], "merge": [], "commit": []}
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            t0, t1 = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
            if "k_score_topk" in name:
                fam["score"].append((t0, t1))
            elif "k_merge_pod" in name:
                fam["merge"].append((t0, t1))
            elif "k_commit" in name:
                fam["commit"].append((t0, t1))
    for k in fam:
        fam[k].sort()
    n = min(len(v) for v in fam.values())
    s, m, c = (np.array(fam[k][:n], dtype=np.int64) for k in ("score", "merge", "commit"))
    rows = []
    for i in range(lag + 1, n):
        dep_s = max(c[i - lag, 1], s[i - 1, 1])
        rows.append((s[i, 0] - dep_s, m[i, 0] - max(s[i, 1], m[i - 1, 1]), c[i, 0] - max(m[i, 1], c[i - 1, 1]),
                     s[i, 1] - s[i, 0], m[i, 1] - m[i, 0], c[i, 1] - c[i, 0],
                     s[i, 0] - c[i - lag, 1], s[i, 0] - s[i - 1, 1]))
    r = np.array(rows, dtype=np.float64) / 1000.0
    names = ["gap score<-commit/score", "gap merge<-score", "gap commit<-merge", "dur score", "dur merge",
             "dur commit", "score.start-commit(i-lag).end", "score.start-score(i-1).end"]
    print(f"batches {n}  per-batch wall {(s[-1, 0] - s[lag + 1, 0]) / 1000.0 / max(1, n - lag - 2):.2f} us")
    for k, nm in enumerate(names):
        col = r[:, k]
        print(f"{nm:34s} p10 {np.percentile(col, 10):8.2f}  p50 {np.percentile(col, 50):8.2f}  "
              f"p90 {np.percentile(col, 90):8.2f}  mean {col.mean():8.2f} us")
    # which dependency released score(i) last
    rel_commit = np.mean([c[i - lag, 1] >= s[i - 1, 1] for i in range(lag + 1, n)])
    print(f"score released by commit(i-{lag}) in {100 * rel_commit:.1f}% of batches (else by score(i-1))")


if __name__ == "__main__":
    main()
