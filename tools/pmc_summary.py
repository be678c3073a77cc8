#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc passes (one pass per directory) -> one JSON file.

  python tools/pmc_summary.py OUT.json DIR [DIR ...]

Each DIR holds a `run_counter_collection.csv` from `rocprofv3 --pmc ... --kernel-trace
--output-format csv -o run`.  For every pipeline kernel family (score / merge / commit) the output
holds the per-launch average of every counter, the launch count and the average profiled duration.
Derived (MI355X_MICROARCH.md "HBM" + "rocprofv3 PMC slots"):
  fabric_bytes_per_launch = (FETCH_SIZE + WRITE_SIZE) * 1024  (both counters are in KiB; no x2
      correction for FETCH_SIZE: the score kernel's row loads are wave-uniform, not 16 B/lane
      streams, and the measured fetch equals one pass over the 96 B node rows)
  valu_issue_frac = SQ_INSTS_VALU / (profiled duration * 256 CU * clock), one VALU wave-instruction
      per CU per clock being the FP64 issue peak (78.6 TFLOP/s = 256 CU x 2.4 GHz x 64 FMA lanes)
bench.py reads the file to fill roofline.traffic.
"""
import csv
import json
import os
import sys
from collections import defaultdict

FAMILIES = {"k_score_topk": "score", "k_merge_pod": "merge", "k_merge": "merge", "k_commit": "commit",
            "k_exact": "exact"}
CUS = 256
CLOCK_HZ = 2.4e9


def family(name):
    base = name.split("(")[0].split("<")[0].split("::")[-1]
    for k, v in FAMILIES.items():
        if base.startswith(k):
            return base, v
    return None, None


def main():
    out_path, dirs = sys.argv[1], sys.argv[2:]
    vals = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)
    for d in dirs:
        seen = set()
        with open(os.path.join(d, "run_counter_collection.csv")) as f:
            for r in csv.DictReader(f):
                kern, fam = family(r["Kernel_Name"])
                if fam is None:
                    continue
                vals[kern][r["Counter_Name"]].append(float(r["Counter_Value"]))
                key = (d, r["Dispatch_Id"])
                if key not in seen:
                    seen.add(key)
                    durs[kern].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    res = {"source_dirs": [os.path.basename(os.path.normpath(d)) for d in dirs], "kernels": {}}
    for kern, cs in vals.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        dur_ns = sum(durs[kern]) / max(len(durs[kern]), 1)
        k = {"launches": max(len(v) for v in cs.values()), "avg_profiled_ns": dur_ns, "counters_per_launch": avg}
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            k["fetch_bytes_per_launch"] = avg["FETCH_SIZE"] * 1024
            k["write_bytes_per_launch"] = avg["WRITE_SIZE"] * 1024
            k["fabric_bytes_per_launch"] = (avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
        if "SQ_INSTS_VALU" in avg and dur_ns > 0:
            k["valu_issue_frac"] = avg["SQ_INSTS_VALU"] / (dur_ns * 1e-9 * CUS * CLOCK_HZ)
        f64 = sum(avg.get(c, 0.0) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                            "SQ_INSTS_VALU_TRANS_F64"))
        if f64:
            k["f64_valu_insts_per_launch"] = f64
        res["kernels"][kern] = k
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    for kern, k in res["kernels"].items():
        print(kern, {x: k[x] for x in k if x != "counters_per_launch"})


if __name__ == "__main__":
    main()
