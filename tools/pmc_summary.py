#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc passes (one pass per directory) -> one JSON file.

  python tools/pmc_summary.py OUT.json DIR [DIR ...]

Each DIR holds a `run_counter_collection.csv` from `rocprofv3 --pmc ... --kernel-trace
--output-format csv -o run`.  For every pipeline kernel family (score / merge / commit) the output
holds the per-launch average of every counter, the launch count and the average profiled duration.
Derived (MI355X_MICROARCH.md "HBM" + "rocprofv3 PMC slots"):
  fabric_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024  (both counters are in KiB; on
      gfx950 FETCH_SIZE reports half the bytes of a coalesced read, MI355X_MICROARCH.md "HBM")
  A wave64 VALU instruction occupies its SIMD (16 FP64 lanes, 32 FP32/INT lanes on gfx950) for 4
  cycles when it is FP64 (ADD/MUL/FMA/TRANS_F64; 78.6 TFLOP/s = 1024 SIMD x 16 lanes x 2 x 2.4 GHz)
  and 2 cycles otherwise, so over a launch of duration T on 1024 SIMDs:
  valu_busy_frac  = (4 * f64 + 2 * (VALU - f64)) / (T * 1024 SIMD * clock)   -- VALU pipe occupancy
  fp64_issue_frac = 4 * f64 / (T * 1024 * clock)                             -- FP64 share of that
  hbm_gbs         = fabric bytes / T
bench.py reads the file to fill roofline.traffic and the VALU fields.
"""
import csv
import json
import os
import sys
from collections import defaultdict

FAMILIES = {"k_pipe": "pipe", "k_persist_score": "score", "k_persist_merge": "merge", "k_persist_commit": "commit",
            "k_score_topk": "score", "k_merge_pod": "merge", "k_merge": "merge", "k_commit": "commit",
            "k_exact": "exact"}
CUS = 256
SIMDS = 4 * CUS
CLOCK_HZ = 2.4e9
F64 = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")


def family(name):
    base = name.replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].split("::")[-1]
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
            k["fabric_bytes_per_launch"] = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
        f64 = sum(avg.get(c, 0.0) for c in F64)
        if f64:
            k["f64_valu_insts_per_launch"] = f64
        if dur_ns > 0:
            cyc = dur_ns * 1e-9 * SIMDS * CLOCK_HZ
            if "fabric_bytes_per_launch" in k:
                k["hbm_gbs"] = k["fabric_bytes_per_launch"] / dur_ns
            if f64:
                k["fp64_issue_frac"] = 4 * f64 / cyc
                if "SQ_INSTS_VALU" in avg:  # from the same run only when both groups were in one pass
                    k["valu_busy_frac"] = (4 * f64 + 2 * (avg["SQ_INSTS_VALU"] - f64)) / cyc
            if "SQ_ACTIVE_INST_VALU" in avg:  # quad-cycles in which a wave issued VALU, summed over waves
                k["active_inst_valu_frac"] = 4 * avg["SQ_ACTIVE_INST_VALU"] / cyc
            if "SQ_BUSY_CYCLES" in avg:
                k["sq_busy_cycles_per_launch"] = avg["SQ_BUSY_CYCLES"]
        res["kernels"][kern] = k
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    for kern, k in res["kernels"].items():
        print(kern, {x: k[x] for x in k if x != "counters_per_launch"})


if __name__ == "__main__":
    main()
