#!/usr/bin/env python3
"""Headline bench: pod-node evaluations/s of the scheduling hot path (BASELINE.json metric).

A step = schedulePods over the whole pending set of the workload from the same initial cluster state:
every pod resolved in order with its placement committed before the next pod is evaluated
(anchor/schedule.go:185-197).  The node state is restored on device at the start of each step; pods
and nodes are HBM-resident before the timed region.  value = P x N / time (every pair the sequential
semantics evaluates), summed over the whole job.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4] [--mode batched|exact]
  N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "k8s-scheduler_amd"))

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X FP64 vector spec
BYTES_PER_PAIR = 24          # node alloc cpu/mem/pods int64 re-read per pod (sequential semantics)
FLOPS_PER_PAIR = 28          # 10 div + 18 add/sub/mul per resource-score pair
# PMC summaries of the same workloads (tools/pmc_summary.py over separate FETCH_SIZE / WRITE_SIZE / SQ
# passes of `bench.py` itself); keyed by (kernel, config, batch, ranks)
PMC_SUMMARIES = {
    ("k_pipe", "c4", 64, 1): os.path.join(ROOT, "profiles", "r06b_pmc_c4_pipe.json"),
    ("k_score_topk", "c4", 64, 1): os.path.join(ROOT, "profiles", "r01_pmc_c4_b64.json"),
}


def pmc_summary(kernel, config, batch, world):
    """HBM-side bytes per launch of `kernel` (FETCH_SIZE + WRITE_SIZE) and its VALU occupancy from the
    committed PMC passes, when they were taken on this workload; else None."""
    path = PMC_SUMMARIES.get((kernel, config, batch, world))
    if not path or not os.path.exists(path):
        return None
    with open(path) as f:
        k = json.load(f)["kernels"].get(kernel)
    if not k or "fabric_bytes_per_launch" not in k:
        return None
    with open(path) as f:
        src_commit = json.load(f).get("source_commit")
    out = {"traffic": k["fabric_bytes_per_launch"], "traffic_source": os.path.relpath(path, ROOT),
           "traffic_unit": "bytes per launch (2 x FETCH_SIZE + WRITE_SIZE)"}
    if src_commit:
        out["traffic_source_commit"] = src_commit
    for f in ("hbm_gbs", "valu_busy_frac", "fp64_issue_frac", "active_inst_valu_frac"):
        if f in k:
            out[f"pmc_{f}"] = k[f]
    c = k.get("counters_per_launch", {})
    for f in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
        if f in c:
            out[f"_{f}"] = c[f]
    if "f64_valu_insts_per_launch" in k:
        out["_F64"] = k["f64_valu_insts_per_launch"]
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c4")
    ap.add_argument("--mode", default="batched", choices=["batched", "exact"])
    ap.add_argument("--pods", type=int, default=None)
    ap.add_argument("--nodes", type=int, default=None)
    ap.add_argument("--topk", type=int, default=16)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--cpu-baseline-s", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the (untimed) prefix check of the timed run's results against the CPU oracle")
    ap.add_argument("--check-pods", type=int, default=5000)
    ap.add_argument("--no-xchg", action="store_true", help="N > 1: RCCL stream pipeline instead of the device-side exchange")
    return ap.parse_args()


def host_cpu():
    """(threads this process may use, CPU model name) -- the host side of the cpu_baseline line."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():  # the GPU box grants a 16-thread CPU share
        n = min(n, int(os.environ["OMP_NUM_THREADS"]))
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return max(1, n), model


def cpu_baseline(cl, budget_s):
    """The oracle's sequential C restatement (single thread, -O2 -ffp-contract=off), timed on this host
    on a bounded prefix of the same workload: the first p pods at full node count (per-pod cost is
    constant in the pod index).  Then the same restatement node-parallel on every thread this process
    may use (OpenMP, one barrier per pod)."""
    nthr, model = host_cpu()
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.lib()
    p = 16
    t = 0.0
    while True:
        t0 = time.perf_counter()
        O.schedule(cl, nthreads=1, n_pods=p)
        t = time.perf_counter() - t0
        if t > budget_s / 4 or p >= cl.n_pods:
            break
        p = min(cl.n_pods, int(p * max(2.0, budget_s / 3 / max(t, 1e-3))))
    rate = p * cl.n_nodes / t
    mt = None
    try:
        pm = max(16, min(cl.n_pods, int(p * max(2, nthr // 2))))
        t0 = time.perf_counter()
        O.schedule(cl, nthreads=nthr, n_pods=pm)
        tm = time.perf_counter() - t0
        mt = dict(value=pm * cl.n_nodes / tm, unit="pod-node evals/s", cores=nthr, kind="port", cpu_model=model,
                  sample=f"first {pm} pods of {cl.name} at {cl.n_nodes} nodes, OpenMP node-parallel on {nthr} threads "
                         f"(all this process may use), one barrier per pod ({tm:.1f} s)")
    except Exception:
        pass
    return dict(value=rate, unit="pod-node evals/s", cores=1, kind="port", cpu_model=model,
                sample=f"first {p} pods of {cl.name} at full {cl.n_nodes} nodes, sequential commit, 1 thread "
                       f"({t:.1f} s; Go reference unbuildable here: no Go toolchain)"), mt


def main():
    args = parse()
    from ksched import MODE_BATCHED, MODE_EXACT, cluster
    from ksched.dist import env_rank, make_sharded_engine
    rank, world, local = env_rank()
    world = max(world, 1)
    if world != args.gpus and args.gpus > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    dist = None
    tdev = "cuda"
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import torch

    cl = cluster.make_cluster(args.config, n_nodes=args.nodes, n_pods=args.pods)
    mode = MODE_EXACT if args.mode == "exact" else MODE_BATCHED
    if world > 1 and mode == MODE_EXACT:
        mode = MODE_BATCHED
    # N > 1: the persistent pipeline with the device-side exchange over xGMI (ksched_xchg_*), the RCCL
    # communicator kept as the fallback transport (stream pipeline, one all-gather per batch)
    eng, (lo, hi) = make_sharded_engine(cl, rank, world, device=local, mode=mode, topk=args.topk,
                                        batch=args.batch, timing=False, xchg=world > 1 and not args.no_xchg)
    eng.save_state()
    eng.upload_pods(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)

    def step():
        """One schedulePods pass: restore the initial node state on device, resolve every pending pod
        in order, wait, and bring the assignments back to the host (the wall ends with
        assignments-on-host)."""
        eng.restore_state()
        eng.run()
        eng.sync()
        return eng.results()

    step_stats = []
    from ksched import KschedError
    for w in range(max(args.warmup, 1 if world > 1 else 0)):
        if world > 1 and w == 0:
            # every rank must take the same transport: if the device exchange failed anywhere (a device
            # timeout), every rank turns it off (ksched_xchg_close) and the RCCL stream pipeline runs
            ok = 1
            try:
                step()
            except KschedError as ex:
                ok = 0
                print(f"rank {rank}: device-side exchange failed ({ex}); falling back to RCCL", file=sys.stderr)
            t = torch.tensor([ok], dtype=torch.int32, device=tdev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            if int(t.item()) == 0:
                eng.xchg_close()
                step()
        else:
            step()
    pipeline = eng.stats()["pipeline"]
    persistent = pipeline == "persistent"
    # the persistent pipeline is ONE score-grid launch per step: its HIP events (on the grid's own
    # stream) cost nothing per batch, so the roofline's launch durations come from the timed steps
    # themselves.  The stream pipeline samples per-batch events in one extra untimed pass instead.
    if persistent:
        eng.set_timing(True, 1)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
        if persistent:
            step_stats.append(eng.stats())
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = elapsed * 1000.0 / args.steps
    pairs = cl.n_pods * cl.n_nodes
    value = pairs * args.steps / elapsed
    st = step_stats[-1] if step_stats else eng.stats()
    if persistent and step_stats:
        eng.set_timing(False)
        kstats = step_stats
    else:
        eng.set_timing(True, 8)
        step()
        kstats = [eng.stats()]
        eng.set_timing(False)
    names = (["k_exact"] if mode == MODE_EXACT else ["k_pipe" if persistent else "k_score_topk"]) + \
        ["k_merge", "k_commit", "rccl_allgather+merge"]
    fam_ms = [sum(s["kernel_ms"][f] for s in kstats) for f in range(4)]
    fam_n = [sum(s["kernel_launches"][f] for s in kstats) for f in range(4)]
    score_pairs = sum(s["kernel_pairs"][0] for s in kstats)
    score_avg_ms = fam_ms[0] / max(fam_n[0], 1)
    score_pairs_per_launch = score_pairs / max(fam_n[0], 1)
    achieved_gbs = score_pairs_per_launch * BYTES_PER_PAIR / (score_avg_ms * 1e-3) / 1e9 if score_avg_ms > 0 else 0.0
    pmc = pmc_summary(names[0], args.config, int(eng.opts.batch) or 8 * args.topk, world)
    fam_share = {names[f]: (fam_ms[f] / max(fam_n[f], 1)) for f in range(4) if fam_n[f]}
    placed = int(st["placed"])
    roof = {
        "kernel": names[0],
        "bound": "hbm",
        "achieved": achieved_gbs,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": achieved_gbs / HBM_PEAK_GBS,
        "traffic": pmc.get("traffic") if pmc else None,
        "algorithmic_bytes_per_pair": BYTES_PER_PAIR,
        "pairs_per_launch": score_pairs_per_launch,
        "avg_launch_ms": score_avg_ms,
        "launches_timed": fam_n[0],
        "timing": "HIP events on the kernel's stream, inside the timed steps" if persistent else
                  "HIP events on the score stream, one batch in 8 of one untimed pass",
    }
    if pmc:
        roof.update({k: v for k, v in pmc.items() if k != "traffic" and not k.startswith("_")})
    if persistent and mode == MODE_BATCHED:
        # What actually binds: the 24 B/pair HBM figure above is SURVEY 8d's
        # bookkeeping -- node rows live in LDS for the whole call, so the score scan moves ~no HBM bytes
        # (traffic, from the FETCH_SIZE/WRITE_SIZE passes, is the merge handoff and control words).  The
        # VALU figures are the SQ passes' counts per launch over the launch's pairs (a wave64 instruction
        # covers 64 pairs: lane = pod); the call is bound by the lagged dependency chain
        # score -> merge -> commit -> score of a later batch.
        # the screened scan scores only its survivors in f64: the algorithmic figure counts every
        # pair of the sequential semantics; exact_rows_frac says how many of them the kernel evaluated in f64
        exact_frac = (st.get("exact_rows", 0) / st["scan_rows"]) if st.get("scan_rows") else None
        lim = {
            "what": "lagged dependency chain (score -> merge -> commit -> later score); VALU issue latency",
            "fp64_tflops_algorithmic": value / max(world, 1) * FLOPS_PER_PAIR / 1e12,
            "fp64_peak_tflops": FP64_VALU_PEAK_TFLOPS,
            "exact_rows_frac": exact_frac,
            "fp64_tflops_executed": (value / max(world, 1) * FLOPS_PER_PAIR / 1e12 * exact_frac) if exact_frac else None,
        }
        if pmc and score_pairs_per_launch > 0:
            for f, name in (("_SQ_INSTS_VALU", "valu"), ("_F64", "fp64_valu"), ("_SQ_INSTS_SALU", "salu"),
                            ("_SQ_INSTS_LDS", "lds")):
                if f in pmc:
                    lim[f"{name}_lane_insts_per_pair"] = pmc[f] * 64 / score_pairs_per_launch
            lim["source"] = pmc["traffic_source"]
        roof["bound_note"] = "bookkeeping: SURVEY 8d's 24 B/pair node re-read; the rows are LDS-resident"
        roof["limiter"] = lim
    out = {
        "metric": "pod-node evaluations/sec",
        "value": value,
        "unit": "pod-node evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": f"{args.config}: {cl.n_pods} pending pods x {cl.n_nodes} nodes, "
                               f"{'resource (balanced+least-requested)' if cl.priority == 0 else 'best-price'} priority, "
                               f"{'feasible-only' if cl.domain else 'all-node'} argmax, labels={bool(cl.use_labels)}",
                   "nodes": cl.n_nodes, "pods": cl.n_pods, "mode": args.mode, "topk": args.topk,
                   "batch": int(eng.opts.batch) or 8 * args.topk, "parallelism": f"node-shard x{world}",
                   "pipeline": pipeline, "transport": ("xgmi-rings" if pipeline == "persistent" else "rccl-allgather")
                                                       if world > 1 else "none"},
        "pods_per_sec": cl.n_pods * args.steps / elapsed,
        "placed_pods": placed,
        "placed_pods_per_sec": placed * args.steps / elapsed,
        "batches_per_step": int(st["batches"]),
        "truncated_batches_per_step": int(st["truncations"]),
        "rescued_lists_per_step": int(st.get("rescues", 0)),
        "kernel_avg_ms": fam_share,
        "roofline": roof,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        base, mt = cpu_baseline(cl, args.cpu_baseline_s)
        out["cpu_baseline"] = base
        if mt:
            out["cpu_baseline_mt"] = mt
    if not args.no_check and rank == 0:
        # the timed run's own results, prefix against the CPU oracle (pods resolve in order, so the
        # first k results of the full run are the results of a k-pod run); outside the timed region
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        oi, os_, of = res
        k = min(cl.n_pods, args.check_pods)
        wi, ws, wf, _ = O.schedule(cl, nthreads=host_cpu()[0], n_pods=k)
        out["check_prefix_pods"] = k
        out["check_ok"] = bool(np.array_equal(oi[:k], wi) and np.array_equal(os_[:k].view(np.int64), ws.view(np.int64))
                               and np.array_equal(of[:k], wf))
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
