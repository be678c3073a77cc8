#!/usr/bin/env python3
"""Which teardown faults at process exit under rocprofv3?  Runs ONE variant of a small
GPU workload and, at Python exit (before the C-level exit handlers run, every library still mapped),
writes /proc/self/maps to gpurun_out/maps_<variant>.txt so the addresses of a crash report can be mapped to
their libraries.

  rocprofv3 --kernel-trace --stats -d gpurun_out/prof_<v> -o run -- python3 tools/exit_probe.py <v>
variants: torch   torch only (one kernel)
          ksched  + libksched: one small batched schedule, context destroyed explicitly
          leak    + libksched: the same, context left to the interpreter's teardown
          oracle  + the OpenMP oracle (the check leg's checker)
"""
import atexit
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "k8s-scheduler_amd"), os.path.join(ROOT, "oracle")]


def dump_maps(v):
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open("/proc/self/maps") as f, open(os.path.join(ROOT, "gpurun_out", f"maps_{v}.txt"), "w") as o:
        o.write(f.read())


def main():
    v = sys.argv[1]
    atexit.register(dump_maps, v)
    import torch
    x = torch.ones(1024, device="cuda")
    print("torch sum", float(x.sum()), flush=True)
    if v == "torch":
        return
    from ksched import MODE_BATCHED, Engine, cluster
    cl = cluster.make_cluster("c3", n_nodes=4000, n_pods=300)
    e = Engine(mode=MODE_BATCHED, topk=16, batch=64, device=0)
    e.load_nodes(cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods)
    oi, _, _ = e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods)
    print("ksched placed", int((oi >= 0).sum()), e.stats()["pipeline"], flush=True)
    if v == "oracle":
        import oracle as O
        want = O.schedule(cl, nthreads=4)
        print("oracle agrees", bool((want[0] == oi).all()), flush=True)
    if v != "leak":
        e.close()
    else:
        globals()["_leaked"] = e


if __name__ == "__main__":
    main()
