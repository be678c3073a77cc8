#!/usr/bin/env python3
"""Which teardown faults at process exit under rocprofv3?  Runs ONE variant of a small
GPU workload and, at Python exit (before the C-level exit handlers run, every library still mapped),
writes /proc/self/maps to gpurun_out/maps_<variant>.txt so the addresses of a crash report can be mapped to
their libraries.

  rocprofv3 --kernel-trace --stats -d gpurun_out/prof_<v> -o run -- python3 tests/diag/exit_probe.py <v>
variants: torch   torch only (one kernel)
          ksched  + libksched: one small batched schedule, context destroyed explicitly
          leak    + libksched: the same, context left to the interpreter's teardown
          oracle  + the OpenMP oracle (the check leg's checker)
          load    + libksched: a context created and destroyed, no kernel launched
          stream  + libksched: the batched schedule on the stream pipeline (plain launches only)
          exact   + libksched: the exact mode (one cooperative launch of k_exact)
          notorch libksched's batched schedule (persistent, cooperative) in a process that never imports torch:
                  libksched then runs on /opt/rocm's HIP runtime instead of the one bundled with torch
          reset   notorch + hipDeviceReset after the context is destroyed (before any exit handler)
          treset  ksched (with torch) + hipDeviceReset after the context is destroyed
"""
import atexit
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "k8s-scheduler_amd"), os.path.join(ROOT, "oracle")]


def dump_maps(v):
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open("/proc/self/maps") as f, open(os.path.join(ROOT, "gpurun_out", f"maps_{v}.txt"), "w") as o:
        o.write(f.read())


def main():
    v = sys.argv[1]
    atexit.register(dump_maps, v)
    if v not in ("notorch", "reset"):
        import torch
        x = torch.ones(1024, device="cuda")
        print("torch sum", float(x.sum()), flush=True)
    if v == "torch":
        return
    from ksched import MODE_BATCHED, MODE_EXACT, Engine, cluster
    cl = cluster.make_cluster("c3", n_nodes=4000, n_pods=300)
    if v == "load":
        Engine(mode=MODE_BATCHED, topk=16, batch=64, device=0).close()
        print("ksched context created and destroyed", flush=True)
        return
    kw = dict(mode=MODE_BATCHED, topk=16, batch=64)
    if v == "stream":
        kw["pipeline"] = 1  # KSCHED_PIPELINE_STREAM
    elif v == "exact":
        kw = dict(mode=MODE_EXACT)
    e = Engine(device=0, **kw)
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
    if v in ("reset", "treset"):
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime libksched is bound to (already loaded)
        print("hipDeviceSynchronize", hip.hipDeviceSynchronize(), "hipDeviceReset", hip.hipDeviceReset(), flush=True)


if __name__ == "__main__":
    main()
