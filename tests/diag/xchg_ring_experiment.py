#!/usr/bin/env python3
"""DESIGN.md section 6.1's experiment on the round-4 exchange failure: a sequence of local rank groups (two ranks
on c3, three on c4 30k nodes, two on c4 100k nodes -- the order that failed), in a fresh process per variant, each
group checked against the oracle.  Variants change one thing at a time: the ring memory, how a ring is zeroed
(KSCHED_XCHG_DIAG=1: hipMemsetAsync as in round 4), whether tags restart at 1 (KSCHED_XCHG_DIAG=2), the history
(the last group alone), poisoned workspace and LDS (KSCHED_POISON), the screened scan (KSCHED_NO_SCREEN).

  python tests/diag/xchg_ring_experiment.py [variant ...]     (one subprocess per variant; default: all)

The *_dump variants need the diagnostics build (the device-side dumps are compiled out of the product):
  bash tools/build_variant.sh xdbg "-DKSCHED_XCHG_DEBUG=1"     -> k8s-scheduler_amd/libksched_xdbg.so
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SEQ = (("c3", 24000, 3000, 2), ("c4", 30000, 2500, 3), ("c4", 100000, 2500, 2))
XDBG = {"KSCHED_LIB": os.path.join(ROOT, "k8s-scheduler_amd", "libksched_xdbg.so")}
VARIANTS = {
    "uncached": ({}, "uncached", SEQ),
    "uncached_memset_tags1": ({"KSCHED_XCHG_DIAG": "3"}, "uncached", SEQ),
    "plain": ({}, "plain", SEQ),
    "uncached_alone": ({}, "uncached", SEQ[-1:]),
    "uncached_poison": ({"KSCHED_POISON": "1"}, "uncached", SEQ),
    "plain_poison": ({"KSCHED_POISON": "1"}, "plain", SEQ),
    "uncached_nosdma": ({"HSA_ENABLE_SDMA": "0"}, "uncached", SEQ),
    "single_poison": ({"KSCHED_POISON": "1"}, "single", (("c4", 100000, 2500, 1),)),
    "uncached_noscreen": ({"KSCHED_NO_SCREEN": "1"}, "uncached", SEQ),
    "uncached_norescue": ({"KSCHED_RESCUE_MAX": "0"}, "uncached", SEQ),
    "plain_dump": ({"KSCHED_XCHG_DUMP": "gpurun_out/xd_plain", **XDBG}, "plain", SEQ),
    "plain_norescue_dump": ({"KSCHED_XCHG_DUMP": "gpurun_out/xd_plain_nr", "KSCHED_RESCUE_MAX": "0", **XDBG}, "plain", SEQ),
    "uncached_norescue_dump": ({"KSCHED_XCHG_DUMP": "gpurun_out/xd_uncached_nr", "KSCHED_RESCUE_MAX": "0",
                                "XCHG_REF_DUMP": "gpurun_out/xd_plain_nr", **XDBG}, "uncached", SEQ),
    "uncached_dump": ({"KSCHED_XCHG_DUMP": "gpurun_out/xd_uncached", "XCHG_REF_DUMP": "gpurun_out/xd_plain", **XDBG},
                      "uncached", SEQ),
}


def load_dump(prefix: str, r: int, c: int, world: int, B: int = 64, K: int = 16):
    """One rank's KSCHED_XCHG_DUMP file: ([active batches][B][R + 1] hashes, [8][B][MW] sent messages)."""
    import numpy as np
    MW = K * 14 + 2
    a = np.fromfile(f"{prefix}.r{r}.c{c}", dtype=np.uint64)
    nm = (16 * B * MW + 1) // 2
    cap = (a.size - nm) // (B * (world + 3) + 16)
    h = a[:cap * B * (world + 1)].reshape(cap, B, world + 1)
    msg = a[cap * B * (world + 1):cap * B * (world + 1) + nm].view(np.uint32)[:16 * B * MW].reshape(16, B, MW)
    o = cap * B * (world + 1) + nm
    sums = a[o:o + cap * B * 2].reshape(cap, B, 2)
    commit = a[o + cap * B * 2:o + cap * B * 2 + cap * 8].reshape(cap, 8)
    resc = a[o + cap * B * 2 + cap * 8:].reshape(cap, 8)
    return h, msg, sums, np.concatenate([commit, resc], axis=1)


def commit_check(pa: str, pb: str, world: int, B: int = 64):
    """Per active batch the commits' summaries: the first batch where the ranks (of run pa) differ, and the first
    where run pa differs from run pb (same rank), with both summaries."""
    import numpy as np
    ca = [load_dump(pa, r, 0, world, B)[3] for r in range(world)]
    out = {}
    def desc(x):
        x = [int(v) for v in x]
        return dict(p0=x[0], done=x[1] & 0xffff, resc=(x[1] >> 16) & 0xffff, rounds=(x[1] >> 32) & 0xffff,
                    fails=x[1] >> 48, n1=x[2] & 0xffff, n2=(x[2] >> 16) & 0xffff, nin=(x[2] >> 32) & 0xffff,
                    nexp=x[2] >> 48, out=hex(x[3]), x1=hex(x[4]), batch=x[7],
                    rescues=[(x[8 + 2 * i] & 0xffffffff, x[8 + 2 * i] >> 32,
                              float(np.array([x[9 + 2 * i]], dtype=np.uint64).view(np.float64)[0])) for i in range(4)])
    for r in range(1, world):
        d = np.argwhere((ca[0] != ca[r]).any(1))
        if len(d):
            a = int(d[0][0])
            out[f"ranks0v{r}"] = dict(act=a, r0=desc(ca[0][a]), rr=desc(ca[r][a]), prev0=desc(ca[0][a - 1]) if a else None)
    if pb and os.path.exists(f"{pb}.r0.c0"):
        cb = load_dump(pb, 0, 0, world, B)[3]
        n = min(len(cb), len(ca[0]))
        d = np.argwhere((ca[0][:n] != cb[:n]).any(1))
        if len(d):
            a = int(d[0][0])
            out["run_vs_ref"] = dict(act=a, run=desc(ca[0][a]), ref=desc(cb[a]), prev_run=desc(ca[0][a - 1]) if a else None,
                                     prev_ref=desc(cb[a - 1]) if a else None)
    return out


def handoff_check(prefix: str, world: int, B: int = 64, calls: int = 2):
    """Per rank: the (active batch, pod) whose merged list as the commit loaded it differs from the list as the
    merger wrote it (a list the commit read before, or apart from, what was written)."""
    import numpy as np
    out = []
    for c in range(calls):
        for r in range(world):
            sums = load_dump(prefix, r, c, world, B)[2]
            live = (sums[:, :, 0] != 0) | (sums[:, :, 1] != 0)
            d = np.argwhere(live & (sums[:, :, 0] != sums[:, :, 1]))
            out.append(dict(call=c, rank=r, lists=int(live.sum()), differ=int(len(d)), first=d[:6].tolist()))
    return out


def delivery(prefix: str, world: int, B: int = 64, calls: int = 2):
    """KSCHED_XCHG_DUMP's message hashes of the last group: for every (active batch, pod), did each rank receive
    from rank q exactly what rank q sent?  Returns the first mismatches."""
    import numpy as np
    bad = []
    for c in range(calls):
        d = [load_dump(prefix, r, c, world, B)[0] for r in range(world)]
        sent = [d[r][:, :, world] for r in range(world)]
        for r in range(world):
            for q in range(world):
                got = d[r][:, :, q]
                live = (got != 0) | (sent[q] != 0)
                mism = np.argwhere(live & (got != sent[q]))
                if len(mism):
                    bad.append(dict(call=c, rank=r, src=q, mismatches=int(len(mism)), first=mism[:4].tolist()))
    return bad


def compare_sent(pa: str, pb: str, world: int, B: int = 64, K: int = 16):
    """The first (rank, active batch, pod) whose sent message differs between two runs' dumps, with both lists."""
    import numpy as np

    def recs(m):
        w = m[:K * 14].reshape(K, 14)
        out = []
        for q in range(K):
            key = float(np.array([w[q, 0], w[q, 1]], dtype=np.uint32).view(np.float64)[0])
            a = [int(np.array([w[q, 4 + 2 * i], w[q, 5 + 2 * i]], dtype=np.uint32).view(np.int64)[0]) for i in range(3)]
            out.append([int(w[q, 3]), int(w[q, 2]), key, a, int(w[q, 13])])
        fc = int(np.array([m[K * 14], m[K * 14 + 1]], dtype=np.uint32).view(np.int64)[0])
        return out, fc
    for r in range(world):
        ha, ma, _, _ = load_dump(pa, r, 0, world, B, K)
        hb, mb, _, _ = load_dump(pb, r, 0, world, B, K)
        n = min(ha.shape[0], hb.shape[0])
        d = np.argwhere(ha[:n, :, world] != hb[:n, :, world])
        if len(d):
            a, m = (int(x) for x in d[0])
            res = dict(rank=r, batch=a, pod=m, differing=int(len(d)))
            if a < 16:
                res["a"], res["b"] = recs(ma[a, m]), recs(mb[a, m])
            return res
    return None


def alias_check(rings: str, world_seq=SEQ, run: bool = False):
    """The node rows read back after load and again after the rings' setup, per group of the sequence: a ring
    allocation that aliases another buffer shows as rows changed by the join (its zeroing)."""
    import numpy as np
    from ksched import cluster
    from ksched.dist import make_sharded_engine
    from ksched.engine import Engine
    import ksched._lib as L
    out = []
    for cfg, nn, pp, world in world_seq:
        cl = cluster.make_cluster(cfg, n_nodes=nn, n_pods=pp)
        eng = [make_sharded_engine(cl, r, world, device=0, mode=L.MODE_BATCHED, comm=False, topk=16, batch=64)
               for r in range(world)]
        before = [bool(all(np.array_equal(x, a[lo:hi]) for x, a in zip(e.read_nodes(), (cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods))))
                  for (e, (lo, hi)) in eng]
        Engine.xchg_join_local([e for e, _ in eng], rings=rings)
        after = [bool(all(np.array_equal(x, a[lo:hi]) for x, a in zip(e.read_nodes(), (cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods))))
                 for (e, (lo, hi)) in eng]
        rec = dict(group=f"{cfg}/{nn}/R{world}", load_ok=before, after_join_ok=after)
        if run:  # the group's schedule calls, as the failing sequence makes them
            import threading
            res = [None] * world

            def work(r):
                e = eng[r][0]
                e.save_state()
                e.restore_state()
                res[r] = e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)[0]
            th = [threading.Thread(target=work, args=(r,)) for r in range(world)]
            for t in th:
                t.start()
            for t in th:
                t.join(timeout=150)
            rec["after_run_ok"] = [bool(all(np.array_equal(x, a[lo:hi]) for x, a in
                                            zip(eng[r][0].read_nodes(), (cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods))))
                                   for r, (e, (lo, hi)) in enumerate(eng)]
        out.append(rec)
        Engine.close_group([e for e, _ in eng])
    return out


def one(name: str) -> None:
    if name.startswith("alias_"):
        env = {"HSA_ENABLE_SDMA": "0"} if name.endswith("_nosdma") else {}
        os.environ.update(env)
        sys.path[:0] = [os.path.join(ROOT, "k8s-scheduler_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
        rings = name.split("_")[1]
        print(json.dumps(dict(variant=name, env=env, alias=alias_check(rings, run="_run" in name))), flush=True)
        return
    env, rings, seq = VARIANTS[name]
    os.environ.update(env)
    sys.path[:0] = [os.path.join(ROOT, "k8s-scheduler_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    import oracle as O
    from ksched import cluster
    from test_gpu_xchg import run_local
    res = []
    for cfg, nn, pp, world in seq:
        cl = cluster.make_cluster(cfg, n_nodes=nn, n_pods=pp)
        want = O.schedule(cl, nthreads=8)
        if rings == "single":  # one rank, no exchange (the same check)
            from ksched import Engine, MODE_BATCHED
            with Engine(mode=MODE_BATCHED, priority=cl.priority, domain=cl.domain, device=0, topk=16, batch=64) as e:
                e.load_nodes(cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods)
                e.save_state()
                res1 = []
                for _ in range(2):
                    e.restore_state()
                    oi, _, _ = e.schedule(cl.req_cpu, cl.req_mem, cl.req_pods)
                    st = e.stats()
                    res1.append((oi, None, None, st["pipeline"], st["batches"], st["truncations"], 0, st["rescues"]))
                out = [(res1, None)]
        else:
            out = run_local(cl, world, rings=rings)
        bad = max(int((x[0] != want[0]).sum()) for r in range(world) for x in out[r][0])
        first = min((int((x[0] != want[0]).nonzero()[0][0]) for r in range(world) for x in out[r][0]
                     if (x[0] != want[0]).any()), default=-1)
        if "KSCHED_XCHG_DUMP" in env:
            import numpy as np
            np.save(env["KSCHED_XCHG_DUMP"] + ".out.npy", np.stack([out[r][0][0][0] for r in range(world)] + [want[0]]))
        res.append(dict(group=f"{cfg}/{nn}/R{world}", differ=bad, first=first, batches=[x[4] for x in out[0][0]],
                        truncated=[x[5] for x in out[0][0]], rescues=[x[7] for x in out[0][0]]))
    extra = {}
    if "KSCHED_XCHG_DUMP" in env:
        extra["delivery"] = delivery(env["KSCHED_XCHG_DUMP"], seq[-1][3], 64)
        extra["handoff"] = handoff_check(env["KSCHED_XCHG_DUMP"], seq[-1][3], 64)
        ref = os.environ.get("XCHG_REF_DUMP")
        if ref and os.path.exists(f"{ref}.r0.c0"):
            extra["vs_ref"] = compare_sent(env["KSCHED_XCHG_DUMP"], ref, seq[-1][3])
        extra["commits"] = commit_check(env["KSCHED_XCHG_DUMP"], ref, seq[-1][3])
    print(json.dumps(dict(variant=name, env=env, rings=rings, groups=res, **extra)), flush=True)


def main() -> int:
    if len(sys.argv) > 2 and sys.argv[1] == "--one":
        one(sys.argv[2])
        return 0
    rc = 0
    for name in sys.argv[1:] or list(VARIANTS):
        name = name.split(":")[0]
        if not name.startswith("alias_") and name not in VARIANTS:
            raise SystemExit(f"unknown variant {name}")
        r = subprocess.run([sys.executable, "-u", __file__, "--one", name], timeout=300)
        rc |= r.returncode
    return rc


if __name__ == "__main__":
    sys.exit(main())
