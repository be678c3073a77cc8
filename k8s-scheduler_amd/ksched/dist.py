"""Node-sharded multi-GPU scheduling (one process per GPU).

The node list is cut into contiguous shards, one per rank (global index = shard offset + local
index, so the lowest-index tie-break is unchanged).  Every rank scores all pending pods against its
shard; per speculative batch the ranks exchange their local top-K candidate records (with the
candidates' snapshot node state) by ONE RCCL all-gather issued inside the engine, merge them
identically, and replay the same ordered commit -- each rank writes back only the nodes it owns.
Two exchange transports: the persistent pipeline's device-side exchange (ksched_xchg_*: merger
workgroups write every pod's list straight into each rank's receive ring over xGMI, no launch per
batch), or one RCCL all-gather per batch in the stream pipeline.  torch.distributed only hands out
the 128-byte RCCL unique id and the 128-byte ring handles (IPC handle + epoch hint).
"""
from __future__ import annotations

import os
from typing import Tuple

import numpy as np


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) of n nodes for `rank` of `world` (sizes differ by at most one)."""
    lo = n * rank // world
    hi = n * (rank + 1) // world
    return lo, hi


def env_rank() -> Tuple[int, int, int]:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def broadcast_bytes(payload, rank: int, src: int = 0) -> bytes:
    """Broadcast a small bytes object from `src` over the default torch.distributed group."""
    import torch.distributed as dist
    obj = [payload if rank == src else None]
    dist.broadcast_object_list(obj, src=src)
    return obj[0]


def setup_exchange(eng, rank: int, world: int, pg=None) -> bool:
    """Device-side candidate exchange (ksched_xchg_*): every rank exports its receive ring's IPC handle,
    the handles are all-gathered over torch.distributed (`pg`, default group), every rank maps them.
    All ranks agree on the outcome: if any rank fails, every rank turns the exchange off again
    (ksched_xchg_close) and False is returned -- no two ranks ever run different transports."""
    import torch.distributed as dist
    ok, h = 1, b""
    try:
        h = eng.xchg_export()
    except Exception:
        ok = 0
    hs = [None] * world
    dist.all_gather_object(hs, (ok, h), group=pg)
    ok = int(all(x[0] for x in hs))
    if ok:
        try:
            eng.xchg_import([x[1] for x in hs])
        except Exception:
            ok = 0
    flags = [None] * world
    dist.all_gather_object(flags, ok, group=pg)
    agreed = all(flags)
    if not agreed:
        eng.xchg_close()
    return agreed


def make_sharded_engine(cl, rank: int, world: int, device: int, mode=None, group=None, comm: bool = True,
                        xchg: bool = False, pg=None, **kw):
    """Engine for this rank's node shard of cluster `cl`.  world > 1: joined to the other ranks by an
    RCCL communicator (one process per GPU, torch.distributed hands out the id; comm=False skips it), or
    -- `group` given -- by an in-process rank group (ranks as threads of this process on one device).
    xchg=True also sets up the device-side exchange of the persistent pipeline (setup_exchange);
    the returned engine's `xchg_ready` tells whether it took."""
    from . import _lib as L
    from .engine import Engine
    lo, hi = shard_range(cl.n_nodes, rank, world)
    if mode is None:
        mode = L.MODE_BATCHED if (world > 1 or cl.mode != "exact") else L.MODE_EXACT
    eng = Engine(mode=mode, priority=cl.priority, domain=cl.domain, use_labels=cl.use_labels, device=device,
                 rank=rank, nranks=world, node_offset=lo, nodes_global=cl.n_nodes, **kw)
    eng.load_nodes(cl.alloc_cpu[lo:hi], cl.alloc_mem[lo:hi], cl.alloc_pods[lo:hi],
                   labels=None if cl.labels is None else cl.labels[lo:hi],
                   price=None if cl.price is None else cl.price[lo:hi])
    if group is not None:
        eng.set_group(group)
    elif world > 1:
        if comm:
            uid = Engine.unique_id() if rank == 0 else None
            uid = broadcast_bytes(uid, rank)
            eng.set_comm(uid)
        if xchg and not setup_exchange(eng, rank, world, pg=pg) and not comm:
            raise RuntimeError("node-sharded engine: the device exchange could not be set up on every rank "
                               "and no RCCL communicator was requested (comm=False)")
    return eng, (lo, hi)


def gather_node_state(local_state, world: int):
    """Concatenate every rank's (cpu, mem, pods) node state in rank order (torch.distributed)."""
    import torch
    import torch.distributed as dist
    out = []
    for arr in local_state:
        t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int64))
        parts = [None] * world
        dist.all_gather_object(parts, t.numpy())
        out.append(np.concatenate(parts))
    return tuple(out)


def make_local_xchg_group(cl, world: int, device: int = 0, rings: str = "plain", **kw):
    """`world` node-sharded ranks of cluster `cl` as contexts of THIS process on ONE device, joined by the
    device-side exchange (ksched_xchg_join_local_ex; rings: "plain", "uncached" = xchg_export's ring kind, "ipc" =
    also mapped through IPC handles): their persistent kernels run as one cooperative launch, so all ranks'
    grids are resident at once.  The caller runs each rank's schedule calls in its own thread.  Returns
    [(engine, (lo, hi)) per rank]."""
    from . import _lib as L
    from .engine import Engine
    out = [make_sharded_engine(cl, r, world, device=device, mode=L.MODE_BATCHED, comm=False, **kw)
           for r in range(world)]
    Engine.xchg_join_local([e for e, _ in out], rings=rings)
    return out
