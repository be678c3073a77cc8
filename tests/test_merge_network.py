"""The merge's wave sort (k8s-scheduler_amd/csrc/ksched_merge.h wave_sort_desc) as a network over 64 lanes, checked
on the CPU: the "flip" form of the bitonic sorter -- stage (M, HB) compares lane l with lane l ^ M and the lane with
bit HB clear keeps the better pair -- sorts any 64 (code, idx) pairs best first (code desc, idx asc), and its
tail (the stages above block size RUN) merges lanes that hold sorted runs of RUN.  The device builds every partner
from DPP / permlane moves; the identities it relies on (xor 4 = xor 7 then xor 3, xor 31 = 15 then 16, xor 63 =
15, 16 then 32; the row mirrors are xor 7 and xor 15) are checked here too.  The device code itself is covered by
every GPU parity test (the merged lists decide every batched result)."""
import random

import pytest


def better(a, b):
    return a[0] > b[0] or (a[0] == b[0] and a[1] < b[1])


# (M, HB) per stage, in the order of wave_sort_desc; block size 2^k starts with the flip M = 2^k - 1
STAGES = {
    1: [(1, 1)],
    2: [(3, 2), (1, 1)],
    4: [(7, 4), (2, 2), (1, 1)],
    8: [(15, 8), (4, 4), (2, 2), (1, 1)],
    16: [(31, 16), (8, 8), (4, 4), (2, 2), (1, 1)],
    32: [(63, 32), (16, 16), (8, 8), (4, 4), (2, 2), (1, 1)],
}


def network(run):
    """The stages wave_sort_desc<RUN> runs: those of every block size above RUN."""
    return [st for k in (1, 2, 4, 8, 16, 32) if k >= run for st in STAGES[k]]


def apply(v, stages):
    v = list(v)
    for m, hb in stages:
        p = [v[l ^ m] for l in range(64)]
        out = []
        for l in range(64):
            pb = better(p[l], v[l])
            take = (not pb) if (l & hb) else pb
            out.append(p[l] if take else v[l])
        v = out
    return v


def rand_pairs(rng, kind):
    empty = (0, 0x7FFFFFFF)
    if kind == "random":
        return [(rng.randrange(1, 1 << 63), i) for i in rng.sample(range(10 ** 6), 64)]
    if kind == "ties":  # a zero-request pod: every key equal, the order is the node index
        c = rng.randrange(1, 1 << 63)
        return [(c, i) for i in rng.sample(range(10 ** 6), 64)]
    if kind == "few":  # a handful of distinct keys
        cs = [rng.randrange(1, 1 << 63) for _ in range(3)]
        return [(rng.choice(cs), i) for i in rng.sample(range(10 ** 6), 64)]
    n = rng.randrange(0, 64)  # empty lists sort last
    return [(rng.randrange(1, 1 << 63), i) for i in rng.sample(range(10 ** 6), n)] + [empty] * (64 - n)


def test_stage_count():
    assert len(network(1)) == 21
    assert len(network(16)) == 11


@pytest.mark.parametrize("kind", ["random", "ties", "few", "empties"])
def test_network_sorts(kind):
    rng = random.Random(7)
    for _ in range(300):
        v = rand_pairs(rng, kind)
        rng.shuffle(v)
        got = apply(v, network(1))
        assert sorted(got) == sorted(v), "not a permutation"
        assert all(not better(got[l + 1], got[l]) for l in range(63))


@pytest.mark.parametrize("run", [2, 4, 8, 16, 32])
def test_network_merges_sorted_runs(run):
    """Phase B: the W waves' K best heads arrive as sorted runs of K (empty slots last in each run)."""
    rng = random.Random(run)
    key = lambda p: (-p[0], p[1])
    for _ in range(300):
        v = rand_pairs(rng, rng.choice(["random", "ties", "few", "empties"]))
        rng.shuffle(v)
        runs = []
        for r in range(0, 64, run):
            runs += sorted(v[r:r + run], key=key)
        got = apply(runs, network(run))
        assert got == sorted(v, key=key)


def test_partner_identities():
    for l in range(64):
        assert l ^ 4 == (l ^ 7) ^ 3
        assert l ^ 31 == (l ^ 15) ^ 16
        assert l ^ 63 == ((l ^ 15) ^ 16) ^ 32
        row, half = l & ~15, l & ~7
        assert l ^ 15 == row + (15 - (l & 15))  # row_mirror
        assert l ^ 7 == half + (7 - (l & 7))  # row_half_mirror
        assert l ^ 8 == row + ((l + 8) & 15)  # row_ror:8
        assert l ^ 3 == (l & ~3) + (3 - (l & 3))  # quad_perm [3,2,1,0]
