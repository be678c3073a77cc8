"""CPU check of the commit kernel's re-scoring filter (ksched_device.h: resource_score_upper).

The filter replaces each a / b of the resource score with a * y, y ~ 1/b, and adds a margin; a touched
node is scored exactly only when that upper bound can reach the decision threshold.  It is sound iff
  (1) upper >= exact score whenever the balanced branch is not flagged "near 1", and
  (2) outside the flag, the branch (fraction >= 1) taken with approximate fractions equals the exact one.
This mirrors the device arithmetic in numpy (float64 ops, no FMA) with the reciprocals perturbed by up
to +-4 ulp -- the device's rcp + two Newton steps is within 1 ulp -- and checks both properties against
the oracle's exact score (oracle/cpu_ref.c:or_score, anchor/scores.go)."""
import numpy as np
import pytest


def _wsub(a, b):
    return (a.astype(np.uint64) - b.astype(np.uint64)).view(np.int64)  # Go int64 wrap-around


def _upper(rc, rm, rp, ac, am, ap, yc, ym, yp, y3):
    with np.errstate(all="ignore"):
        rcf, rmf, rpf = (x.astype(np.float64) for x in (rc, rm, rp))
        c = np.where(ac == 0, 1.0, rcf * yc)
        m = np.where(am == 0, 1.0, rmf * ym)
        p = np.where(ap == 0, 1.0, rpf * yp)
        near1 = ((ac != 0) & (np.abs(c - 1.0) < 1e-12)) | ((am != 0) & (np.abs(m - 1.0) < 1e-12)) | \
                ((ap != 0) & (np.abs(p - 1.0) < 1e-12))
        mean = ((c + m) + p) * y3
        var = (((c - mean) * (c - mean) + (m - mean) * (m - mean)) + (p - mean) * (p - mean)) * y3
        b = np.where((c >= 1.0) | (m >= 1.0) | (p >= 1.0), 0.0, (1.0 - var) * 10.0)
        dc, dm, dp = (_wsub(a, r).astype(np.float64) for a, r in ((ac, rc), (am, rm), (ap, rp)))
        lc = np.where((ac == 0) | (rc > ac), 0.0, dc * 10.0 * yc)
        lm = np.where((am == 0) | (rm > am), 0.0, dm * 10.0 * ym)
        lp = np.where((ap == 0) | (rp > ap), 0.0, dp * 10.0 * yp)
        l = ((lc + lm) + lp) * y3
        s = (b + l) * 0.5
        return s + 1e-9 * (np.abs(b) + np.abs(l) + 1.0), near1, (c >= 1) | (m >= 1) | (p >= 1)


def _cases(rng, n):
    def one_res(scale):
        a = rng.integers(-scale // 4, scale, n)
        kind = rng.integers(0, 6, n)
        r = rng.integers(0, scale, n)
        r = np.where(kind == 0, a, r)                       # exactly full
        r = np.where(kind == 1, a - rng.integers(0, 3, n), r)  # one or two below full
        r = np.where(kind == 2, a + 1, r)
        a = np.where(kind == 3, 0, a)                       # zero allocatable
        r = np.where(kind == 4, 0, r)
        return r.astype(np.int64), a.astype(np.int64)
    rc, ac = one_res(64_000)
    rm, am = one_res(1 << 36)
    rp, ap = one_res(120)
    big = rng.random(n) < 0.05
    ac = np.where(big, rng.integers(-(1 << 62), 1 << 62, n), ac)
    rc = np.where(big, rng.integers(0, 1 << 62, n), rc)
    return rc, rm, rp, ac, am, ap


def _exact(oracle_mod, rc, rm, rp, ac, am, ap):
    return np.array([oracle_mod.score(*t) for t in zip(rc.tolist(), rm.tolist(), rp.tolist(),
                                                       ac.tolist(), am.tolist(), ap.tolist())])


@pytest.mark.parametrize("seed", range(4))
def test_upper_bound_sound(oracle_mod, seed):
    rng = np.random.default_rng(1234 + seed)
    n = 40_000
    rc, rm, rp, ac, am, ap = _cases(rng, n)
    ex = _exact(oracle_mod, rc, rm, rp, ac, am, ap)
    with np.errstate(all="ignore"):
        inv = [np.where(a == 0, 0.0, 1.0 / a.astype(np.float64)) for a in (ac, am, ap)]
    for k in (-4, -1, 0, 1, 4):
        f = 1.0 + k * 2.0 ** -52
        yc, ym, yp = (y * f for y in inv)
        y3 = (1.0 / 3.0) * f
        hi, near1, br = _upper(rc, rm, rp, ac, am, ap, yc, ym, yp, y3)
        with np.errstate(all="ignore"):
            ec = np.where(ac == 0, 1.0, rc / np.where(ac == 0, 1, ac).astype(np.float64))
            em = np.where(am == 0, 1.0, rm / np.where(am == 0, 1, am).astype(np.float64))
            ep = np.where(ap == 0, 1.0, rp / np.where(ap == 0, 1, ap).astype(np.float64))
        ebr = (ec >= 1) | (em >= 1) | (ep >= 1)
        ok = near1 | (br == ebr)
        assert ok.all(), np.nonzero(~ok)[0][:5]
        sound = near1 | (hi >= ex)
        assert sound.all(), [(int(i), hi[i], ex[i]) for i in np.nonzero(~sound)[0][:5]]
        # and the filter is tight enough to reject: margin is tiny relative to the score scale
        slack = (hi - ex)[~near1]
        scale = 1e-8 * (np.abs(ex[~near1]) + 10.0)
        assert (slack <= scale).mean() > 0.999
