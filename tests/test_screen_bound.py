"""The f32 screen of the screened scan (csrc/ksched_device.h screen_score) against
the reference's f64 resource score.

The screen never decides a result: a pair is skipped only when screen + kScreenEps < L, L being a lower
bound (screen - kScreenEps) of KC eligible keys of the same workgroup.  That is sound iff
|screen - score| < kScreenEps for every fitting pair whose fractions are all < 1, and screen + kScreenEps
>= score for fitting pairs with a fraction of exactly 1 (balanced part 0).  numpy's float32 arithmetic is
IEEE round-to-nearest like the device's (no contraction: the library builds with -ffp-contract=off), so
the emulation below is the device computation bit for bit.
"""
import numpy as np
import pytest

EPS = np.float32(1e-4)      # kScreenEps
BOUND = 1.3e-5              # the error bound DESIGN.md derives (the test also reports the worst case seen)
F = np.float32


def screen_req(r):
    r = np.asarray(r, dtype=np.int64)
    out = r.astype(np.float32)
    out[(r < 0) | (r >= (1 << 52))] = np.nan
    return out


def screen_recip(a):
    a = np.asarray(a, dtype=np.int64)
    with np.errstate(divide="ignore"):
        out = (1.0 / a.astype(np.float64)).astype(np.float32)
    out[(a <= 0) | (a >= (1 << 52))] = np.nan
    return out


def screen_score(rc, rm, rp, ac, am, ap):
    qc, qm, qp = screen_req(rc), screen_req(rm), screen_req(rp)
    yc, ym, yp = screen_recip(ac), screen_recip(am), screen_recip(ap)
    with np.errstate(all="ignore"):
        c, m, p = qc * yc, qm * ym, qp * yp
        fmax = np.fmax(np.fmax(c, m), p)
        S = (c + m) + p
        Q = (c * c + m * m) + p * p
        s = ((F(10.0) - (F(5.0) / F(3.0)) * S) - (F(5.0) / F(3.0)) * Q) + (F(5.0) / F(9.0)) * (S * S)
    return s.astype(np.float32), fmax


def exact_score(rc, rm, rp, ac, am, ap):
    """anchor/priorities.go:5-23,45-50 + scores.go:3-25 in the reference's f64 operation order."""
    rcf, rmf, rpf = (np.asarray(x, np.int64).astype(np.float64) for x in (rc, rm, rp))
    acf, amf, apf = (np.asarray(x, np.int64).astype(np.float64) for x in (ac, am, ap))
    with np.errstate(all="ignore"):
        c = np.where(acf == 0, 1.0, rcf / acf)
        m = np.where(amf == 0, 1.0, rmf / amf)
        p = np.where(apf == 0, 1.0, rpf / apf)
        mean = ((c + m) + p) / 3.0
        var = (((c - mean) * (c - mean) + (m - mean) * (m - mean)) + (p - mean) * (p - mean)) / 3.0
        b = np.where((c >= 1) | (m >= 1) | (p >= 1), 0.0, (1.0 - var) * 10.0)
        lc = np.where((acf == 0) | (rcf > acf), 0.0, ((acf - rcf) * 10.0) / acf)
        lm = np.where((amf == 0) | (rmf > amf), 0.0, ((amf - rmf) * 10.0) / amf)
        lp = np.where((apf == 0) | (rpf > apf), 0.0, ((apf - rpf) * 10.0) / apf)
        l = ((lc + lm) + lp) / 3.0
        return ((0.0 + b) + l) / 2.0


def _pairs(rng, n):
    """Fitting pairs (0 <= r <= a < 2^52) over every magnitude, plus near-1 and zero fractions."""
    def mag(size):
        e = rng.uniform(0, 51.9, size)
        return np.maximum(1, (2.0 ** e)).astype(np.int64)
    a = np.stack([mag(n), mag(n), mag(n)])
    frac = rng.random((3, n))
    kind = rng.integers(0, 6, (3, n))
    frac = np.where(kind == 0, 0.0, frac)                       # zero request
    frac = np.where(kind == 1, 1.0 - rng.random((3, n)) * 1e-9, frac)  # fraction just below 1
    frac = np.where(kind == 2, rng.random((3, n)) * 1e-6, frac)  # tiny fraction
    r = np.minimum(a, np.floor(frac * a).astype(np.int64))
    eq = rng.random((3, n)) < 0.02
    r = np.where(eq, a, r)                                       # fraction exactly 1
    return r, a


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_screen_error_below_eps(seed):
    rng = np.random.default_rng(seed)
    r, a = _pairs(rng, 400_000)
    s32, fmax = screen_score(r[0], r[1], r[2], a[0], a[1], a[2])
    s64 = exact_score(r[0], r[1], r[2], a[0], a[1], a[2])
    assert np.all(np.isfinite(s32))
    one = (r == a).any(axis=0)                      # a fraction of exactly 1: balanced part is 0
    err = np.abs(s32[~one].astype(np.float64) - s64[~one])
    assert err.max() < BOUND, f"worst screen error {err.max():.3e}"
    # the upper bound holds where the balanced part vanishes; the lower bound is never taken there
    assert np.all(s32[one].astype(np.float64) + float(EPS) >= s64[one])
    assert np.all(fmax[one] >= np.float32(0.999))
    # lower-bound use (fmax < 0.999): screen - eps < score and the pair is eligible
    lo = ~one & (fmax < np.float32(0.999))
    assert np.all((s32[lo] - EPS).astype(np.float64) < s64[lo])
    assert np.all(s64[lo] > 0)


def test_screen_bench_like_values():
    """c4-like pairs (cpu millicores, memory KiB, pod counts): the regime the bench runs in."""
    rng = np.random.default_rng(7)
    n = 300_000
    ac = rng.integers(1, 64_001, n); am = rng.integers(1, 256 << 20, n); ap = rng.integers(1, 111, n)
    rc = (rng.random(n) * ac).astype(np.int64); rm = (rng.random(n) * am).astype(np.int64)
    rp = (rng.random(n) * ap).astype(np.int64)
    s32, _ = screen_score(rc, rm, rp, ac, am, ap)
    s64 = exact_score(rc, rm, rp, ac, am, ap)
    one = (rc == ac) | (rm == am) | (rp == ap)
    err = np.abs(s32[~one].astype(np.float64) - s64[~one])
    assert err.max() < BOUND


def test_unscreenable_values_are_nan():
    """Negative or >= 2^52 requests and non-positive or >= 2^52 allocatables make the screen NaN, which
    every comparison of the scan treats as 'score exactly'."""
    s, _ = screen_score([-5, 1, 1, 1], [1, 1 << 53, 1, 1], [1, 1, 1, 1], [10, 10, 0, -3], [10, 1 << 60, 10, 10],
                        [10, 10, 10, 10])
    assert np.all(np.isnan(s))
