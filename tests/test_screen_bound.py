"""The f32 screen of the screened scan (csrc/ksched_device.h screen_pair) against
the reference's f64 resource score.

The screen never decides a result: a pair is skipped only when screen + kScreenEps < L, L being a lower
bound (screen - kScreenEps) of KC eligible keys of the same workgroup.  That is sound iff
|screen - score| < kScreenEps wherever the screen serves as a lower bound (resource-fitting pairs whose
fractions are all < 0.999, and non-fitting pairs), and screen + kScreenEps >= score everywhere.  numpy's
float32 arithmetic is IEEE round-to-nearest like the device's (no contraction: the library builds with
-ffp-contract=off), so the emulation below is the device computation bit for bit.
"""
import numpy as np
import pytest

EPS = np.float32(4e-5)      # kScreenEps
BOUND = 1.3e-5              # the polynomial's error bound ksched_device.h derives
BOUND_NF = 2e-6             # the non-fitting form's
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


def screen_pair(rc, rm, rp, ac, am, ap):
    """(value, lo_ok) as screen_pair computes them; ok_k = a_k >= r_k exactly."""
    rc, rm, rp, ac, am, ap = (np.asarray(x, np.int64) for x in (rc, rm, rp, ac, am, ap))
    qc, qm, qp = screen_req(rc), screen_req(rm), screen_req(rp)
    yc, ym, yp = screen_recip(ac), screen_recip(am), screen_recip(ap)
    okc, okm, okp = ac >= rc, am >= rm, ap >= rp
    with np.errstate(all="ignore"):
        c, m, p = qc * yc, qm * ym, qp * yp
        rf = okc & okm & okp
        fmax = np.fmax(np.fmax(c, m), p)
        S = (c + m) + p
        Q = (c * c + m * m) + p * p
        poly = ((F(10.0) - (F(5.0) / F(3.0)) * S) - (F(5.0) / F(3.0)) * Q) + (F(5.0) / F(9.0)) * (S * S)
        one = F(1.0)
        nf = (F(5.0) / F(3.0)) * ((np.where(okc, one - c, F(0)) + np.where(okm, one - m, F(0))) + np.where(okp, one - p, F(0)))
        nf = nf + F(0.0) * S
        v = np.where(rf, poly, nf).astype(np.float32)
        lo_ok = np.where(rf, fmax < F(0.999), True) & (v > EPS)
    return v, lo_ok


def screen_score(rc, rm, rp, ac, am, ap):
    """The resource-fitting form alone (the polynomial) and the largest fraction."""
    v, _ = screen_pair(rc, rm, rp, ac, am, ap)
    qc, qm, qp = screen_req(rc), screen_req(rm), screen_req(rp)
    with np.errstate(all="ignore"):
        c, m, p = qc * screen_recip(ac), qm * screen_recip(am), qp * screen_recip(ap)
    return v, np.fmax(np.fmax(c, m), p)


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


@pytest.mark.parametrize("seed", [4, 5])
def test_non_fitting_form(seed):
    """Pairs with some request above its allocatable (the all-node domain still ranks them, anchor/
    priorities.go:5-23): balanced part 0, that resource's least-requested term 0."""
    rng = np.random.default_rng(seed)
    n = 300_000
    r, a = _pairs(rng, n)
    over = rng.random((3, n)) < 0.4
    over[rng.integers(0, 3, n), np.arange(n)] = True                  # at least one resource over
    big = np.minimum(a + 1 + (rng.random((3, n)) * a * 4).astype(np.int64), (1 << 52) - 1)
    r = np.where(over & (a < (1 << 52) - 1), big, r)
    v, lo_ok = screen_pair(r[0], r[1], r[2], a[0], a[1], a[2])
    s64 = exact_score(r[0], r[1], r[2], a[0], a[1], a[2])
    nf = (r > a).any(axis=0)
    assert nf.mean() > 0.5
    err = np.abs(v[nf].astype(np.float64) - s64[nf])
    assert err.max() < BOUND_NF, f"worst non-fitting screen error {err.max():.3e}"
    # a lower bound only of eligible keys
    assert np.all(s64[nf & lo_ok] > 0)
    assert np.all((v[nf & lo_ok] - EPS).astype(np.float64) < s64[nf & lo_ok])


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



def screen_rec(v):
    """ksched_device.h screen_rec: the f16 pattern of w = max(RN(10 - v), 0) rounded down (NaN -> 0)."""
    v = np.asarray(v, np.float32)
    with np.errstate(invalid="ignore"):
        w = np.fmax(F(10.0) - v, F(0.0))
    h = w.astype(np.float16)  # round to nearest even, like v_cvt_f16_f32
    hb = h.view(np.uint16).astype(np.int64)
    return hb - (h.astype(np.float32) > w)


def rec_value(hb):
    return np.asarray(hb, np.int64).astype(np.uint16).view(np.float16).astype(np.float64)


def screen_rec_threshold(L):
    """ksched_device.h screen_rec_threshold."""
    L = np.asarray(L, np.float32)
    T = 11.0 + np.float64(EPS) + 2.0 ** -20 - L.astype(np.float64)
    h = T.astype(np.float32).astype(np.float16)
    return np.where(T >= 0, h.view(np.uint16).astype(np.int64) + 1, -1)


def test_screen_record_is_an_upper_bound():
    rng = np.random.default_rng(7)
    v = np.concatenate([rng.uniform(0, 10, 2_000_000), 10 - rng.uniform(0, 0.5, 500_000) ** 2]).astype(np.float32)
    h16 = np.arange(0, 0x4900 + 1, dtype=np.uint16).view(np.float16).astype(np.float32)  # every f16 in [0, 10]
    grid = np.float32(10.0) - h16
    v = np.concatenate([v, grid, np.nextafter(grid, F(0)), np.nextafter(grid, F(11)), F([0.0, 10.0, 1e-30, 9.9999995])])
    v = v[(v >= 0) & (v <= 10)]
    hb = screen_rec(v)
    assert hb.min() >= 0 and hb.max() <= 0x4900  # 16 bits, 0xffff stays free for "no key"
    ub = 10.0 - rec_value(hb)  # the bound pass 2 implies, before its 2^-20 slack
    assert np.all(ub + 2.0 ** -21 >= v)
    w = 10.0 - v.astype(np.float64)
    assert np.all(10.0 - ub <= w + 2.0 ** -21) and np.all(10.0 - ub >= w * (1 - 2.0 ** -10) - 2.0 ** -24 - 2.0 ** -21)
    assert screen_rec(F([np.nan]))[0] == 0  # an unscreenable pair: always needed


def test_pass2_integer_threshold_is_a_superset():
    """Pass 2 tests hb <= screen_rec_threshold(L) instead of decoding every record: every pair whose bound
    10 - value(hb) (+ the 2^-21 of w's own rounding) + 1 + eps reaches L must pass."""
    rng = np.random.default_rng(11)
    L = np.concatenate([rng.uniform(0, 11.001, 40000), 11 - rng.uniform(0, 0.3, 20000) ** 2, F([0.0, 1.0, 11.0])]).astype(np.float32)
    hb = np.concatenate([rng.integers(0, 0x4901, 40000), rng.integers(0, 0x3000, 20003)])
    tq = screen_rec_threshold(L)
    need = (10.0 - rec_value(hb)) + 2.0 ** -21 + 1.0 + np.float64(EPS) >= L.astype(np.float64)
    got = hb <= tq
    assert np.all(got[need])
    # tight: admitted beyond the exact test only within two f16 steps of the threshold
    extra = got & ~need
    assert np.all(rec_value(hb[extra]) <= (11.0 + np.float64(EPS) + 2.0 ** -20 - L[extra]) * (1 + 2.0 ** -9) + 2.0 ** -23)
    # L = 0 (fewer than KC bounds): every pair with a key passes, none without one (0xffff)
    t0 = int(screen_rec_threshold(F([0.0]))[0])
    assert 0x4900 <= t0 < 0xFFFF


# ---- the non-fitting records (ksched_device.h screen_rec_nf / screen_rec_threshold_nf) -------------------------
NF_BASE = F(3.375)  # kNfBase


def screen_rec_nf(v):
    """0x8000 | the f16 pattern of w = max(RN(kNfBase - v), 0) rounded down."""
    v = np.asarray(v, np.float32)
    with np.errstate(invalid="ignore"):
        w = np.fmax(NF_BASE - v, F(0.0))
    h = w.astype(np.float16)
    hb = h.view(np.uint16).astype(np.int64)
    return 0x8000 | (hb - (h.astype(np.float32) > w))


def screen_rec_threshold_nf(L):
    L = np.asarray(L, np.float32)
    T = np.float64(NF_BASE) + 1.0 + np.float64(EPS) + 2.0 ** -20 - L.astype(np.float64)
    h = T.astype(np.float32).astype(np.float16)
    return np.where(T >= 0, h.view(np.uint16).astype(np.int64) + 1, -1)


def needed(hb, tq, tqn):
    """ksched_device.h screen_rec_needed"""
    hb = np.asarray(hb, np.int64)
    return np.where(hb & 0x8000, (hb & 0x7FFF) <= tqn, hb <= tq)


def test_non_fitting_values_below_the_record_base():
    """Every non-fitting screen value stays below kNfBase (at most two (1 - f) terms of (5/3))."""
    rng = np.random.default_rng(21)
    n = 400_000
    r, a = _pairs(rng, n)
    over = np.zeros((3, n), bool)
    over[rng.integers(0, 3, n), np.arange(n)] = True
    big = np.minimum(a + 1 + (rng.random((3, n)) * a).astype(np.int64), (1 << 52) - 1)
    r = np.where(over & (a < (1 << 52) - 1), big, np.where(rng.random((3, n)) < 0.5, 0, r))  # zero requests: 1 - f = 1
    v, _ = screen_pair(r[0], r[1], r[2], a[0], a[1], a[2])
    nf = (r > a).any(axis=0)
    assert nf.mean() > 0.9
    assert np.nanmax(v[nf]) < NF_BASE and np.nanmax(v[nf]) > F(3.3)


def test_non_fitting_record_is_an_upper_bound():
    rng = np.random.default_rng(22)
    v = np.concatenate([rng.uniform(0, 10 / 3, 2_000_000), 10 / 3 - rng.uniform(0, 0.3, 500_000) ** 2]).astype(np.float32)
    h16 = np.arange(0, 0x42C0, dtype=np.uint16).view(np.float16).astype(np.float32)  # every f16 in [0, 3.375]
    grid = NF_BASE - h16
    v = np.concatenate([v, grid, np.nextafter(grid, F(0)), np.nextafter(grid, F(4)), F([0.0, 10 / 3, 3.3333337])])
    v = v[(v >= 0) & (v < NF_BASE)]
    hb = screen_rec_nf(v)
    assert np.all(hb & 0x8000) and (hb & 0x7FFF).max() <= 0x42C0 and (hb & 0x7FFF).min() >= 0
    ub = np.float64(NF_BASE) - rec_value(hb & 0x7FFF)
    assert np.all(ub + 2.0 ** -21 >= v)
    # tight where the late-c4 keys crowd (~3.25): within 2^-12 of v (the polynomial form there: 2^-8)
    crowd = (v > F(3.2)) & (v < F(3.34))
    assert np.all(ub[crowd] - v[crowd] < 2.0 ** -12)


def test_pass2_two_form_threshold_is_a_superset():
    """needed(): every record whose form's bound (+ 2^-21 + 1 + eps) reaches L passes, in both forms; the no-key
    pattern 0xffff never does, an always-needed 0 always does."""
    rng = np.random.default_rng(23)
    L = np.concatenate([rng.uniform(0, 11.001, 60000), 4.25 - rng.uniform(0, 0.1, 20000), F([0.0, 1.0, 4.375, 11.0])]).astype(np.float32)
    n = L.size
    poly = rng.integers(0, 0x4901, n)
    nfr = 0x8000 | rng.integers(0, 0x42C1, n)
    tq, tqn = screen_rec_threshold(L), screen_rec_threshold_nf(L)
    Ld = L.astype(np.float64)
    need_p = (10.0 - rec_value(poly)) + 2.0 ** -21 + 1.0 + np.float64(EPS) >= Ld
    need_n = (np.float64(NF_BASE) - rec_value(nfr & 0x7FFF)) + 2.0 ** -21 + 1.0 + np.float64(EPS) >= Ld
    assert np.all(needed(poly, tq, tqn)[need_p])
    assert np.all(needed(nfr, tq, tqn)[need_n])
    assert not needed(np.full(n, 0xFFFF), tq, tqn).any()
    assert needed(np.zeros(n, np.int64), tq, tqn)[Ld <= 11.0].all()
    # an inactive lane (-1, -1) needs nothing
    assert not needed(np.array([0, 0x8000, 0x4900, 0xFFFF]), -1, -1).any()


# ---- pass 1's VALU form (ksched_device.h screen_fast) ------------------------------------------------------------
def fma32(a, b, c):
    """f32 fused multiply-add: a * b + c rounded once (the product is exact in long double, the sum to 64 bits)"""
    L = np.longdouble
    return (np.asarray(a, np.float32).astype(L) * np.asarray(b, np.float32).astype(L) + np.asarray(c, np.float32).astype(L)).astype(np.float32)


def screen_fast(rc, rm, rp, ac, am, ap):
    """(v, mx, amb, rf) as screen_fast computes them from pass 1's f32 fractions."""
    rc, rm, rp, ac, am, ap = (np.asarray(x, np.int64) for x in (rc, rm, rp, ac, am, ap))
    with np.errstate(all="ignore"):
        c, m, p = screen_req(rc) * screen_recip(ac), screen_req(rm) * screen_recip(am), screen_req(rp) * screen_recip(ap)
        S = (c + m) + p
        mx = np.fmax(np.fmax(c, m), p)
        d = np.fmin(np.fmin(np.abs(c - F(1)), np.abs(m - F(1))), np.abs(p - F(1)))
        amb = ~(fma32(F(0), S, d) > F(2.0 ** -20))
        rf = mx < F(1)
        Q = fma32(c, c, fma32(m, m, p * p))
        poly = fma32(F(5.0 / 9.0), S * S, fma32(F(-5.0 / 3.0), S + Q, F(10)))
        sat = lambda x: np.clip(x, F(0), F(1))  # noqa: E731
        nf = F(5.0 / 3.0) * ((sat(F(1) - c) + sat(F(1) - m)) + sat(F(1) - p))
        v = np.where(rf, poly, nf).astype(np.float32)
    return v, mx, amb, rf


@pytest.mark.parametrize("seed", [41, 42, 43])
def test_screen_fast_matches_the_bounds(seed):
    """screen_fast: the same ambiguity and fit classes as screen_q's compares, and the same error bounds: the
    polynomial within BOUND of the f64 score (lower-bound use where mx < 0.999), the non-fitting form within BOUND_NF
    and below kNfBase."""
    rng = np.random.default_rng(seed)
    n = 300_000
    r, a = _pairs(rng, n)
    over = rng.random((3, n)) < 0.25
    big = np.minimum(a + 1 + (rng.random((3, n)) * a * 3).astype(np.int64), (1 << 52) - 1)
    r = np.where(over & (a < (1 << 52) - 1), big, r)
    near = rng.random(n) < 0.05                                   # fractions within a few ulps of 1
    k = rng.integers(0, 3, n)
    r[k[near], np.nonzero(near)[0]] = a[k[near], np.nonzero(near)[0]] + rng.integers(-2, 3, near.sum())
    r = np.maximum(r, 0)
    v, mx, amb, rf = screen_fast(r[0], r[1], r[2], a[0], a[1], a[2])
    qc, qm, qp = screen_req(r[0]), screen_req(r[1]), screen_req(r[2])
    with np.errstate(all="ignore"):
        c, m, p = qc * screen_recip(a[0]), qm * screen_recip(a[1]), qp * screen_recip(a[2])
        lo, hi = F(1) - F(2.0 ** -20), F(1) + F(2.0 ** -20)
        amb_q = ~((c < lo) | (c > hi)) | ~((m < lo) | (m > hi)) | ~((p < lo) | (p > hi))
    assert np.array_equal(amb, amb_q), "ambiguity classes differ from screen_q's compares"
    ok = ~amb
    assert np.array_equal(rf[ok], ((c < lo) & (m < lo) & (p < lo))[ok])
    s64 = exact_score(r[0], r[1], r[2], a[0], a[1], a[2])
    pf = ok & rf & (mx < F(0.999))
    err = np.abs(v[pf].astype(np.float64) - s64[pf])
    assert err.max() < BOUND, f"polynomial: worst error {err.max():.3e}"
    upf = ok & rf                                             # every resource-fitting pair: an upper bound
    assert np.all(v[upf].astype(np.float64) + float(EPS) >= s64[upf])
    nfm = ok & ~rf
    assert nfm.mean() > 0.2
    err = np.abs(v[nfm].astype(np.float64) - s64[nfm])
    assert err.max() < BOUND_NF, f"non-fitting: worst error {err.max():.3e}"
    assert v[nfm].max() < NF_BASE
    # the pass-1 lower bound (lo_ok) only of eligible keys
    lo_ok = ok & ~(rf & (mx >= F(0.999))) & (v > EPS)
    assert np.all((v[lo_ok] - EPS).astype(np.float64) < s64[lo_ok]) and np.all(s64[lo_ok] > 0)


def test_screen_fast_nan_is_ambiguous():
    """An unscreenable operand (negative or >= 2^52 request, zero or negative allocatable) makes a fraction NaN: the
    pair is ambiguous whichever resource it is (the min of the |f - 1| drops NaN; 0 * S carries it)."""
    for k in range(3):
        r = np.array([[10], [10], [1]], np.int64)
        a = np.array([[100], [100], [10]], np.int64)
        a[k, 0] = 0
        v, mx, amb, rf = screen_fast(r[0], r[1], r[2], a[0], a[1], a[2])
        assert amb[0], k
        r2 = r.copy(); a2 = np.array([[100], [100], [10]], np.int64)
        r2[k, 0] = -3
        assert screen_fast(r2[0], r2[1], r2[2], a2[0], a2[1], a2[2])[2][0], k
