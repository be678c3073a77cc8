"""Independent pure-Python restatement of the reference hot path (small cases only).

TEST INFRASTRUCTURE ONLY.  Written separately from oracle/cpu_ref.c so the two restatements can be
cross-checked bit-for-bit.  Python floats are IEEE doubles and CPython never
fuses multiply-add, so each expression below rounds exactly as Go amd64 does.

Anchors (relative to /root/reference): parseCpu anchor/predicate.go:10-24, parseMemory :26-44,
parsePod :46-53, fit anchor/predicate.go:134-148, scores anchor/scores.go:3-25 and
anchor/priorities.go:5-23,45-50, argmax anchor/priorities.go:55-61 (deterministic lowest-index
tie-break), sequential commit anchor/schedule.go:68-89,185-197 and anchor/predicate.go:83-105.
"""
from __future__ import annotations

import math
import re
import struct
from fractions import Fraction

INT64_MIN = -(1 << 63)
INT64_MAX = (1 << 63) - 1


class Fatal(ValueError):
    """The reference's errFatal (log.Fatal) paths."""


def _wrap64(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= (1 << 63) else v


def go_parse_int(s: str) -> int:
    if not re.fullmatch(r"[+-]?[0-9]+", s):
        raise Fatal(s)
    v = int(s, 10)
    if v < INT64_MIN or v > INT64_MAX:
        raise Fatal(s)
    return v


def _f32_bits(x: float) -> int:
    return struct.unpack("<I", struct.pack("<f", x))[0]


def _round_to_f32(q: Fraction) -> float:
    """Correctly rounded (nearest-even) float32 value of the exact rational q, as a Python float."""
    if q == 0:
        return 0.0
    sign = -1.0 if q < 0 else 1.0
    a = abs(q)
    # float32: 24-bit significand, min normal 2^-126, subnormal step 2^-149, max < 2^128
    e = a.numerator.bit_length() - a.denominator.bit_length()
    while Fraction(2) ** e > a:
        e -= 1
    while Fraction(2) ** (e + 1) <= a:
        e += 1
    step_e = max(e - 23, -149)
    step = Fraction(2) ** step_e
    m = a / step
    fl = m.numerator // m.denominator
    rem = m - fl
    if rem > Fraction(1, 2) or (rem == Fraction(1, 2) and fl % 2 == 1):
        fl += 1
    val = fl * step
    if val >= Fraction(2) ** 128 - Fraction(2) ** 103:  # rounds to infinity
        return sign * math.inf
    return sign * float(val)


def _underscore_ok(s: str) -> bool:
    """strconv.underscoreOK (Go atoi.go): underscores only between two digits, or between a base prefix
    and a digit (restated from the Go language spec's digit-separator rule)."""
    if s[:1] in ("+", "-"):
        s = s[1:]
    prev = "^"  # ^ start, 0 digit or base prefix, _ underscore, ! anything else
    i = 0
    hexd = False
    if len(s) >= 2 and s[0] == "0" and s[1] in "bBoOxX":
        i, prev, hexd = 2, "0", s[1] in "xX"
    for ch in s[i:]:
        if ch.isdigit() and ch.isascii() or (hexd and ch in "abcdefABCDEF"):
            prev = "0"
        elif ch == "_":
            if prev != "0":
                return False
            prev = "_"
        else:
            if prev == "_":
                return False
            prev = "!"
    return prev != "_"


_SPECIAL = re.compile(r"([+-])?(inf|infinity)", re.IGNORECASE)
# Go floating-point literal forms accepted by strconv.ParseFloat (digit separators checked separately):
#   decimal  [+-] digits [. digits] [e [+-] digit {digit|_}]      (at least one mantissa digit)
#   hex      [+-] 0x hexdigits [. hexdigits] p [+-] digit {digit|_} (the binary exponent is mandatory)
_DEC_FORM = re.compile(r"([+-]?)([0-9_]*)(?:\.([0-9_]*))?(?:[eE]([+-]?[0-9][0-9_]*))?")
_HEX_FORM = re.compile(r"([+-]?)0[xX]([0-9a-fA-F_]*)(?:\.([0-9a-fA-F_]*))?[pP]([+-]?[0-9][0-9_]*)")


def go_parse_float32(s: str):
    """strconv.ParseFloat(s, 32): the special words (optional sign only on the infinities), decimal and
    hexadecimal literals with Go digit separators, correctly rounded to float32 (round half to even).
    Returns (value, err) with err in {None, "syntax", "range"}; the value is float32-exact."""
    m = _SPECIAL.fullmatch(s)
    if m:
        return (-math.inf if m.group(1) == "-" else math.inf), None
    if s.lower() == "nan":
        return math.nan, None
    hx = _HEX_FORM.fullmatch(s)
    dc = None if hx else _DEC_FORM.fullmatch(s)
    m = hx or dc
    if not m or not _underscore_ok(s):
        return 0.0, "syntax"
    sign = -1 if m.group(1) == "-" else 1
    ip = m.group(2).replace("_", "")
    fp = (m.group(3) or "").replace("_", "")
    if not ip and not fp:
        return 0.0, "syntax"  # no mantissa digit
    ex = int(m.group(4).replace("_", "")) if m.group(4) else 0
    base = 16 if hx else 10
    mant = int(ip + fp, base) if ip + fp else 0
    if mant == 0:
        return (-0.0 if sign < 0 else 0.0), None
    if hx:
        q = Fraction(mant) * Fraction(2) ** (ex - 4 * len(fp))
    else:
        mag = len(str(mant)) + ex - len(fp)  # decimal digits of the integer part
        if mag > 40:                          # beyond float32's range: +-Inf, ErrRange
            return sign * math.inf, "range"
        if mag < -60:                         # below half the smallest subnormal: +-0
            return (-0.0 if sign < 0 else 0.0), None
        q = Fraction(mant) * Fraction(10) ** (ex - len(fp))
    v = _round_to_f32(q)
    if math.isinf(v):
        return sign * v, "range"
    return sign * v, None


def go_f64_to_i64(x: float) -> int:
    if math.isnan(x) or x >= 9223372036854775808.0 or x < -9223372036854775808.0:
        return INT64_MIN
    return int(x)


def parse_cpu(s):
    if s is None:
        return 0
    if s.endswith("m"):
        return go_parse_int(s[:-1])
    v, err = go_parse_float32(s)
    if err is None:
        return go_f64_to_i64(v * 1000.0)
    return 0


def parse_memory(s):
    if s is None:
        return 0
    if s.endswith("Ki"):
        return go_parse_int(s[:-2])
    if s.endswith("Mi"):
        return _wrap64(go_parse_int(s[:-2]) * 1024)
    return 0


def parse_pods(s):
    if s is None:
        return 0
    return go_parse_int(s)


def fraction_of_capacity(req: int, cap: int) -> float:
    if cap == 0:
        return 1.0
    return float(req) / float(cap)


def least_requested(req: int, cap: int) -> float:
    if cap == 0 or req > cap:
        return 0.0
    return float(_wrap64(cap - req)) * 10.0 / float(cap)


def balanced(rc, rm, rp, ac, am, ap) -> float:
    c = fraction_of_capacity(rc, ac)
    m = fraction_of_capacity(rm, am)
    p = fraction_of_capacity(rp, ap)
    if c >= 1 or m >= 1 or p >= 1:
        return 0.0
    mean = (c + m + p) / 3.0
    cr = (c - mean) * (c - mean)
    mr = (m - mean) * (m - mean)
    pr = (p - mean) * (p - mean)
    var = (cr + mr + pr) / 3.0
    return (1 - var) * 10.0


def score(rc, rm, rp, ac, am, ap) -> float:
    s = 0.0
    s += balanced(rc, rm, rp, ac, am, ap)
    s += (least_requested(rc, ac) + least_requested(rm, am) + least_requested(rp, ap)) / 3
    s /= 2
    return s


def schedule(nodes, pods, priority=0, domain=0, use_labels=False, labels=None, selector=None, price=None):
    """nodes: list of [cpu, mem, pods] allocatable (mutated copy returned); pods: list of
    (cpu, mem, pods) requests.  Returns (idx list, score list, feasible list, final nodes)."""
    st = [list(map(int, n)) for n in nodes]
    out_i, out_s, out_f = [], [], []
    for i, (rc, rm, rp) in enumerate(pods):
        sel = int(selector[i]) if (use_labels and selector is not None) else 0
        fc, best, bkey = 0, -1, 0.0
        for j, (ac, am, ap) in enumerate(st):
            feas = ac >= rc and am >= rm and ap >= rp
            if use_labels and labels is not None and (int(labels[j]) & sel) != sel:
                feas = False
            fc += feas
            if priority == 1:
                if not feas:
                    continue
                key = -float(price[j])
            else:
                if domain == 1 and not feas:
                    continue
                key = score(rc, rm, rp, ac, am, ap)
                if not key > 0:
                    continue
            if best < 0 or key > bkey or (key == bkey and j < best):
                best, bkey = j, key
        out_f.append(fc)
        if fc == 0:
            out_i.append(-1); out_s.append(0.0)
            continue
        if best < 0:
            out_i.append(-2); out_s.append(0.0)
            continue
        out_i.append(best)
        out_s.append(0.0 - bkey if priority == 1 else bkey)  # the price; "-0" and "0" both give +0
        st[best][0] = _wrap64(st[best][0] - rc)
        st[best][1] = _wrap64(st[best][1] - rm)
        st[best][2] = _wrap64(st[best][2] - 1)
    return out_i, out_s, out_f, st
