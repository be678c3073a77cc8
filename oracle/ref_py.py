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


_DEC = re.compile(r"[+-]?(?:[0-9]+\.?[0-9]*|\.[0-9]+)(?:[eE][+-]?[0-9]+)?")


def go_parse_float32(s: str):
    """strconv.ParseFloat(s, 32) for the forms the generator and tests use: decimal literals and the
    special words.  Returns (value, err) with err in {None, "syntax", "range"}.  Hex and underscore
    forms are only covered by the C oracle."""
    low = s.lower()
    body = low[1:] if low[:1] in "+-" else low
    sign = -1.0 if low[:1] == "-" else 1.0
    if body in ("inf", "infinity"):
        return sign * math.inf, None
    if low == "nan":
        return math.nan, None
    if not _DEC.fullmatch(s):
        return 0.0, "syntax"
    v = _round_to_f32(Fraction(s))
    if math.isinf(v):
        return v, "range"
    return v, None


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
