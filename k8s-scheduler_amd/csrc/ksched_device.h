// ksched_device.h -- device-side restatement of the reference's per-pair semantics (gfx950).
//
// Every floating-point expression follows the reference's operation order exactly and the whole
// library is compiled with -ffp-contract=off (no FMA contraction), so scores are bit-identical to
// the Go amd64 reference (and to oracle/cpu_ref.c):
//   fractionOfCapacity         anchor/scores.go:3-8
//   getBalancedResourceScore   anchor/scores.go:10-18
//   getLeastRequestedScore     anchor/scores.go:20-25
//   balancedResourceScore      anchor/priorities.go:5-15
//   leastRequestedScore        anchor/priorities.go:17-23
//   score accumulation         anchor/priorities.go:45-50   ((0 + balanced) + least) / 2
//   fit predicate              anchor/predicate.go:134-148  (+ build-defined label bitsets)
//   argmax                     anchor/priorities.go:55-61   strict '>' from 0; ties -> lowest index
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ksched {

// ---- coherent (sc1) 8-byte accesses: hand-offs between workgroups of persistent kernels ----------
// MI355X_MICROARCH "valid forms", row 1: every store of the handed-off bytes an sc1 store (relaxed
// agent-scope atomic = global_store ... sc1), drained (s_waitcnt vmcnt(0)) before ONE lane's flag /
// counter update; every load of them an sc1 load, after the poll.  No fences, no L2 write-back.
__device__ __forceinline__ uint64_t ld_coh(const void *p) {
    return __hip_atomic_load(reinterpret_cast<const uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_coh(void *p, uint64_t v) {
    __hip_atomic_store(reinterpret_cast<uint64_t *>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_coh_f64(const void *p) { return __longlong_as_double((long long)ld_coh(p)); }
__device__ __forceinline__ void st_coh_f64(void *p, double v) { st_coh(p, (uint64_t)__double_as_longlong(v)); }
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// 16-byte sc1 accesses (same valid form: write-through stores, L2-served loads) through a buffer resource over
// `base` (byte offsets < 2^31): one 16-B record per lane in one request, where two 8-B stores to the same
// 16 B are two partial-line write requests.  gfx950 buffer aux bit 4 = sc1.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t coh_rsrc(const void *base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void st_coh16(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, 16);
}
__device__ __forceinline__ u32x4 ld_coh16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16);
}

constexpr int kPrioResource = 0;
constexpr int kPrioPrice = 1;
constexpr int kDomAll = 0;
constexpr int kDomFeasible = 1;
constexpr int32_t kNoIdx = 0x7fffffff;  // "no candidate" index (ranks after every real node)

// Node state as kept in HBM (AoS, 96 B: s_load_dwordx16 + s_load_dwordx8 when wave-uniform).
struct alignas(16) NodeRec {
    int64_t a[3];      // allocatable cpu (millicores), memory (KiB), pods = capacity - used
    uint64_t labels;   // label bitset (build extension)
    double af[3];      // (double)a[k], kept in sync with a[k] by every writer (device side)
    double y[3];       // recip(af[k]): hipcc's refined reciprocal of the divisor (0 when a[k] == 0)
    float ys[3];       // screen_recip(a[k]): f32 reciprocal for the screened scan (maintained in the
                       // persistent pipeline's LDS rows only; stale in HBM)
    float price;       // node price (best-price priority)
};
static_assert(sizeof(NodeRec) == 96, "NodeRec layout");
// The same rows seen through the constant address space: wave-uniform reads become scalar loads.
typedef __attribute__((address_space(4))) NodeRec NodeRecC;

__device__ __forceinline__ NodeRec load_row(const NodeRecC *p) {
    NodeRec r;
    r.a[0] = p->a[0]; r.a[1] = p->a[1]; r.a[2] = p->a[2];
    r.labels = p->labels;
    r.af[0] = p->af[0]; r.af[1] = p->af[1]; r.af[2] = p->af[2];
    r.y[0] = p->y[0]; r.y[1] = p->y[1]; r.y[2] = p->y[2];
    r.price = p->price;
    return r;
}

// One candidate of a partial top-K list (score kernels -> merge kernels).  The persistent pipeline carries a
// list's predicate count in entry 0's pad (one 16-B store per entry, no separate count word).
struct alignas(16) Cand {
    double key;
    int32_t idx;  // global node index, kNoIdx = empty slot
    int32_t pad;
};
static_assert(sizeof(Cand) == 16, "Cand layout");

// A merged top-K entry with the node's snapshot state: what ranks exchange (RCCL all-gather) so any
// rank can re-score a node it does not own after a commit.  Same layout as oracle or_rec.
struct alignas(8) Rec {
    double key;
    int32_t idx;
    int32_t valid;
    int64_t a[3];
    uint64_t labels;
    float price;
    int32_t pad;
};
static_assert(sizeof(Rec) == 56, "Rec layout");

// Rec loads / stores, plain or coherent (COH: 8-byte sc1 accesses, Rec words w0..w6).
template <bool COH>
__device__ __forceinline__ Rec load_rec(const Rec *p) {
    if constexpr (!COH) {
        return *p;
    } else {
        const uint64_t *w = reinterpret_cast<const uint64_t *>(p);
        Rec r;
        const uint64_t w1 = ld_coh(w + 1), w6 = ld_coh(w + 6);
        r.key = __longlong_as_double((long long)ld_coh(w));
        r.idx = (int32_t)(uint32_t)w1; r.valid = (int32_t)(uint32_t)(w1 >> 32);
        r.a[0] = (int64_t)ld_coh(w + 2); r.a[1] = (int64_t)ld_coh(w + 3); r.a[2] = (int64_t)ld_coh(w + 4);
        r.labels = ld_coh(w + 5);
        r.price = __uint_as_float((uint32_t)w6); r.pad = (int32_t)(uint32_t)(w6 >> 32);
        return r;
    }
}
// The node-state words of a Rec only (a[3], labels, price: words w2..w6) -- what a commit needs of a
// candidate it already knows by key and index.
template <bool COH>
__device__ __forceinline__ void load_rec_state(const Rec *p, int64_t *a, uint64_t *labels, float *price) {
    const uint64_t *w = reinterpret_cast<const uint64_t *>(p);
    uint64_t v[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) v[i] = COH ? ld_coh(w + 2 + i) : w[2 + i];
    a[0] = (int64_t)v[0]; a[1] = (int64_t)v[1]; a[2] = (int64_t)v[2];
    *labels = v[3];
    *price = __uint_as_float((uint32_t)v[4]);
}
template <bool COH>
__device__ __forceinline__ void store_rec(Rec *p, const Rec &r) {
    if constexpr (!COH) {
        *p = r;
    } else {
        uint64_t *w = reinterpret_cast<uint64_t *>(p);
        st_coh(w, (uint64_t)__double_as_longlong(r.key));
        st_coh(w + 1, (uint64_t)(uint32_t)r.idx | ((uint64_t)(uint32_t)r.valid << 32));
        st_coh(w + 2, (uint64_t)r.a[0]); st_coh(w + 3, (uint64_t)r.a[1]); st_coh(w + 4, (uint64_t)r.a[2]);
        st_coh(w + 5, r.labels);
        st_coh(w + 6, (uint64_t)__float_as_uint(r.price) | ((uint64_t)(uint32_t)r.pad << 32));
    }
}
template <bool COH>
__device__ __forceinline__ int64_t load_i64(const int64_t *p) { return COH ? (int64_t)ld_coh(p) : *p; }
template <bool COH>
__device__ __forceinline__ void store_i64(int64_t *p, int64_t v) { if (COH) st_coh(p, (uint64_t)v); else *p = v; }

__host__ __device__ inline int64_t wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }



// (key desc, idx asc): the deterministic restatement of the reference's map-order argmax.
__device__ __forceinline__ bool better(double ka, int32_t ia, double kb, int32_t ib) {
    return ka > kb || (ka == kb && ia < ib);
}

__device__ __forceinline__ bool fits(int64_t rc, int64_t rm, int64_t rp, uint64_t sel, int64_t ac, int64_t am,
                                     int64_t ap, uint64_t lab, bool use_labels) {
    bool f = (ac >= rc) & (am >= rm) & (ap >= rp);
    if (use_labels) f &= ((lab & sel) == sel);
    return f;
}

// ---- f64 division with a hoisted divisor reciprocal, bit-identical to hipcc's `a / b` ----------
// hipcc lowers a double division to (gfx950 ISA, checked in DESIGN.md):
//   d = v_div_scale(b, b, a); r = v_rcp(d); e = fma(-d, r, 1); r = fma(r, e, r);
//   e = fma(-d, r, 1); r = fma(r, e, r);  n = v_div_scale(a, b, a); q = n * r;
//   rm = fma(-d, q, n); q = v_div_fmas(rm, r, q); result = v_div_fixup(q, b, a)
// For the operands of this path -- integer-valued divisors 1 <= |b| <= 2^63 or b = 3, numerators
// that are integer-valued, or sums/squares of such quotients (|a| >= 2^-200 or a == 0) -- both
// div_scale are identities (no exponent gap >= 768, no denormal divisor or reciprocal, numerator
// exponent far above the 2^-970 rescale threshold), div_fmas is a plain fma (VCC = 0) and div_fixup
// passes a finite normal quotient through.  So the refined reciprocal r depends on b alone and can
// be computed once per divisor; the per-numerator part is 3 instructions.  Signed zeros of a zero
// numerator may differ from the native sequence but never reach a score.
__device__ __forceinline__ double recip(double b) {
    double r = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-b, r, 1.0);
    return __builtin_fma(r, e, r);
}

__device__ __forceinline__ double qdiv(double a, double b, double y) {
    const double q = a * y;
    const double rm = __builtin_fma(-b, q, a);
    return __builtin_fma(rm, y, q);
}

// Resource score with hoisted reciprocals y* of the allocatable values and y3 = recip(3.0).
// FAST53: every |alloc| and |request| < 2^52 (host-checked for the whole call), so
// (double)(a - r) == (double)a - (double)r exactly and the int64->f64 conversion is skipped.
template <bool FAST53>
__device__ __forceinline__ double resource_score_fast(int64_t rc, int64_t rm, int64_t rp, double rcf, double rmf,
                                                      double rpf, int64_t ac, int64_t am, int64_t ap, double acf,
                                                      double amf, double apf, double yc, double ym, double yp,
                                                      double y3) {
    const double c = (ac == 0) ? 1.0 : qdiv(rcf, acf, yc);
    const double m = (am == 0) ? 1.0 : qdiv(rmf, amf, ym);
    const double p = (ap == 0) ? 1.0 : qdiv(rpf, apf, yp);
    double b = 0.0;
    if (!(c >= 1.0 || m >= 1.0 || p >= 1.0)) {
        const double mean = qdiv((c + m) + p, 3.0, y3);
        const double cr = (c - mean) * (c - mean);
        const double mr = (m - mean) * (m - mean);
        const double pr = (p - mean) * (p - mean);
        const double var = qdiv((cr + mr) + pr, 3.0, y3);
        b = (1.0 - var) * 10.0;
    }
    const double dc = FAST53 ? acf - rcf : (double)wsub(ac, rc);
    const double dm = FAST53 ? amf - rmf : (double)wsub(am, rm);
    const double dp = FAST53 ? apf - rpf : (double)wsub(ap, rp);
    const double lc = (ac == 0 || rc > ac) ? 0.0 : qdiv(dc * 10.0, acf, yc);
    const double lm = (am == 0 || rm > am) ? 0.0 : qdiv(dm * 10.0, amf, ym);
    const double lp = (ap == 0 || rp > ap) ? 0.0 : qdiv(dp * 10.0, apf, yp);
    const double l = qdiv((lc + lm) + lp, 3.0, y3);
    double s = 0.0;
    s += b;
    s += l;
    s *= 0.5;  // x / 2 == x * 0.5 exactly (both are the correctly rounded x/2)
    return s;
}

// Best-price key: -price, with +0.0 for both signed zeros (x + 0.0 maps -0 to +0 in round-to-nearest
// and is not folded under -fno-fast-math): ranked by bit pattern in the merge, a price of -0 must not
// outrank a price of 0 at a lower node index.
__host__ __device__ __forceinline__ double price_key(float price) { return -(double)price + 0.0; }

template <int PRIO, int DOM, bool FAST53>
__device__ __forceinline__ bool pair_key_fast(bool feas, int64_t rc, int64_t rm, int64_t rp, double rcf, double rmf,
                                              double rpf, int64_t ac, int64_t am, int64_t ap, double acf,
                                              double amf, double apf, double yc, double ym, double yp, double y3,
                                              float price, double *key) {
    if (PRIO == kPrioPrice) {
        *key = price_key(price);
        return feas;
    } else {
        if (DOM == kDomFeasible && !feas) return false;
        const double s = resource_score_fast<FAST53>(rc, rm, rp, rcf, rmf, rpf, ac, am, ap, acf, amf, apf, yc, ym,
                                                     yp, y3);
        *key = s;
        return s > 0.0;
    }
}

__device__ __forceinline__ double recip_or_zero(int64_t a, double af) { return a == 0 ? 0.0 : recip(af); }

// ---- f32 screen of the resource score (the persistent pipeline's screened scan) ----
// With fractions f_k = r_k / a_k (0 < a_k < 2^52, 0 <= r_k < 2^52) the reference score (anchor/priorities.go:
// 5-23,45-50) is, in real arithmetic,
//   resource-fitting pair (every r_k <= a_k), every f_k < 1:
//     s = ((1 - var) * 10 + 10 (1 - mu)) / 2 = 10 - (5/3) S - (5/3) Q + (5/9) S^2,
//     S = f_c + f_m + f_p,  Q = f_c^2 + f_m^2 + f_p^2      (mu = S / 3, var = Q / 3 - mu^2);
//   some f_k == 1 exactly: the balanced part is 0 (priorities.go:10-12) and s = 5 (1 - mu) <= the polynomial;
//   some r_k > a_k: balanced part 0, that resource's least-requested term 0 (scores.go:21), so
//     s = (5/3) * sum over the k with r_k <= a_k of (1 - f_k).
// screen_pair evaluates the applicable form in f32 from f32 requests and f32 reciprocals.  Error against the
// f64 score of the reference's operation order: < 1.3e-5 for the polynomial (f_k relative error <= 3u,
// u = 2^-24; S <= 15u, Q <= 30u, S^2 <= 100u absolute; the final combination of values <= 10 adds <= 80u;
// the f64 score is within 1e-14 of the real one), < 2e-6 for the non-fitting form.  kScreenEps = 4e-5 keeps
// a 3x margin (tests/test_screen_bound.py checks both forms on random, adversarial and c4-like pairs).  A screen
// never decides a result: it only proves that a pair cannot enter a workgroup's top-KC list; every pair it
// cannot exclude is scored exactly.
constexpr float kScreenEps = 4e-5f;
// 1/a in f32 for 0 < a < 2^52; NaN otherwise (every pair with this node is then scored exactly)
__host__ __device__ __forceinline__ float screen_recip(int64_t a) {
    return (a > 0 && a < (1ll << 52)) ? (float)(1.0 / (double)a) : __builtin_nanf("");
}
// a request in f32; NaN when negative or >= 2^52 (scored exactly)
__host__ __device__ __forceinline__ float screen_req(int64_t r) {
    return (r >= 0 && r < (1ll << 52)) ? (float)r : __builtin_nanf("");
}
// A fraction q = RN(RN(r) * RN(1/a)) (f32) is within 3u = 1.8e-7 (relative) of r/a: below kFracLo it proves
// r < a, above kFracHi r > a; in between (or NaN) the int64 compare decides.
constexpr float kFracLo = 1.0f - 0x1p-20f;
constexpr float kFracHi = 1.0f + 0x1p-20f;

// The screen of one pair from its f32 fractions c, m, p; ok* = (a_k >= r_k) per resource, exact.
__device__ __forceinline__ float screen_q(float c, float m, float p, bool okc, bool okm, bool okp, bool *lo_ok) {
    const bool rf = okc & okm & okp;
    const float fmax = __builtin_fmaxf(__builtin_fmaxf(c, m), p);
    const float S = (c + m) + p;
    const float Q = (c * c + m * m) + p * p;
    const float poly = ((10.0f - (5.0f / 3.0f) * S) - (5.0f / 3.0f) * Q) + (5.0f / 9.0f) * (S * S);
    const float nf = (5.0f / 3.0f) * (((okc ? 1.0f - c : 0.0f) + (okm ? 1.0f - m : 0.0f)) + (okp ? 1.0f - p : 0.0f)) +
                     0.0f * S;
    const float v = rf ? poly : nf;
    *lo_ok = (rf ? fmax < 0.999f : true) && v > kScreenEps;  // false for NaN
    return v;
}

// Pass 1's screen of one pair from its f32 fractions (c, m, p), in a VALU-only form (no per-resource predicate
// masks, whose combination costs scalar-unit instructions shared by the workgroup's 12 waves):
//   amb: some fraction within 2^-20 of 1, or NaN -- the int64 compares decide such a pair.  |f - 1| is exact near 1
//        (Sterbenz) and >= 0.5 elsewhere, so |f - 1| > 2^-20 is exactly screen_q's (f < kFracLo || f > kFracHi); the
//        min of the three carries a NaN through 0 * S (min itself drops NaN operands);
//   rf:  every resource fits -- for a non-ambiguous pair, the largest fraction mx below 1;
//   v:   rf ? 10 - (5/3)(S + Q) + (5/9) S^2 : (5/3) * sum_k sat(1 - f_k), sat(x) = clamp(x, 0, 1): a non-fitting
//        resource's f > 1 (not ambiguous) clamps to 0, a fitting one's 1 - f is in (0, 1].  Fused multiply-adds in the
//        polynomial (Q, and its two combinations), so its rounding error is at most screen_q's bound (< 1.3e-5;
//        tests/test_screen_bound.py emulates this form too).
struct ScreenV {
    float v, mx;
    bool amb, rf;
};
__device__ __forceinline__ float sat01(float x) { return __builtin_amdgcn_fmed3f(x, 0.0f, 1.0f); }
__device__ __forceinline__ ScreenV screen_fast(float c, float m, float p) {
    ScreenV o;
    const float S = (c + m) + p;
    o.mx = __builtin_fmaxf(__builtin_fmaxf(c, m), p);
    const float d = __builtin_fminf(__builtin_fminf(__builtin_fabsf(c - 1.0f), __builtin_fabsf(m - 1.0f)),
                                    __builtin_fabsf(p - 1.0f));
    o.amb = !(__builtin_fmaf(0.0f, S, d) > 0x1p-20f);
    o.rf = o.mx < 1.0f;
    const float Q = __builtin_fmaf(c, c, __builtin_fmaf(m, m, p * p));
    const float poly = __builtin_fmaf(5.0f / 9.0f, S * S, __builtin_fmaf(-5.0f / 3.0f, S + Q, 10.0f));
    const float nf = (5.0f / 3.0f) * ((sat01(1.0f - c) + sat01(1.0f - m)) + sat01(1.0f - p));
    o.v = o.rf ? poly : nf;
    return o;
}

// The screened scan's per-pair record (pass 1 -> pass 2): a 16-bit upper bound of a screen value v (NaN allowed),
// in two forms by the pair's screen form (screen_q's rf):
//   resource-fitting (polynomial, v <= 10): the f16 bit pattern h of w = RN(10 - v) rounded DOWN (round toward
//     zero: v_cvt_pkrtz_f16_f32 of two rows at once), so 10 - value(h) >= v - 2^-21; bit 15 clear;
//   non-fitting (v <= (5/3) * 2 < kNfBase): the same of w = RN(kNfBase - v), with bit 15 set -- f16's relative
//     precision is then fine near the non-fitting keys (~3.3: late in c4 most pods fit nowhere and rank only
//     these), where 10 - v was coarse (ulp 2^-8 at w ~ 6.7).
// NaN -> w = 0 (maxNum): always needed.  0 = always needed, 0xffff = no key (a non-fitting NaN pattern, above every
// threshold).  Pass 2 compares the 15 low bits as integers against the form's threshold (screen_rec_threshold).
constexpr float kNfBase = 3.375f;  // > every non-fitting screen value (<= (5/3) * 2 + rounding)
__device__ __forceinline__ uint32_t screen_rec_w(float w) {  // f16 pattern of w >= 0 rounded down
    const _Float16 h = (_Float16)w;
    const uint32_t hb = (uint32_t)__builtin_bit_cast(uint16_t, h);
    return hb - ((float)h > w ? 1u : 0u);
}
__device__ __forceinline__ uint32_t screen_rec(float v) { return screen_rec_w(__builtin_fmaxf(10.0f - v, 0.0f)); }
__device__ __forceinline__ uint32_t screen_rec_nf(float v) {
    return 0x8000u | screen_rec_w(__builtin_fmaxf(kNfBase - v, 0.0f));
}
// The largest record (+ one) a pod needs with bound L (shifted by +1, 0 = none): base - value(h) + 2^-20 + 1 + eps
// >= L  <=>  value(h) <= T = base + 1 + eps + 2^-20 - L; -1 when T < 0.  RN to f16 of T (as f32), plus one pattern:
// a superset of the exact test (tests/test_screen_bound.py).  base = 10 (resource-fitting records) or kNfBase.
__device__ __forceinline__ int screen_rec_threshold_at(double base, float L) {
    const double T = base + 1.0 + (double)kScreenEps + 0x1p-20 - (double)L;
    if (!(T >= 0.0)) return -1;
    const _Float16 h = (_Float16)(float)T;
    return (int)__builtin_bit_cast(uint16_t, h) + 1;
}
__device__ __forceinline__ int screen_rec_threshold(float L) { return screen_rec_threshold_at(10.0, L); }
__device__ __forceinline__ int screen_rec_threshold_nf(float L) { return screen_rec_threshold_at((double)kNfBase, L); }
// pass 2's test of one record against the pod's two thresholds (-1, -1: an inactive lane)
__device__ __forceinline__ bool screen_rec_needed(uint32_t h, int tq, int tqn) {
    return (h & 0x8000u) ? (int)(h & 0x7fffu) <= tqn : (int)h <= tq;
}

// The screen of one pair.  ok* = (a_k >= r_k) per resource (exact int64 compares).  Returns the f32 value
// (NaN: unscreenable, every comparison then asks for the exact score); *lo_ok: the pair surely carries an
// eligible key >= value - eps (its value may serve as a lower bound: a polynomial pair with a fraction near 1
// may have lost its balanced part, so it never does).
__device__ __forceinline__ float screen_pair(float qc, float qm, float qp, float yc, float ym, float yp, bool okc,
                                             bool okm, bool okp, bool *lo_ok) {
    const float c = qc * yc, m = qm * ym, p = qp * yp;
    const bool rf = okc & okm & okp;
    const float fmax = __builtin_fmaxf(__builtin_fmaxf(c, m), p);
    const float S = (c + m) + p;
    const float Q = (c * c + m * m) + p * p;
    const float poly = ((10.0f - (5.0f / 3.0f) * S) - (5.0f / 3.0f) * Q) + (5.0f / 9.0f) * (S * S);
    // any unscreenable input (S is NaN) makes the value NaN in both forms (0 * S: no branch; S is finite
    // otherwise): the non-fitting form drops a resource's term only when its request exceeds a POSITIVE
    // allocatable (fraction > 1)
    const float nf = (5.0f / 3.0f) * (((okc ? 1.0f - c : 0.0f) + (okm ? 1.0f - m : 0.0f)) + (okp ? 1.0f - p : 0.0f)) +
                     0.0f * S;
    const float v = rf ? poly : nf;
    *lo_ok = (rf ? fmax < 0.999f : true) && v > kScreenEps;  // false for NaN
    return v;
}

// Upper bound of the resource score without the division corrections: every a / b is replaced by
// a * recip(b) (relative error <= 2^-51 per quotient), so |approx - exact| <= ~1e3 * 2^-52 *
// (|balanced| + |least| + 20); the bound adds 1e-9 * (|balanced| + |least| + 1), orders of magnitude
// more.  *near1 flags a fraction within 1e-12 of 1, where the balanced branch (fraction >= 1) could
// differ from the exact one -- such pairs must be scored exactly.
template <bool FAST53>
__device__ __forceinline__ double resource_score_upper(int64_t rc, int64_t rm, int64_t rp, double rcf, double rmf,
                                                       double rpf, int64_t ac, int64_t am, int64_t ap, double acf,
                                                       double amf, double apf, double yc, double ym, double yp,
                                                       double y3, bool *near1) {
    const double c = (ac == 0) ? 1.0 : rcf * yc;
    const double m = (am == 0) ? 1.0 : rmf * ym;
    const double p = (ap == 0) ? 1.0 : rpf * yp;
    *near1 = (ac != 0 && __builtin_fabs(c - 1.0) < 1e-12) | (am != 0 && __builtin_fabs(m - 1.0) < 1e-12) |
             (ap != 0 && __builtin_fabs(p - 1.0) < 1e-12);
    double b = 0.0;
    if (!(c >= 1.0 || m >= 1.0 || p >= 1.0)) {
        const double mean = ((c + m) + p) * y3;
        const double var = (((c - mean) * (c - mean) + (m - mean) * (m - mean)) + (p - mean) * (p - mean)) * y3;
        b = (1.0 - var) * 10.0;
    }
    const double dc = FAST53 ? acf - rcf : (double)wsub(ac, rc);
    const double dm = FAST53 ? amf - rmf : (double)wsub(am, rm);
    const double dp = FAST53 ? apf - rpf : (double)wsub(ap, rp);
    const double lc = (ac == 0 || rc > ac) ? 0.0 : dc * 10.0 * yc;
    const double lm = (am == 0 || rm > am) ? 0.0 : dm * 10.0 * ym;
    const double lp = (ap == 0 || rp > ap) ? 0.0 : dp * 10.0 * yp;
    const double l = ((lc + lm) + lp) * y3;
    const double s = (b + l) * 0.5;
    return s + 1e-9 * (__builtin_fabs(b) + __builtin_fabs(l) + 1.0);
}

// The resource score of one (request, allocatable) pair.  rcf/... are (double) of the int64 values
// (hoisted by callers; (double)int64 is correctly rounded, identical wherever it is computed).
__device__ __forceinline__ double resource_score(int64_t rc, int64_t rm, int64_t rp, double rcf, double rmf,
                                                 double rpf, int64_t ac, int64_t am, int64_t ap, double acf,
                                                 double amf, double apf) {
    // fractionOfCapacity
    const double c = (ac == 0) ? 1.0 : rcf / acf;
    const double m = (am == 0) ? 1.0 : rmf / amf;
    const double p = (ap == 0) ? 1.0 : rpf / apf;
    double b = 0.0;
    if (!(c >= 1.0 || m >= 1.0 || p >= 1.0)) {
        const double mean = ((c + m) + p) / 3.0;
        const double cr = (c - mean) * (c - mean);
        const double mr = (m - mean) * (m - mean);
        const double pr = (p - mean) * (p - mean);
        const double var = ((cr + mr) + pr) / 3.0;
        b = (1.0 - var) * 10.0;
    }
    // getLeastRequestedScore: int64 subtraction first, then conversion
    const double lc = (ac == 0 || rc > ac) ? 0.0 : ((double)wsub(ac, rc) * 10.0) / acf;
    const double lm = (am == 0 || rm > am) ? 0.0 : ((double)wsub(am, rm) * 10.0) / amf;
    const double lp = (ap == 0 || rp > ap) ? 0.0 : ((double)wsub(ap, rp) * 10.0) / apf;
    const double l = ((lc + lm) + lp) / 3.0;
    double s = 0.0;
    s += b;
    s += l;
    s /= 2.0;
    return s;
}

// Eligibility and key of a pair: resource priority -> key = score, must be > 0 (and feasible for
// the feasible-only domain); best-price -> key = -price among feasible nodes.
template <int PRIO, int DOM>
__device__ __forceinline__ bool pair_key(bool feas, int64_t rc, int64_t rm, int64_t rp, double rcf, double rmf,
                                         double rpf, int64_t ac, int64_t am, int64_t ap, double acf, double amf,
                                         double apf, float price, double *key) {
    if (PRIO == kPrioPrice) {
        *key = price_key(price);
        return feas;
    } else {
        if (DOM == kDomFeasible && !feas) return false;
        const double s = resource_score(rc, rm, rp, rcf, rmf, rpf, ac, am, ap, acf, amf, apf);
        *key = s;
        return s > 0.0;
    }
}

// ---- register-only wave butterflies (no LDS round trip) --------------------------------------
// Partner exchange for butterfly stage S (every lane ends with the all-reduce):
//   S0 quad_perm[1,0,3,2]  S1 quad_perm[2,3,0,1]  S2 row_half_mirror  S3 row_mirror   (DPP)
//   S4 v_permlane16_swap (lane ^ 16)               S5 v_permlane32_swap (lane ^ 32)   (gfx950)
// After S0..S1 a quad holds its result in every lane; half_mirror pairs the two quads of an
// 8-lane group, mirror the two 8-groups of a row, then rows exchange across 16 and 32.
template <int S>
__device__ __forceinline__ uint32_t wpartner(uint32_t v) {
    if constexpr (S == 0) return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false);
    else if constexpr (S == 1) return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false);
    else if constexpr (S == 2) return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false);
    else if constexpr (S == 3) return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false);
    else if constexpr (S == 4) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);  // {vdst_new, vsrc_new}
        return ((__lane_id() >> 4) & 1) ? r[0] : r[1];
    } else {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (__lane_id() >> 5) ? r[0] : r[1];
    }
}

template <int S>
__device__ __forceinline__ double wpartner_f64(double v) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint64_t hi = wpartner<S>((uint32_t)(u >> 32)), lo = wpartner<S>((uint32_t)u);
    return __longlong_as_double((long long)((hi << 32) | lo));
}

template <int S>
__device__ __forceinline__ void argbest_stage(double &key, int32_t &idx, int32_t &aux) {
    const double ok = wpartner_f64<S>(key);
    const int32_t oi = (int32_t)wpartner<S>((uint32_t)idx);
    const int32_t oa = (int32_t)wpartner<S>((uint32_t)aux);
    if (better(ok, oi, key, idx)) { key = ok; idx = oi; aux = oa; }
}

// Wave-wide (64 lanes) arg-best of (key desc, idx asc) carrying aux; every lane ends with the result.
__device__ __forceinline__ void wave_argbest(double &key, int32_t &idx, int32_t &aux) {
    argbest_stage<0>(key, idx, aux);
    argbest_stage<1>(key, idx, aux);
    argbest_stage<2>(key, idx, aux);
    argbest_stage<3>(key, idx, aux);
    argbest_stage<4>(key, idx, aux);
    argbest_stage<5>(key, idx, aux);
}

template <int S>
__device__ __forceinline__ int64_t sum_stage(int64_t v) {
    const uint64_t u = (uint64_t)v;
    const uint64_t hi = wpartner<S>((uint32_t)(u >> 32)), lo = wpartner<S>((uint32_t)u);
    return v + (int64_t)((hi << 32) | lo);
}

// Order-preserving map of a double key to uint64 (larger key -> larger code; -inf/none -> 0).
__device__ __forceinline__ uint64_t key_code(double k) {
    const uint64_t u = (uint64_t)__double_as_longlong(k);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

template <int S>
__device__ __forceinline__ uint64_t umax_stage(uint64_t v) {
    const uint64_t o = ((uint64_t)wpartner<S>((uint32_t)(v >> 32)) << 32) | wpartner<S>((uint32_t)v);
    return o > v ? o : v;
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
    v = umax_stage<0>(v); v = umax_stage<1>(v); v = umax_stage<2>(v);
    v = umax_stage<3>(v); v = umax_stage<4>(v); v = umax_stage<5>(v);
    return v;
}

__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
    v = sum_stage<0>(v); v = sum_stage<1>(v); v = sum_stage<2>(v);
    v = sum_stage<3>(v); v = sum_stage<4>(v); v = sum_stage<5>(v);
    return v;
}

template <int S>
__device__ __forceinline__ int32_t min_stage(int32_t v) {
    const int32_t o = (int32_t)wpartner<S>((uint32_t)v);
    return o < v ? o : v;
}

__device__ __forceinline__ int32_t wave_min_i32(int32_t v) {
    v = min_stage<0>(v); v = min_stage<1>(v); v = min_stage<2>(v);
    v = min_stage<3>(v); v = min_stage<4>(v); v = min_stage<5>(v);
    return v;
}

// Wave arg-best via a 64-bit order-preserving max, then (ties only) the lowest node index.
__device__ __forceinline__ void wave_argbest_fast(double &tk, int32_t &ti, int32_t &ts) {
    const uint64_t mine = ti == kNoIdx ? 0ull : key_code(tk);
    const uint64_t best = wave_max_u64(mine);
    if (best == 0) { tk = -__builtin_inf(); ti = kNoIdx; ts = -1; return; }
    const uint64_t tie = __ballot(mine == best);
    int src;
    if (__popcll(tie) == 1) {
        src = __ffsll((unsigned long long)tie) - 1;
    } else {
        const int32_t mi = wave_min_i32(mine == best ? ti : kNoIdx);
        src = __ffsll((unsigned long long)__ballot(mine == best && ti == mi)) - 1;
    }
    const uint64_t kb = (uint64_t)__double_as_longlong(tk);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(kb >> 32), src);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)kb, src);
    tk = __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
    ti = __builtin_amdgcn_readlane(ti, src);
    ts = __builtin_amdgcn_readlane(ts, src);
}

__device__ __forceinline__ double readlane_f64(double v, int src) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(b >> 32), src);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, src);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

}  // namespace ksched
