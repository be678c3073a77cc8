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

constexpr int kPrioResource = 0;
constexpr int kPrioPrice = 1;
constexpr int kDomAll = 0;
constexpr int kDomFeasible = 1;
constexpr int32_t kNoIdx = 0x7fffffff;  // "no candidate" index (ranks after every real node)

// Node state as kept in HBM (AoS, 64 B: one s_load_dwordx16 when wave-uniform).
struct alignas(16) NodeRec {
    int64_t a[3];      // allocatable cpu (millicores), memory (KiB), pods = capacity - used
    uint64_t labels;   // label bitset (build extension)
    double af[3];      // (double)a[k], kept in sync with a[k] by every writer
    float price;       // node price (best-price priority)
    uint32_t pad;
};
static_assert(sizeof(NodeRec) == 64, "NodeRec layout");

// One candidate of a partial top-K list (score kernels -> merge kernels).
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
        *key = -(double)price;
        return feas;
    } else {
        if (DOM == kDomFeasible && !feas) return false;
        const double s = resource_score(rc, rm, rp, rcf, rmf, rpf, ac, am, ap, acf, amf, apf);
        *key = s;
        return s > 0.0;
    }
}

// Wave-wide (64 lanes) arg-best of (key, idx, aux) by butterfly; every lane ends with the result.
__device__ __forceinline__ void wave_argbest(double &key, int32_t &idx, int32_t &aux) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const double ok = __shfl_xor(key, off, 64);
        const int32_t oi = __shfl_xor(idx, off, 64);
        const int32_t oa = __shfl_xor(aux, off, 64);
        if (better(ok, oi, key, idx)) { key = ok; idx = oi; aux = oa; }
    }
}

__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__device__ __forceinline__ int32_t wave_min_i32(int32_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const int32_t o = __shfl_xor(v, off, 64);
        v = o < v ? o : v;
    }
    return v;
}

}  // namespace ksched
