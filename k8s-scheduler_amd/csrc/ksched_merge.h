// ksched_merge.h -- device code shared by the stream pipeline (ksched_kernels.hip) and the persistent
// pipeline (ksched_persist.hip): per-lane sorted top-K insert and the per-pod rank merge of the score
// workgroups' lists.
#pragma once

#include "ksched_kernels.h"

namespace ksched {

template <int KC>
__device__ __forceinline__ void list_insert_ordered(double (&key)[KC], int32_t (&idx)[KC], double ck, int32_t ci) {
    bool moved = false;  // once placed, every later entry shifts down one slot
#pragma unroll
    for (int q = 0; q < KC; ++q) {
        const bool sw = moved || better(ck, ci, key[q], idx[q]);
        moved = sw;
        const double tk = key[q];
        const int32_t ti = idx[q];
        key[q] = sw ? ck : tk; idx[q] = sw ? ci : ti;
        ck = sw ? tk : ck; ci = sw ? ti : ci;
    }
}

// ------------------------------------------------------------------------------------------------
// Merge of one pod's workgroup lists (C_in <= 512 lists of KC entries, cut when full) into its K-entry
// Rec list: one 512-thread workgroup per pod, thread = list.  Selection by RANK, every compare
// independent (broadcast LDS reads of order-preserving 64-bit key codes; no serial rounds):
//   1. each list head is ranked within its wave; the K best heads of each wave survive;
//   2. the <= 8K survivors are ranked against each other; the K best heads' lists are kept -- every
//      entry of the pod's top K lies in one of them (K better heads exist for any entry outside them);
//   3. the kept lists' K*KC entries are ranked against each other; rank < K is the output position.
// Exact prefix: the result keeps only entries ranking at or above the best cutoff (the last entry of
// every cut input list) and is cut (flag in entry 0's pad) when any input was cut or entries were left
// over.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ bool code_better(uint64_t ca, int32_t ia, uint64_t cb, int32_t ib) {
    return ca > cb || (ca == cb && ia < ib);
}

// The merge's LDS (one pod at a time): MT lists of KC entries as key codes, plus the rank stages.
template <int KC, int K, int MT>
struct MergeSmem {
    static constexpr int W = MT / 64;
    uint64_t code[MT][KC];  // every list, as key codes (0 = empty)
    int32_t idx[MT][KC];
    uint64_t ccode[W * K];  // surviving heads
    int32_t cidx[W * K], clist[W * K];
    int32_t keep[K];        // list of global head rank g
    uint64_t ecode[K * KC]; // the kept lists' entries
    int32_t eidx[K * KC];
    uint64_t ocode[K];
    int32_t oidx[K];
    uint64_t wck[W];
    int32_t wci[W], wcut[W], wnv[W];
    int64_t wcnt[W];
};

struct BlockSync {
    __device__ void operator()() const { __syncthreads(); }
};

// tid: this thread's index among the MT merging threads; sync(): a barrier of exactly those threads
// (the whole workgroup in k_merge_pod, the merge waves of a pipeline workgroup in k_pipe).
template <int KC, int K, bool COH, int MT, typename Sync>
__device__ __forceinline__ void merge_pod_body(const MergeArgs &A, const int b, const int tid, MergeSmem<KC, K, MT> &sm,
                                               Sync sync) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical: win issue arbitration over co-resident score waves
    constexpr int W = MT / 64;
    auto &s_code = sm.code;
    auto &s_idx = sm.idx;
    auto &s_ccode = sm.ccode;
    auto &s_cidx = sm.cidx;
    auto &s_clist = sm.clist;
    auto &s_keep = sm.keep;
    auto &s_ecode = sm.ecode;
    auto &s_eidx = sm.eidx;
    auto &s_ocode = sm.ocode;
    auto &s_oidx = sm.oidx;
    auto &s_wck = sm.wck;
    auto &s_wci = sm.wci;
    auto &s_wcut = sm.wcut;
    auto &s_wnv = sm.wnv;
    auto &s_wcnt = sm.wcnt;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const bool dbg = A.dbg != nullptr;
    uint64_t ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (dbg) ts[0] = __builtin_amdgcn_s_memtime();
    const int64_t p0 = A.p0_known ? A.p0v : load_i64<COH>(A.cursor);
    if (p0 < 0 || p0 >= A.P || b >= A.B || p0 + b >= A.P) return;  // uniform over the merging threads
    const bool has = tid < A.C_in;
    uint64_t code[KC];
    int32_t idx[KC];
    int n = 0;
    int64_t cnt = 0;
    {
        const Cand *src = static_cast<const Cand *>(A.in) + ((size_t)b * A.C_in + (has ? tid : 0)) * KC;
#pragma unroll
        for (int q = 0; q < KC; ++q) {
            int32_t x;
            double kq;
            if (COH) {
                x = has ? (int32_t)(uint32_t)ld_coh(&src[q].idx) : kNoIdx;
                kq = has ? ld_coh_f64(&src[q].key) : 0.0;
            } else {
                x = has ? src[q].idx : kNoIdx;
                kq = has ? src[q].key : 0.0;
            }
            idx[q] = x;
            code[q] = x == kNoIdx ? 0ull : key_code(kq);
            n += x != kNoIdx;
        }
        if (has) cnt = load_i64<COH>(A.in_cnt + (size_t)b * A.C_in + tid);
    }
#pragma unroll
    for (int q = 0; q < KC; ++q) { s_code[tid][q] = code[q]; s_idx[tid][q] = idx[q]; }
    if (tid < W * K) { s_ccode[tid] = 0ull; s_cidx[tid] = kNoIdx; }  // empty survivor slots never rank
    if (dbg) { asm volatile("" ::"v"(code[0]), "v"(cnt)); ts[1] = __builtin_amdgcn_s_memtime(); }
    // wave partials: best cutoff (last entry of a full list), count, cut flag
    {
        const bool cut = n == KC;
        uint64_t ck = cut ? code[KC - 1] : 0ull;
        int32_t ci = cut ? idx[KC - 1] : kNoIdx;
        const uint64_t bc = wave_max_u64(ck);
        const int32_t bi = wave_min_i32((ck == bc && ci != kNoIdx) ? ci : kNoIdx);
        const int64_t wc = wave_sum_i64(cnt);
        const bool wcut = __ballot(cut) != 0;
        const int nv = __popcll(__ballot(idx[0] != kNoIdx));
        if (lane == 0) { s_wck[wave] = bc; s_wci[wave] = bi; s_wcut[wave] = wcut; s_wcnt[wave] = wc; s_wnv[wave] = nv; }
    }
    sync();
    // 1. rank each head within its wave (broadcast reads, independent compares; waves without lists idle)
    const int nw = (A.C_in + 63) / 64 < W ? (A.C_in + 63) / 64 : W;
    if (wave < nw) {
        int rank = 0;
        const int base = wave * 64;
#pragma unroll 16
        for (int t = 0; t < 64; ++t)
            rank += code_better(s_code[base + t][0], s_idx[base + t][0], code[0], idx[0]) ? 1 : 0;
        if (idx[0] != kNoIdx && rank < K) {
            s_ccode[wave * K + rank] = code[0];
            s_cidx[wave * K + rank] = idx[0];
            s_clist[wave * K + rank] = tid;
        }
    }
    if (dbg) ts[2] = __builtin_amdgcn_s_memtime();
    sync();
    if (dbg) ts[3] = __builtin_amdgcn_s_memtime();
    // 2. rank the survivors against each other
    int ntot = 0;  // valid heads in total (survivors: the first min(K, nv) slots of each wave)
    for (int w = 0; w < nw; ++w) ntot += s_wnv[w];
    if (tid < nw * K) {
        const int w = tid / K, p = tid % K;
        const int nvw = s_wnv[w] < K ? s_wnv[w] : K;
        if (p < nvw) {
            const uint64_t mc = s_ccode[tid];
            const int32_t mi = s_cidx[tid];
            int g = 0;
#pragma unroll 16
            for (int c = 0; c < nw * K; ++c) g += code_better(s_ccode[c], s_cidx[c], mc, mi) ? 1 : 0;
            if (g < K) s_keep[g] = s_clist[tid];
        }
    }
    if (dbg) ts[4] = __builtin_amdgcn_s_memtime();
    sync();
    // 3. gather the kept lists' entries (empty slots never rank), then rank them against each other
    const int nkeep = ntot < K ? ntot : K;
    const int ne = nkeep * KC;
    if (tid < K * KC) {
        const bool in = tid < ne;
        const int l = in ? s_keep[tid / KC] : 0;
        s_ecode[tid] = in ? s_code[l][tid % KC] : 0ull;
        s_eidx[tid] = in ? s_idx[l][tid % KC] : kNoIdx;
    }
    sync();
    int nvalid = 0;
    if (tid < ne) {
        const uint64_t mc = s_ecode[tid];
        const int32_t mi = s_eidx[tid];
        if (mi != kNoIdx) {
            int r = 0;
#pragma unroll 16
            for (int e = 0; e < K * KC; ++e) r += code_better(s_ecode[e], s_eidx[e], mc, mi) ? 1 : 0;
            if (r < K) { s_ocode[r] = mc; s_oidx[r] = mi; }
        }
    }
    if (wave == 0) {
        int cntv = 0;
        for (int e0 = 0; e0 < K * KC; e0 += 64) {
            const int e = e0 + lane;
            cntv += __popcll(__ballot(e < K * KC && s_eidx[e < K * KC ? e : 0] != kNoIdx));
        }
        nvalid = cntv;
    }
    if (dbg) ts[5] = __builtin_amdgcn_s_memtime();
    sync();
    if (wave != 0) return;
    uint64_t gk = 0ull;
    int32_t gi = kNoIdx;
    bool gcut = false;
    int64_t gcnt = 0;
    for (int w = 0; w < nw; ++w) {
        if (s_wci[w] != kNoIdx && (gi == kNoIdx || code_better(s_wck[w], s_wci[w], gk, gi))) { gk = s_wck[w]; gi = s_wci[w]; }
        gcut = gcut || s_wcut[w] != 0;
        gcnt += s_wcnt[w];
    }
    const int nout = nvalid < K ? nvalid : K;
    // lists outside the kept K, or entries beyond K, remain: the output is cut
    const bool left = ntot > nkeep || nvalid > K;
    const int32_t cut_out = (gcut || left) ? 1 : 0;
    if (lane < K) {
        Rec r{};
        const uint64_t mc = s_ocode[lane < nout ? lane : 0];
        const int32_t mi = s_oidx[lane < nout ? lane : 0];
        const bool ok = lane < nout && !(gi != kNoIdx && code_better(gk, gi, mc, mi));
        if (ok) {
            const NodeRec &nd = A.nodes[mi - A.node_offset];
            const uint64_t u = (mc >> 63) ? (mc & 0x7fffffffffffffffull) : ~mc;  // inverse of key_code
            r.key = __longlong_as_double((long long)u); r.idx = mi; r.valid = 1;
            r.a[0] = load_i64<COH>(&nd.a[0]); r.a[1] = load_i64<COH>(&nd.a[1]); r.a[2] = load_i64<COH>(&nd.a[2]);
            r.labels = nd.labels; r.price = nd.price;  // never written during a call
        } else {
            r.key = -__builtin_inf(); r.idx = kNoIdx; r.valid = 0;
        }
        r.pad = lane == 0 ? cut_out : 0;
        if (A.lds_msg) {
            const uint32_t *w = reinterpret_cast<const uint32_t *>(&r);
#pragma unroll
            for (int x = 0; x < kRecWords; ++x) A.lds_msg[lane * kRecWords + x] = w[x];
        } else {
            store_rec<COH>(A.out_rec + (size_t)b * K + lane, r);
        }
    }
    if (lane == 0) {
        if (A.lds_msg) {
            A.lds_msg[K * kRecWords] = (uint32_t)(uint64_t)gcnt;
            A.lds_msg[K * kRecWords + 1] = (uint32_t)((uint64_t)gcnt >> 32);
        } else {
            store_i64<COH>(A.out_fc + b, gcnt);
        }
    }
    if (dbg && lane == 0) {
        ts[6] = __builtin_amdgcn_s_memtime();
        for (int k = 1; k < 7; ++k) atomicAdd((unsigned long long *)&A.dbg[k - 1], (unsigned long long)(ts[k] - ts[k - 1]));
        atomicAdd((unsigned long long *)&A.dbg[7], 1ull);
    }
}



// ------------------------------------------------------------------------------------------------
// The same merge for the persistent pipeline's merge waves (MT = 256: W = 4 waves, one list per thread),
// with ONE barrier and no LDS-latency-bound loops: every selection is a register-only wave sort (DPP and
// permlane swaps):
//   A. (every wave) sort the wave's 64 list heads (wave_sort_desc); the K best go to LDS;
//   B. (wave 0, lane = one of the W*K <= 64 survivors) sort the survivors; the K best heads' lists are kept;
//   C. (wave 0, lane = one of the kept lists' K*KC <= 64 entries) sort the entries; lane r < K is output
//      position r (K*KC > 64: rank each entry by rotations, wave_rank).
// Then the exact-prefix cut and the Rec rows as in merge_pod_body.  (Round 6: the sorts replaced 63-rotation
// rank counts -- cycles per merge 20.3k -> 15.2k, c4 merge leg p50 15.2 -> 12.1 us.)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// how many lanes of this wave hold a (code, idx) better than (mc, mi) -- (code, idx) pairs are distinct.
// The 64 values travel around the wave by DPP wave_ror:1 (63 rotations, all VALU: no SGPR round trips).
__device__ __forceinline__ uint32_t wave_ror1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x13C, 0xF, 0xF, false);
}
__device__ __forceinline__ int wave_rank(uint64_t code, int32_t idx, uint64_t mc, int32_t mi) {
    uint32_t lo = (uint32_t)code, hi = (uint32_t)(code >> 32), ix = (uint32_t)idx;
    int r = code_better(code, idx, mc, mi) ? 1 : 0;
#pragma unroll 9
    for (int l = 1; l < 64; ++l) {
        lo = wave_ror1(lo); hi = wave_ror1(hi); ix = wave_ror1(ix);
        r += code_better(((uint64_t)hi << 32) | lo, (int32_t)ix, mc, mi) ? 1 : 0;
    }
    return r;
}

// ---- a wave-wide sort of 64 (code, idx) pairs, best first (key desc, idx asc): the bitonic network in its
// "flip" form, every comparator in one direction -- stage (M, HB) compares lane l with lane l ^ M, the lane
// with bit HB clear keeps the better.  M = 2^k - 1 is the flip of the aligned 2^k block (its mirror), M = 2^j
// the half-cleaners.  Every partner is a DPP or permlane swap (no LDS): xor 1/2/3 quad_perm, 7 row_half_mirror,
// 15 row_mirror, 8 row_ror:8, 4 = 7 then 3, 16/32 the permlane swaps, 31 and 63 their compositions.  21 stages
// of 3 partner words, a compare and 3 selects: ~2x fewer VALU instructions than 63 wave_ror1 rank rotations.
template <int M>
__device__ __forceinline__ uint32_t xpartner(uint32_t v) {
    if constexpr (M == 1 || M == 2) return wpartner<M - 1>(v);
    else if constexpr (M == 3) return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x1B, 0xF, 0xF, false);
    else if constexpr (M == 7) return wpartner<2>(v);
    else if constexpr (M == 15) return wpartner<3>(v);
    else if constexpr (M == 8) return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x128, 0xF, 0xF, false);
    else if constexpr (M == 4) return xpartner<3>(xpartner<7>(v));
    else if constexpr (M == 16) return wpartner<4>(v);
    else if constexpr (M == 32) return wpartner<5>(v);
    else if constexpr (M == 31) return xpartner<16>(xpartner<15>(v));
    else { static_assert(M == 63, "partner"); return xpartner<32>(xpartner<16>(xpartner<15>(v))); }
}
template <int M, int HB>
__device__ __forceinline__ void sort_stage(uint32_t &lo, uint32_t &hi, uint32_t &ix, const int lane) {
    const uint32_t plo = xpartner<M>(lo), phi = xpartner<M>(hi), pix = xpartner<M>(ix);
    const bool pb = code_better(((uint64_t)phi << 32) | plo, (int32_t)pix, ((uint64_t)hi << 32) | lo, (int32_t)ix);
    const bool take = (lane & HB) ? !pb : pb;
    lo = take ? plo : lo;
    hi = take ? phi : hi;
    ix = take ? pix : ix;
}
// Lanes hold sorted runs of RUN pairs (aligned; RUN = 1: anything): the stages of the block sizes above RUN merge
// them.  On return lane r holds the wave's rank-r pair.  (code, idx) pairs are distinct except empty ones (0, kNoIdx).
template <int RUN>
__device__ __forceinline__ void wave_sort_desc(uint64_t &code, int32_t &idx, const int lane) {
    static_assert(RUN == 1 || RUN == 2 || RUN == 4 || RUN == 8 || RUN == 16 || RUN == 32, "runs");
    uint32_t lo = (uint32_t)code, hi = (uint32_t)(code >> 32), ix = (uint32_t)idx;
    if constexpr (RUN <= 1) sort_stage<1, 1>(lo, hi, ix, lane);
    if constexpr (RUN <= 2) { sort_stage<3, 2>(lo, hi, ix, lane); sort_stage<1, 1>(lo, hi, ix, lane); }
    if constexpr (RUN <= 4) {
        sort_stage<7, 4>(lo, hi, ix, lane); sort_stage<2, 2>(lo, hi, ix, lane);
        sort_stage<1, 1>(lo, hi, ix, lane);
    }
    if constexpr (RUN <= 8) {
        sort_stage<15, 8>(lo, hi, ix, lane); sort_stage<4, 4>(lo, hi, ix, lane);
        sort_stage<2, 2>(lo, hi, ix, lane); sort_stage<1, 1>(lo, hi, ix, lane);
    }
    if constexpr (RUN <= 16) {
        sort_stage<31, 16>(lo, hi, ix, lane); sort_stage<8, 8>(lo, hi, ix, lane);
        sort_stage<4, 4>(lo, hi, ix, lane); sort_stage<2, 2>(lo, hi, ix, lane);
        sort_stage<1, 1>(lo, hi, ix, lane);
    }
    sort_stage<63, 32>(lo, hi, ix, lane); sort_stage<16, 16>(lo, hi, ix, lane);
    sort_stage<8, 8>(lo, hi, ix, lane); sort_stage<4, 4>(lo, hi, ix, lane);
    sort_stage<2, 2>(lo, hi, ix, lane); sort_stage<1, 1>(lo, hi, ix, lane);
    code = ((uint64_t)hi << 32) | lo;
    idx = (int32_t)ix;
}

// The touched-node screen's threshold of a merged list (lane = output entry; okm: the valid entries, a prefix;
// mc: this lane's key code): RN_f32(last key - 5e-5) when the list is cut, -inf otherwise, as f32 bits.
__device__ __forceinline__ int32_t list_thr_bits(bool cut, uint64_t okm, uint64_t mc) {
    const int nv = __popcll(okm);
    float t = -__builtin_inff();
    if (cut && nv > 0) {
        const uint64_t c = readlane_u64(mc, nv - 1);
        const uint64_t u = (c >> 63) ? (c & 0x7fffffffffffffffull) : ~c;  // inverse of key_code
        t = (float)(__longlong_as_double((long long)u) - 5e-5);
    }
    return (int32_t)__float_as_uint(t);
}

__device__ __forceinline__ void wave_lds_order() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int KC, int K, bool COH, int MT, typename Sync>
__device__ __forceinline__ void merge_pod_fast(const MergeArgs &A, const int b, const int tid, MergeSmem<KC, K, MT> &sm,
                                               Sync sync) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical: win issue arbitration over co-resident score waves
    constexpr int W = MT / 64;
    static_assert(W * K <= 64, "survivors must fit one wave");
    constexpr int E = K * KC;              // the kept lists' entries
    constexpr int EP = (E + 63) / 64;      // entries per lane
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const bool dbg = A.dbg != nullptr;
    uint64_t ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (dbg) ts[0] = __builtin_amdgcn_s_memtime();
    const int64_t p0 = A.p0_known ? A.p0v : load_i64<COH>(A.cursor);
    if (p0 < 0 || p0 >= A.P || b >= A.B || p0 + b >= A.P) return;  // uniform over the merging threads
    static_assert(COH, "merge_pod_fast reads the persistent pipeline's 16-B list records");
    const bool has = tid < A.C_in;
    uint64_t code[KC];
    int32_t idx[KC];
    int n = 0;
    int64_t cnt = 0;
    {
        // one 16-B sc1 load per entry {key, idx, pad}; entry 0's pad is the list's predicate count
        const __amdgpu_buffer_rsrc_t rs = coh_rsrc(A.in);
        const uint32_t off = (uint32_t)(((size_t)b * A.C_in + (has ? tid : 0)) * KC * sizeof(Cand));
        u32x4 w[KC];
#pragma unroll
        for (int q = 0; q < KC; ++q) w[q] = ld_coh16(rs, off + (uint32_t)(q * sizeof(Cand)));
        // every record carries its batch's tag (word 3, bits 16..31): a score workgroup arrives without draining
        // its record stores, so a record may still be on its way -- read again until all KC are this batch's
        if (has) {
            auto stale = [&]() {
                bool st = false;
#pragma unroll
                for (int q = 0; q < KC; ++q) st |= (w[q].w >> 16) != A.tag;
                return st;
            };
            for (int it = 0; stale(); ++it) {
                if (it == (1 << 22)) {  // (never seen: a lost store) -- report, do not hang
                    if (A.err) atomicCAS(A.err, 0, 11);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
#pragma unroll
                for (int q = 0; q < KC; ++q) w[q] = ld_coh16(rs, off + (uint32_t)(q * sizeof(Cand)));
            }
        }
#pragma unroll
        for (int q = 0; q < KC; ++q) {
            const int32_t x = has ? (int32_t)w[q].z : kNoIdx;
            const double kq = __longlong_as_double((long long)(((uint64_t)w[q].y << 32) | w[q].x));
            idx[q] = x;
            code[q] = x == kNoIdx ? 0ull : key_code(kq);
            n += x != kNoIdx;
        }
        cnt = has ? (int64_t)(w[0].w & 0xffffu) : 0;
    }
#pragma unroll
    for (int q = 0; q < KC; ++q) { sm.code[tid][q] = code[q]; sm.idx[tid][q] = idx[q]; }
    if (lane < K) { sm.ccode[wave * K + lane] = 0ull; sm.cidx[wave * K + lane] = kNoIdx; }  // before this wave's survivors
    if (dbg) { asm volatile("" ::"v"(code[0]), "v"(cnt)); ts[1] = __builtin_amdgcn_s_memtime(); }
    {   // wave partials: best cutoff (last entry of a full list), count, cut flag, valid heads
        const bool cut = n == KC;
        const uint64_t ck = cut ? code[KC - 1] : 0ull;
        const int32_t ci = cut ? idx[KC - 1] : kNoIdx;
        const uint64_t bc = wave_max_u64(ck);
        const int32_t bi = wave_min_i32((ck == bc && ci != kNoIdx) ? ci : kNoIdx);
        const int64_t wc = wave_sum_i64(cnt);
        const bool wcut = __ballot(cut) != 0;
        const int nv = __popcll(__ballot(idx[0] != kNoIdx));
        if (lane == 0) { sm.wck[wave] = bc; sm.wci[wave] = bi; sm.wcut[wave] = wcut; sm.wcnt[wave] = wc; sm.wnv[wave] = nv; }
    }
    // A. the wave's heads sorted: lanes < K hold its K best (an empty list's head (0, kNoIdx) sorts last and is
    // written as the empty slot it replaces)
    {
        uint64_t hc = code[0];
        int32_t hx = idx[0];
        wave_sort_desc<1>(hc, hx, lane);
        wave_lds_order();  // the slot initialisation above precedes every survivor write of this wave
        if (lane < K) { sm.ccode[wave * K + lane] = hc; sm.cidx[wave * K + lane] = hx; }
    }
    if (dbg) ts[2] = __builtin_amdgcn_s_memtime();
    sync();
    if (wave != 0) return;
    if (dbg) ts[3] = __builtin_amdgcn_s_memtime();
    // B. rank the survivors (lane = slot); the K best heads' lists hold the pod's top K
    int ntot = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) ntot += sm.wnv[w];
    {
        const bool in = lane < W * K;
        uint64_t sc = in ? sm.ccode[lane] : 0ull;
        int32_t si = in ? sm.cidx[lane] : kNoIdx;
        wave_sort_desc<K>(sc, si, lane);  // the W waves' K survivors are sorted runs: only the merge stages
        // a head's list is its score workgroup's: workgroup g holds the nodes idx - node_offset = g (mod C_in)
        if (lane < K && si != kNoIdx) sm.keep[lane] = (int32_t)((si - (int32_t)A.node_offset) % A.C_in);
    }
    wave_lds_order();
    if (dbg) ts[4] = __builtin_amdgcn_s_memtime();
    // C. the kept lists' entries (lane holds entries lane + 64 p), ranked against each other
    const int nkeep = ntot < K ? ntot : K;
    uint64_t ec[EP];
    int32_t ei[EP];
    int nvalid = 0;
#pragma unroll
    for (int p = 0; p < EP; ++p) {
        const int e = lane + 64 * p;
        const bool in = e < E && e / KC < nkeep;
        const int l = in ? sm.keep[e / KC] : 0;
        ec[p] = in ? sm.code[l][e % KC] : 0ull;
        ei[p] = in ? sm.idx[l][e % KC] : kNoIdx;
        nvalid += __popcll(__ballot(ei[p] != kNoIdx));
    }
    if constexpr (EP == 1) {
        wave_sort_desc<1>(ec[0], ei[0], lane);  // lane r: the rank-r entry
        if (lane < K && ei[0] != kNoIdx) { sm.ocode[lane] = ec[0]; sm.oidx[lane] = ei[0]; }
    } else {
#pragma unroll
        for (int p = 0; p < EP; ++p) {
            int r = 0;
#pragma unroll
            for (int p2 = 0; p2 < EP; ++p2) r += wave_rank(ec[p2], ei[p2], ec[p], ei[p]);
            if (ei[p] != kNoIdx && r < K) { sm.ocode[r] = ec[p]; sm.oidx[r] = ei[p]; }
        }
    }
    wave_lds_order();
    if (dbg) ts[5] = __builtin_amdgcn_s_memtime();
    uint64_t gk = 0ull;
    int32_t gi = kNoIdx;
    bool gcut = false;
    int64_t gcnt = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        if (sm.wci[w] != kNoIdx && (gi == kNoIdx || code_better(sm.wck[w], sm.wci[w], gk, gi))) { gk = sm.wck[w]; gi = sm.wci[w]; }
        gcut = gcut || sm.wcut[w] != 0;
        gcnt += sm.wcnt[w];
    }
    const int nout = nvalid < K ? nvalid : K;
    // lists outside the kept K, or entries beyond K, remain: the output is cut
    const bool left = ntot > nkeep || nvalid > K;
    const int32_t cut_out = (gcut || left) ? 1 : 0;
    const uint64_t mc = sm.ocode[lane < nout ? lane : 0];
    const int32_t mi = sm.oidx[lane < nout ? lane : 0];
    const bool ok = lane < K && lane < nout && !(gi != kNoIdx && code_better(gk, gi, mc, mi));
    // the commit's touched-node threshold (ksched_commit.h, kSkipKeyBits) in entry 1's pad: the last entry's key
    // - 5e-5 as an f32 below it, for a cut list; -inf (never skip) for a complete one
    const int32_t thr_bits = list_thr_bits(cut_out != 0, __ballot(ok), mc);
    if (lane < K) {
        Rec r{};
        if (ok) {
            const uint64_t u = (mc >> 63) ? (mc & 0x7fffffffffffffffull) : ~mc;  // inverse of key_code
            r.key = __longlong_as_double((long long)u); r.idx = mi; r.valid = 1;
            const NodeRec &nd = A.nodes[mi - A.node_offset];
            r.a[0] = load_i64<COH>(&nd.a[0]); r.a[1] = load_i64<COH>(&nd.a[1]); r.a[2] = load_i64<COH>(&nd.a[2]);
            r.labels = nd.labels; r.price = nd.price;  // never written during a call
        } else {
            r.key = -__builtin_inf(); r.idx = kNoIdx; r.valid = 0;
        }
        r.pad = lane == 0 ? cut_out : (lane == 1 ? thr_bits : 0);
        if (A.lds_msg) {
            const uint32_t *w = reinterpret_cast<const uint32_t *>(&r);
#pragma unroll
            for (int x = 0; x < kRecWords; ++x) A.lds_msg[lane * kRecWords + x] = w[x];
        } else {
            store_rec<COH>(A.out_rec + (size_t)b * K + lane, r);
        }
    }
    if (lane == 0) {
        if (A.lds_msg) {
            A.lds_msg[K * kRecWords] = (uint32_t)(uint64_t)gcnt;
            A.lds_msg[K * kRecWords + 1] = (uint32_t)((uint64_t)gcnt >> 32);
        } else {
            store_i64<COH>(A.out_fc + b, gcnt);
        }
    }
    if (dbg && lane == 0) {
        ts[6] = __builtin_amdgcn_s_memtime();
        for (int k = 1; k < 7; ++k) atomicAdd((unsigned long long *)&A.dbg[k - 1], (unsigned long long)(ts[k] - ts[k - 1]));
        atomicAdd((unsigned long long *)&A.dbg[7], 1ull);
    }
}

}  // namespace ksched
