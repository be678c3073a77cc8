// ksched_kernels.hip -- CDNA4 (gfx950) kernels of the scheduling core.  Compiled with
// -ffp-contract=off: every double op rounds individually, exactly like the Go reference.
#include <hip/hip_runtime.h>

#include "ksched_kernels.h"

namespace ksched {

namespace {

__device__ __forceinline__ uint64_t ld_granule(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_granule(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// Exact mode: one persistent launch schedules every pod in order.
//   - workgroup g owns nodes [g*per_wg, (g+1)*per_wg); thread t holds nodes g*per_wg + t + k*256
//     (k < NPT) in registers for the whole launch;
//   - per pod: each lane scores its nodes (predicate.go:127-150 + priorities.go:45-50), wave
//     butterfly arg-best + count, 4-wave combine through LDS;
//   - G > 1: wave 0 publishes the workgroup's (key, idx, count) as four tagged 8-byte granules
//     (write-through sc1 stores, epoch = pod + 1) and sweeps all G records until every tag matches
//     (MI355X_MICROARCH "handoff-1to1"/"allgather" R2 granules: no fences needed); every workgroup
//     then folds the same G records into the same decision;
//   - the owner lane of the winning node commits it in registers; nodes are written back at exit.
// ------------------------------------------------------------------------------------------------
template <int NPT, int PRIO, int DOM, bool LAB>
__global__ __launch_bounds__(kExactBlock) void k_exact(ExactArgs A) {
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int g = blockIdx.x;
    const int64_t lo = (int64_t)g * A.per_wg;
    const int64_t hi = (lo + A.per_wg < A.n) ? lo + A.per_wg : A.n;

    int64_t a0[NPT], a1[NPT], a2[NPT];
    uint64_t lab[NPT];
    float pr[NPT];
    int32_t id[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        const int64_t j = lo + tid + (int64_t)k * kExactBlock;
        if (j < hi) {
            const NodeRec nd = A.nodes[j];
            a0[k] = nd.a[0]; a1[k] = nd.a[1]; a2[k] = nd.a[2];
            lab[k] = nd.labels; pr[k] = nd.price; id[k] = (int32_t)j;
        } else {
            a0[k] = a1[k] = a2[k] = 0; lab[k] = 0; pr[k] = 0.f; id[k] = kNoIdx;
        }
    }

    __shared__ double s_key[2][kExactBlock / 64];
    __shared__ int32_t s_idx[2][kExactBlock / 64];
    __shared__ int64_t s_cnt[2][kExactBlock / 64];
    __shared__ double s_rkey[2];
    __shared__ int32_t s_ridx[2];
    __shared__ int64_t s_rcnt[2];
    __shared__ int32_t s_abort;
    if (tid == 0) s_abort = 0;

    for (int64_t i = 0; i < A.pods.p; ++i) {
        const int par = (int)(i & 1);
        const int64_t rc = A.pods.rc[i], rm = A.pods.rm[i], rp = A.pods.rp[i];
        const uint64_t sel = LAB ? A.pods.sel[i] : 0;
        const double rcf = (double)rc, rmf = (double)rm, rpf = (double)rp;
        double bk = -__builtin_inf();
        int32_t bi = kNoIdx;
        int64_t cnt = 0;
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            if (id[k] != kNoIdx) {
                const bool f = fits(rc, rm, rp, sel, a0[k], a1[k], a2[k], lab[k], LAB);
                cnt += f;
                double key;
                if (pair_key<PRIO, DOM>(f, rc, rm, rp, rcf, rmf, rpf, a0[k], a1[k], a2[k], (double)a0[k],
                                        (double)a1[k], (double)a2[k], pr[k], &key) &&
                    better(key, id[k], bk, bi)) {
                    bk = key;
                    bi = id[k];
                }
            }
        }
        int32_t aux = 0;
        wave_argbest(bk, bi, aux);
        cnt = wave_sum_i64(cnt);
        if (lane == 0) { s_key[par][wave] = bk; s_idx[par][wave] = bi; s_cnt[par][wave] = cnt; }
        __syncthreads();
        double gk = s_key[par][0];
        int32_t gi = s_idx[par][0];
        int64_t gc = s_cnt[par][0];
#pragma unroll
        for (int w = 1; w < kExactBlock / 64; ++w) {
            gc += s_cnt[par][w];
            if (better(s_key[par][w], s_idx[par][w], gk, gi)) { gk = s_key[par][w]; gi = s_idx[par][w]; }
        }
        if (A.G > 1) {
            if (wave == 0) {
                const uint64_t ep = (uint64_t)(uint32_t)(i + 1) << 32;
                uint64_t *mine = A.slots + ((size_t)par * A.G + g) * 4;
                const uint64_t kb = (uint64_t)__double_as_longlong(gk);
                if (lane < 4) {
                    const uint32_t v = lane == 0 ? (uint32_t)(kb >> 32)
                                     : lane == 1 ? (uint32_t)kb
                                     : lane == 2 ? (uint32_t)gi
                                                 : (uint32_t)gc;
                    st_granule(mine + lane, ep | v);
                }
                const int64_t t0 = wall_clock64();
                double fk;
                int32_t fi;
                int64_t fc;
                for (;;) {
                    bool ok = true;
                    fk = -__builtin_inf(); fi = kNoIdx; fc = 0;
                    for (int g2 = lane; g2 < A.G; g2 += 64) {
                        const uint64_t *sl = A.slots + ((size_t)par * A.G + g2) * 4;
                        const uint64_t x0 = ld_granule(sl), x1 = ld_granule(sl + 1);
                        const uint64_t x2 = ld_granule(sl + 2), x3 = ld_granule(sl + 3);
                        ok &= ((x0 & 0xffffffff00000000ull) == ep) & ((x1 & 0xffffffff00000000ull) == ep) &
                              ((x2 & 0xffffffff00000000ull) == ep) & ((x3 & 0xffffffff00000000ull) == ep);
                        const double k2 = __longlong_as_double((long long)((x0 << 32) | (x1 & 0xffffffffull)));
                        const int32_t i2 = (int32_t)(uint32_t)x2;
                        fc += (int64_t)(uint32_t)x3;
                        if (better(k2, i2, fk, fi)) { fk = k2; fi = i2; }
                    }
                    if (__all(ok)) break;
                    if (wall_clock64() - t0 > A.timeout_ticks) {
                        if (lane == 0) { atomicExch(A.err, 1); s_abort = 1; }
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                int32_t aux2 = 0;
                wave_argbest(fk, fi, aux2);
                fc = wave_sum_i64(fc);
                if (lane == 0) { s_rkey[par] = fk; s_ridx[par] = fi; s_rcnt[par] = fc; }
            }
            __syncthreads();
            if (s_abort) break;
            gk = s_rkey[par]; gi = s_ridx[par]; gc = s_rcnt[par];
        }
        int32_t oidx;
        double osc = 0.0;
        if (gc == 0) {
            oidx = -1;  // NO_FIT (anchor/schedule.go:74-76)
        } else if (gi == kNoIdx) {
            oidx = -2;  // NO_POSITIVE_SCORE (reference: nil node, anchor/priorities.go:55-62)
        } else {
            oidx = gi;
            osc = PRIO == kPrioPrice ? -gk : gk;
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                if (id[k] == gi) {  // commit: used += request, ONE pod (anchor/predicate.go:99-102)
                    a0[k] = wsub(a0[k], rc); a1[k] = wsub(a1[k], rm); a2[k] = wsub(a2[k], 1);
                }
            }
        }
        if (g == 0 && tid == 0) {
            A.out.idx[i] = oidx;
            A.out.score[i] = osc;
            A.out.feas[i] = (int32_t)gc;
        }
    }
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        if (id[k] != kNoIdx) {
            NodeRec *nd = A.nodes + id[k];
            nd->a[0] = a0[k]; nd->a[1] = a1[k]; nd->a[2] = a2[k];
            nd->af[0] = (double)a0[k]; nd->af[1] = (double)a1[k]; nd->af[2] = (double)a2[k];
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Batched mode, stage 1: fused predicate + score + per-lane top-K.  Lane = pod of the batch, wave =
// one node chunk; node rows are wave-uniform (scalar loads of the 64-B NodeRec).  The list is kept
// sorted by (key desc, idx asc) with a register bubble insert.
// ------------------------------------------------------------------------------------------------
template <int K, int PRIO, int DOM, bool LAB>
__global__ __launch_bounds__(256) void k_score_topk(ScoreArgs A) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int chunk = blockIdx.x * 4 + wave;
    if (chunk >= A.n_chunks) return;
    const int64_t p0 = *A.cursor;
    if (p0 >= A.pods.p) return;
    const int b = blockIdx.y * 64 + lane;
    const int64_t pod = p0 + b;
    const bool active = (b < A.B) && (pod < A.pods.p);
    const int64_t rc = active ? A.pods.rc[pod] : 0;
    const int64_t rm = active ? A.pods.rm[pod] : 0;
    const int64_t rp = active ? A.pods.rp[pod] : 0;
    const uint64_t sel = (LAB && active) ? A.pods.sel[pod] : 0;
    const double rcf = (double)rc, rmf = (double)rm, rpf = (double)rp;

    double key[K];
    int32_t idx[K];
#pragma unroll
    for (int q = 0; q < K; ++q) { key[q] = -__builtin_inf(); idx[q] = kNoIdx; }
    int64_t cnt = 0;
    const int64_t j0 = (int64_t)chunk * A.S;
    const int64_t j1 = (j0 + A.S < A.n_local) ? j0 + A.S : A.n_local;
    for (int64_t j = j0; j < j1; ++j) {
        const NodeRec &nd = A.nodes[j];
        const int64_t ac = nd.a[0], am = nd.a[1], ap = nd.a[2];
        const bool f = fits(rc, rm, rp, sel, ac, am, ap, nd.labels, LAB);
        cnt += f;
        double k;
        if (pair_key<PRIO, DOM>(f, rc, rm, rp, rcf, rmf, rpf, ac, am, ap, nd.af[0], nd.af[1], nd.af[2], nd.price,
                                &k)) {
            int32_t ci = (int32_t)(A.node_offset + j);
            if (better(k, ci, key[K - 1], idx[K - 1])) {
                double ck = k;
#pragma unroll
                for (int q = 0; q < K; ++q) {
                    if (better(ck, ci, key[q], idx[q])) {
                        const double tk = key[q];
                        const int32_t ti = idx[q];
                        key[q] = ck; idx[q] = ci;
                        ck = tk; ci = ti;
                    }
                }
            }
        }
    }
    if (!active) return;
    Cand *dst = A.part + ((size_t)b * A.n_chunks + chunk) * K;
#pragma unroll
    for (int q = 0; q < K; ++q) { dst[q].key = key[q]; dst[q].idx = idx[q]; dst[q].pad = 0; }
    A.part_cnt[(size_t)b * A.n_chunks + chunk] = cnt;
}

// ------------------------------------------------------------------------------------------------
// Merge: one wave per (pod, group of <= 64 sorted lists).  Each lane stages one list in LDS; K
// rounds of wave arg-best over the lanes' heads (the winning lane advances).  Final stage writes
// Rec entries carrying the node snapshot state; INPUT_REC merges the ranks' Rec lists.
// ------------------------------------------------------------------------------------------------
template <int K, bool INPUT_REC, bool FINAL>
__global__ __launch_bounds__(64) void k_merge(MergeArgs A) {
    __shared__ double s_key[64 * K];
    __shared__ int32_t s_idx[64 * K];
    const int lane = threadIdx.x;
    const int grp = blockIdx.x;
    const int b = blockIdx.y;
    const int64_t p0 = *A.cursor;
    if (p0 >= A.P || b >= A.B || p0 + b >= A.P) return;
    const int list = grp * 64 + lane;
    const bool has = list < A.C_in;
    int64_t cnt = 0;
    if (has) {
        if (INPUT_REC) {
            const char *blk = static_cast<const char *>(A.in) + (size_t)list * A.rank_stride;
            const Rec *src = reinterpret_cast<const Rec *>(blk) + (size_t)b * K;
#pragma unroll
            for (int q = 0; q < K; ++q) {
                s_key[lane * K + q] = src[q].valid ? src[q].key : -__builtin_inf();
                s_idx[lane * K + q] = src[q].valid ? src[q].idx : kNoIdx;
            }
            cnt = reinterpret_cast<const int64_t *>(blk + (size_t)A.B * K * sizeof(Rec))[b];
        } else {
            const Cand *src = static_cast<const Cand *>(A.in) + ((size_t)b * A.C_in + list) * K;
#pragma unroll
            for (int q = 0; q < K; ++q) { s_key[lane * K + q] = src[q].key; s_idx[lane * K + q] = src[q].idx; }
            cnt = A.in_cnt[(size_t)b * A.C_in + list];
        }
    }
    cnt = wave_sum_i64(cnt);
    __syncthreads();
    int h = 0;
    double mk = -__builtin_inf();
    int32_t mi = kNoIdx, msrc = -1;
    for (int r = 0; r < K; ++r) {
        double k = (has && h < K) ? s_key[lane * K + h] : -__builtin_inf();
        int32_t ix = (has && h < K) ? s_idx[lane * K + h] : kNoIdx;
        int32_t src = lane * K + h;
        wave_argbest(k, ix, src);
        if (ix == kNoIdx) break;  // wave-uniform
        if (src == lane * K + h) ++h;
        if (lane == r) { mk = k; mi = ix; msrc = src; }
    }
    if (!FINAL) {
        if (lane < K) {
            Cand *dst = A.out + ((size_t)b * A.C_out + grp) * K + lane;
            dst->key = mk; dst->idx = mi; dst->pad = 0;
        }
        if (lane == 0) A.out_cnt[(size_t)b * A.C_out + grp] = cnt;
    } else {
        if (lane < K) {
            Rec r{};
            if (mi != kNoIdx) {
                if (INPUT_REC) {
                    const int srcl = msrc / K, srcq = msrc % K;
                    const char *blk = static_cast<const char *>(A.in) + (size_t)(grp * 64 + srcl) * A.rank_stride;
                    r = reinterpret_cast<const Rec *>(blk)[(size_t)b * K + srcq];
                } else {
                    const NodeRec &nd = A.nodes[mi - A.node_offset];
                    r.key = mk; r.idx = mi; r.valid = 1;
                    r.a[0] = nd.a[0]; r.a[1] = nd.a[1]; r.a[2] = nd.a[2];
                    r.labels = nd.labels; r.price = nd.price; r.pad = 0;
                }
            } else {
                r.key = -__builtin_inf(); r.idx = kNoIdx; r.valid = 0;
            }
            A.out_rec[(size_t)b * K + lane] = r;
        }
        if (lane == 0) A.out_fc[b] = cnt;
    }
}

// ------------------------------------------------------------------------------------------------
// Ordered commit of one batch (one workgroup).  For pod i of the batch, with T = nodes committed by
// pods < i of this batch (LDS table; s0 = snapshot state, cur = current state):
//   fc   = fc0[i] - sum_T fits(s0) + sum_T fits(cur)                          (predicate count)
//   t*   = best of T re-scored at cur;  u* = first list entry not in T (exact: untouched)
//   list full and all touched: t* must beat list[K-1] (every unlisted untouched node ranks below
//   it), otherwise the batch stops before pod i (overflow) and the next batch restarts there.
// ------------------------------------------------------------------------------------------------
template <int K, int PRIO, int DOM, bool LAB>
__global__ __launch_bounds__(kCommitBlock) void k_commit(CommitArgs A) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint32_t *bitmap = reinterpret_cast<uint32_t *>(smem);
    Touched *T = reinterpret_cast<Touched *>(smem + (size_t)A.bitmap_words * 4);
    __shared__ double s_tk[kCommitBlock / 64];
    __shared__ int32_t s_ti[kCommitBlock / 64], s_ts[kCommitBlock / 64], s_uq[kCommitBlock / 64];
    __shared__ int32_t s_cv[kCommitBlock / 64];
    __shared__ int64_t s_df[kCommitBlock / 64];
    __shared__ int32_t s_nT, s_stop;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t p0 = *A.cursor;
    if (p0 >= A.pods.p) return;
    const int64_t nb = (A.pods.p - p0 < A.B) ? A.pods.p - p0 : A.B;
    for (int w = tid; w < A.bitmap_words; w += kCommitBlock) bitmap[w] = 0;
    if (tid == 0) { s_nT = 0; s_stop = 0; }
    __syncthreads();

    int64_t done = nb;
    int64_t placed = 0;
    for (int64_t i = 0; i < nb; ++i) {
        const int64_t pod = p0 + i;
        const int64_t rc = A.pods.rc[pod], rm = A.pods.rm[pod], rp = A.pods.rp[pod];
        const uint64_t sel = LAB ? A.pods.sel[pod] : 0;
        const double rcf = (double)rc, rmf = (double)rm, rpf = (double)rp;
        const int nT = s_nT;
        int64_t df = 0;
        double tk = -__builtin_inf();
        int32_t ti = kNoIdx, ts = -1;
        for (int t = tid; t < nT; t += kCommitBlock) {
            const Touched &x = T[t];
            const bool f0 = fits(rc, rm, rp, sel, x.s0[0], x.s0[1], x.s0[2], x.labels, LAB);
            const bool f1 = fits(rc, rm, rp, sel, x.cur[0], x.cur[1], x.cur[2], x.labels, LAB);
            df += (int64_t)f1 - (int64_t)f0;
            double k;
            if (pair_key<PRIO, DOM>(f1, rc, rm, rp, rcf, rmf, rpf, x.cur[0], x.cur[1], x.cur[2], (double)x.cur[0],
                                    (double)x.cur[1], (double)x.cur[2], x.price, &k) &&
                better(k, x.idx, tk, ti)) {
                tk = k; ti = x.idx; ts = t;
            }
        }
        int32_t uq = K, cv = 0;
        if (tid < K) {
            const Rec &L = A.lists[(size_t)i * K + tid];
            if (L.valid) {
                cv = 1;
                const uint32_t bit = bitmap[(uint32_t)L.idx >> 5] & (1u << ((uint32_t)L.idx & 31));
                if (!bit) uq = tid;
            }
        }
        wave_argbest(tk, ti, ts);
        df = wave_sum_i64(df);
        uq = wave_min_i32(uq);
        cv = (int32_t)wave_sum_i64(cv);
        if (lane == 0) { s_tk[wave] = tk; s_ti[wave] = ti; s_ts[wave] = ts; s_uq[wave] = uq; s_cv[wave] = cv; s_df[wave] = df; }
        __syncthreads();
        if (tid == 0) {
            for (int w = 1; w < kCommitBlock / 64; ++w) {
                df += s_df[w];
                uq = s_uq[w] < uq ? s_uq[w] : uq;
                cv += s_cv[w];
                if (better(s_tk[w], s_ti[w], tk, ti)) { tk = s_tk[w]; ti = s_ti[w]; ts = s_ts[w]; }
            }
            const int64_t fc = A.fc0[i] + df;
            int32_t oidx = -1;
            double osc = 0.0;
            bool stop = false;
            if (fc != 0) {
                int slot = -1;
                const Rec *u = nullptr;
                double wk = 0.0;
                int32_t wi = kNoIdx;
                if (uq < cv) {
                    u = &A.lists[(size_t)i * K + uq];
                    if (ti != kNoIdx && better(tk, ti, u->key, u->idx)) { wk = tk; wi = ti; slot = ts; u = nullptr; }
                    else { wk = u->key; wi = u->idx; }
                } else if (cv < K) {
                    if (ti != kNoIdx) { wk = tk; wi = ti; slot = ts; }
                } else {
                    const Rec &last = A.lists[(size_t)i * K + (K - 1)];
                    if (ti != kNoIdx && better(tk, ti, last.key, last.idx)) { wk = tk; wi = ti; slot = ts; }
                    else stop = true;
                }
                if (!stop) {
                    if (wi == kNoIdx) {
                        oidx = -2;
                    } else {
                        if (u) {  // first touch of this node in the batch
                            slot = s_nT++;
                            Touched &x = T[slot];
                            x.idx = u->idx; x.pad = 0;
                            x.s0[0] = x.cur[0] = u->a[0];
                            x.s0[1] = x.cur[1] = u->a[1];
                            x.s0[2] = x.cur[2] = u->a[2];
                            x.labels = u->labels; x.price = u->price; x.pad2 = 0;
                            bitmap[(uint32_t)u->idx >> 5] |= 1u << ((uint32_t)u->idx & 31);
                        }
                        Touched &x = T[slot];
                        x.cur[0] = wsub(x.cur[0], rc); x.cur[1] = wsub(x.cur[1], rm); x.cur[2] = wsub(x.cur[2], 1);
                        oidx = wi;
                        osc = PRIO == kPrioPrice ? -wk : wk;
                        ++placed;
                    }
                }
            }
            if (stop) {
                s_stop = 1;
            } else {
                A.out.idx[pod] = oidx;
                A.out.score[pod] = osc;
                A.out.feas[pod] = (int32_t)fc;
            }
        }
        __syncthreads();
        if (s_stop) { done = i; break; }
    }
    // write back committed nodes of this shard
    const int nT = s_nT;
    for (int t = tid; t < nT; t += kCommitBlock) {
        const Touched &x = T[t];
        const int64_t j = (int64_t)x.idx - A.node_lo;
        if (j >= 0 && j < A.n_local) {
            NodeRec *nd = A.nodes + j;
            nd->a[0] = x.cur[0]; nd->a[1] = x.cur[1]; nd->a[2] = x.cur[2];
            nd->af[0] = (double)x.cur[0]; nd->af[1] = (double)x.cur[1]; nd->af[2] = (double)x.cur[2];
        }
    }
    if (tid == 0) {
        *A.cursor = p0 + done;
        A.stats[0] += 1;
        A.stats[1] += (done < nb) ? 1 : 0;
        A.stats[2] += placed;
    }
}

// ------------------------------------------------------------------------------------------------
// Ordered commit, single-wave sequencer (the default).  Same decision rule as k_commit, but:
//   - one wave, no barriers: every per-pod reduction is a wave butterfly and every lane evaluates the
//     (wave-uniform) decision itself; the touched table and node bitmap live in LDS;
//   - the batch's requests and feasible counts are staged into LDS once, up front;
//   - lane q < K holds candidate q of the current pod and already has the NEXT pod's candidate load
//     in flight (software prefetch), so no dependent global load sits on the serial path.
// ------------------------------------------------------------------------------------------------
struct alignas(8) PodStage {
    int64_t rc, rm, rp;
    uint64_t sel;
    int64_t fc0;
};

template <int K, int PRIO, int DOM, bool LAB>
__global__ __launch_bounds__(64) void k_commit1(CommitArgs A) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint32_t *bitmap = reinterpret_cast<uint32_t *>(smem);
    Touched *T = reinterpret_cast<Touched *>(smem + (size_t)A.bitmap_words * 4);
    PodStage *PS = reinterpret_cast<PodStage *>(smem + (size_t)A.bitmap_words * 4 + (size_t)A.B * sizeof(Touched));
    const int lane = threadIdx.x;
    const int64_t p0 = *A.cursor;
    if (p0 >= A.pods.p) return;
    const int nb = (int)((A.pods.p - p0 < A.B) ? A.pods.p - p0 : A.B);
    for (int w = lane; w < A.bitmap_words; w += 64) bitmap[w] = 0;
    for (int b = lane; b < nb; b += 64) {
        PodStage s;
        s.rc = A.pods.rc[p0 + b]; s.rm = A.pods.rm[p0 + b]; s.rp = A.pods.rp[p0 + b];
        s.sel = LAB ? A.pods.sel[p0 + b] : 0;
        s.fc0 = A.fc0[b];
        PS[b] = s;
    }
    Rec nxt;
    if (lane < K) nxt = A.lists[lane];
    else { nxt.valid = 0; nxt.idx = kNoIdx; nxt.key = -__builtin_inf(); }
    __syncthreads();  // one wave: orders the staging writes before the loop's reads

    int nT = 0;
    int done = nb;
    int64_t placed = 0;
    for (int i = 0; i < nb; ++i) {
        const Rec my = nxt;
        if (lane < K && i + 1 < nb) nxt = A.lists[(size_t)(i + 1) * K + lane];
        const PodStage ps = PS[i];
        const int64_t rc = ps.rc, rm = ps.rm, rp = ps.rp;
        const uint64_t sel = ps.sel;
        const double rcf = (double)rc, rmf = (double)rm, rpf = (double)rp;
        // re-score the nodes already committed in this batch
        int64_t df = 0;
        double tk = -__builtin_inf();
        int32_t ti = kNoIdx, ts = -1;
        for (int t = lane; t < nT; t += 64) {
            const Touched &x = T[t];
            const bool f0 = fits(rc, rm, rp, sel, x.s0[0], x.s0[1], x.s0[2], x.labels, LAB);
            const bool f1 = fits(rc, rm, rp, sel, x.cur[0], x.cur[1], x.cur[2], x.labels, LAB);
            df += (int64_t)f1 - (int64_t)f0;
            double k;
            if (pair_key<PRIO, DOM>(f1, rc, rm, rp, rcf, rmf, rpf, x.cur[0], x.cur[1], x.cur[2], (double)x.cur[0],
                                    (double)x.cur[1], (double)x.cur[2], x.price, &k) &&
                better(k, x.idx, tk, ti)) {
                tk = k; ti = x.idx; ts = t;
            }
        }
        // candidate list: valid prefix, first entry not committed in this batch
        const bool valid = lane < K && my.valid;
        const bool untouched = valid && !(bitmap[(uint32_t)my.idx >> 5] & (1u << ((uint32_t)my.idx & 31)));
        const uint64_t vmask = __ballot(valid);
        const uint64_t umask = __ballot(untouched);
        const int cv = __popcll(vmask);
        const int uq = umask ? __ffsll((unsigned long long)umask) - 1 : K;
        wave_argbest(tk, ti, ts);
        df = wave_sum_i64(df);
        const int64_t fc = ps.fc0 + df;
        int32_t oidx = -1;
        double osc = 0.0;
        int kind = 0;  // 0 none, 1 winner from list (new touch), 2 winner already touched, 3 overflow
        double wk = 0.0;
        int32_t wi = kNoIdx;
        if (fc != 0) {
            if (uq < cv) {
                const double uk = __shfl(my.key, uq, 64);
                const int32_t ui = __shfl(my.idx, uq, 64);
                if (ti != kNoIdx && better(tk, ti, uk, ui)) { kind = 2; wk = tk; wi = ti; }
                else { kind = 1; wk = uk; wi = ui; }
            } else if (cv < K) {
                if (ti != kNoIdx) { kind = 2; wk = tk; wi = ti; }
            } else {
                const double lk = __shfl(my.key, K - 1, 64);
                const int32_t li = __shfl(my.idx, K - 1, 64);
                if (ti != kNoIdx && better(tk, ti, lk, li)) { kind = 2; wk = tk; wi = ti; }
                else kind = 3;
            }
        }
        if (kind == 3) { done = i; break; }  // wave-uniform
        if (fc != 0) {
            if (kind == 0) {
                oidx = -2;
            } else {
                oidx = wi;
                osc = PRIO == kPrioPrice ? -wk : wk;
                ++placed;
                if (kind == 1) {
                    if (lane == uq) {  // first touch: the holder of the candidate opens the slot
                        Touched &x = T[nT];
                        x.idx = my.idx; x.pad = 0;
                        x.s0[0] = my.a[0]; x.s0[1] = my.a[1]; x.s0[2] = my.a[2];
                        x.cur[0] = wsub(my.a[0], rc); x.cur[1] = wsub(my.a[1], rm); x.cur[2] = wsub(my.a[2], 1);
                        x.labels = my.labels; x.price = my.price; x.pad2 = 0;
                        bitmap[(uint32_t)my.idx >> 5] |= 1u << ((uint32_t)my.idx & 31);
                    }
                    ++nT;
                } else if (lane == 0) {
                    Touched &x = T[ts];
                    x.cur[0] = wsub(x.cur[0], rc); x.cur[1] = wsub(x.cur[1], rm); x.cur[2] = wsub(x.cur[2], 1);
                }
            }
        }
        if (lane == 0) {
            const int64_t pod = p0 + i;
            A.out.idx[pod] = oidx;
            A.out.score[pod] = osc;
            A.out.feas[pod] = (int32_t)fc;
        }
    }
    __syncthreads();
    for (int t = lane; t < nT; t += 64) {
        const Touched &x = T[t];
        const int64_t j = (int64_t)x.idx - A.node_lo;
        if (j >= 0 && j < A.n_local) {
            NodeRec *nd = A.nodes + j;
            nd->a[0] = x.cur[0]; nd->a[1] = x.cur[1]; nd->a[2] = x.cur[2];
            nd->af[0] = (double)x.cur[0]; nd->af[1] = (double)x.cur[1]; nd->af[2] = (double)x.cur[2];
        }
    }
    if (lane == 0) {
        *A.cursor = p0 + done;
        A.stats[0] += 1;
        A.stats[1] += (done < nb) ? 1 : 0;
        A.stats[2] += placed;
    }
}

__global__ void k_apply_delta(NodeRec *nodes, int64_t n, int64_t k, const int32_t *idx, const int64_t *d) {
    // Sequential in one lane: deltas may repeat a node and must apply in order (wrapping adds).
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    for (int64_t i = 0; i < k; ++i) {
        const int64_t j = idx[i];
        if (j < 0 || j >= n) continue;
        NodeRec *nd = nodes + j;
        for (int r = 0; r < 3; ++r) {
            nd->a[r] = (int64_t)((uint64_t)nd->a[r] + (uint64_t)d[r * k + i]);
            nd->af[r] = (double)nd->a[r];
        }
    }
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
namespace {

template <int NPT, int PRIO, int DOM, bool LAB>
hipError_t exact_one(const ExactArgs &a, int block, bool coop, hipStream_t s) {
    auto fn = k_exact<NPT, PRIO, DOM, LAB>;
    if (coop && a.G > 1) {
        ExactArgs copy = a;
        void *args[] = {&copy};
        return hipLaunchCooperativeKernel((const void *)fn, dim3(a.G), dim3(block), args, 0, s);
    }
    hipLaunchKernelGGL(fn, dim3(a.G), dim3(block), 0, s, a);
    return hipGetLastError();
}

template <int PRIO, int DOM, bool LAB>
hipError_t exact_npt(int npt, const ExactArgs &a, int block, bool coop, hipStream_t s) {
    switch (npt) {
        case 1: return exact_one<1, PRIO, DOM, LAB>(a, block, coop, s);
        case 2: return exact_one<2, PRIO, DOM, LAB>(a, block, coop, s);
        case 4: return exact_one<4, PRIO, DOM, LAB>(a, block, coop, s);
        case 8: return exact_one<8, PRIO, DOM, LAB>(a, block, coop, s);
        case 16: return exact_one<16, PRIO, DOM, LAB>(a, block, coop, s);
        default: return hipErrorInvalidValue;
    }
}

template <int K, int PRIO, int DOM, bool LAB>
hipError_t score_one(const ScoreArgs &a, int pod_groups, hipStream_t s) {
    dim3 grid((a.n_chunks + 3) / 4, pod_groups);
    hipLaunchKernelGGL((k_score_topk<K, PRIO, DOM, LAB>), grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

template <int PRIO, int DOM, bool LAB>
hipError_t score_k(int K, const ScoreArgs &a, int pg, hipStream_t s) {
    switch (K) {
        case 4: return score_one<4, PRIO, DOM, LAB>(a, pg, s);
        case 8: return score_one<8, PRIO, DOM, LAB>(a, pg, s);
        case 16: return score_one<16, PRIO, DOM, LAB>(a, pg, s);
        default: return hipErrorInvalidValue;
    }
}

template <int K>
hipError_t merge_k(bool rec, bool fin, const MergeArgs &a, hipStream_t s) {
    dim3 grid(a.C_out, a.B);
    if (rec) {
        if (!fin) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_merge<K, true, true>), grid, dim3(64), 0, s, a);
    } else if (fin) {
        hipLaunchKernelGGL((k_merge<K, false, true>), grid, dim3(64), 0, s, a);
    } else {
        hipLaunchKernelGGL((k_merge<K, false, false>), grid, dim3(64), 0, s, a);
    }
    return hipGetLastError();
}

template <int K, int PRIO, int DOM, bool LAB>
hipError_t commit_one(const CommitArgs &a, size_t lds, bool single_wave, hipStream_t s) {
    static bool attr_set[2] = {false, false};
    const void *fn = single_wave ? (const void *)k_commit1<K, PRIO, DOM, LAB> : (const void *)k_commit<K, PRIO, DOM, LAB>;
    if (!attr_set[single_wave]) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 4096);
        if (e != hipSuccess) return e;
        attr_set[single_wave] = true;
    }
    if (single_wave) hipLaunchKernelGGL((k_commit1<K, PRIO, DOM, LAB>), dim3(1), dim3(64), lds, s, a);
    else hipLaunchKernelGGL((k_commit<K, PRIO, DOM, LAB>), dim3(1), dim3(kCommitBlock), lds, s, a);
    return hipGetLastError();
}

template <int PRIO, int DOM, bool LAB>
hipError_t commit_k(int K, const CommitArgs &a, size_t lds, bool sw, hipStream_t s) {
    switch (K) {
        case 4: return commit_one<4, PRIO, DOM, LAB>(a, lds, sw, s);
        case 8: return commit_one<8, PRIO, DOM, LAB>(a, lds, sw, s);
        case 16: return commit_one<16, PRIO, DOM, LAB>(a, lds, sw, s);
        default: return hipErrorInvalidValue;
    }
}

// (priority, domain, labels) -> instantiation.  Best-price always ranges over feasible nodes.
#define KSCHED_DISPATCH(prio, dom, lab, CALL)                                   \
    do {                                                                        \
        if ((prio) == kPrioPrice) {                                             \
            if (lab) { constexpr int P_ = kPrioPrice, D_ = kDomFeasible; constexpr bool L_ = true; return CALL; } \
            else { constexpr int P_ = kPrioPrice, D_ = kDomFeasible; constexpr bool L_ = false; return CALL; }    \
        } else if ((dom) == kDomFeasible) {                                     \
            if (lab) { constexpr int P_ = kPrioResource, D_ = kDomFeasible; constexpr bool L_ = true; return CALL; } \
            else { constexpr int P_ = kPrioResource, D_ = kDomFeasible; constexpr bool L_ = false; return CALL; }    \
        } else {                                                                \
            if (lab) { constexpr int P_ = kPrioResource, D_ = kDomAll; constexpr bool L_ = true; return CALL; }      \
            else { constexpr int P_ = kPrioResource, D_ = kDomAll; constexpr bool L_ = false; return CALL; }         \
        }                                                                       \
    } while (0)

}  // namespace

hipError_t launch_exact(int npt, int prio, int dom, bool lab, const ExactArgs &a, int block, bool coop,
                        hipStream_t s) {
    KSCHED_DISPATCH(prio, dom, lab, (exact_npt<P_, D_, L_>(npt, a, block, coop, s)));
}

hipError_t launch_score_topk(int K, int prio, int dom, bool lab, const ScoreArgs &a, int pod_groups, hipStream_t s) {
    KSCHED_DISPATCH(prio, dom, lab, (score_k<P_, D_, L_>(K, a, pod_groups, s)));
}

hipError_t launch_merge(int K, bool input_rec, bool final_stage, const MergeArgs &a, hipStream_t s) {
    switch (K) {
        case 4: return merge_k<4>(input_rec, final_stage, a, s);
        case 8: return merge_k<8>(input_rec, final_stage, a, s);
        case 16: return merge_k<16>(input_rec, final_stage, a, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_commit(int K, int prio, int dom, bool lab, const CommitArgs &a, size_t lds_bytes, bool single_wave,
                         hipStream_t s) {
    KSCHED_DISPATCH(prio, dom, lab, (commit_k<P_, D_, L_>(K, a, lds_bytes, single_wave, s)));
}

hipError_t launch_apply_delta(NodeRec *nodes, int64_t n, int64_t k, const int32_t *idx, const int64_t *d,
                              hipStream_t s) {
    hipLaunchKernelGGL(k_apply_delta, dim3(1), dim3(64), 0, s, nodes, n, k, idx, d);
    return hipGetLastError();
}

}  // namespace ksched
