// ksched_kernels.hip -- CDNA4 (gfx950) kernels of the scheduling core.  Compiled with
// -ffp-contract=off: every double op rounds individually, exactly like the Go reference.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "ksched_kernels.h"
#include "ksched_merge.h"

namespace ksched {

namespace {

__device__ __forceinline__ uint64_t ld_granule(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_granule(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void set_node(NodeRec *nd, int64_t a0, int64_t a1, int64_t a2) {
    nd->a[0] = a0; nd->a[1] = a1; nd->a[2] = a2;
    const double f0 = (double)a0, f1 = (double)a1, f2 = (double)a2;
    nd->af[0] = f0; nd->af[1] = f1; nd->af[2] = f2;
    nd->y[0] = recip_or_zero(a0, f0); nd->y[1] = recip_or_zero(a1, f1); nd->y[2] = recip_or_zero(a2, f2);
}

}  // namespace

// (re)derive af / y of every node row from its int64 allocatable
__global__ void k_prep_nodes(NodeRec *nodes, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    NodeRec *nd = nodes + i;
    set_node(nd, nd->a[0], nd->a[1], nd->a[2]);
}

// ------------------------------------------------------------------------------------------------
// Exact mode: one persistent launch schedules every pod in order.
//   - workgroup g owns nodes [g*per_wg, (g+1)*per_wg); thread t holds nodes g*per_wg + t + k*256
//     (k < NPT) in registers for the whole launch, with their (double) values and reciprocals;
//   - per pod: each lane scores its nodes (predicate.go:127-150 + priorities.go:45-50), wave
//     butterfly arg-best + count, 4-wave combine through LDS;
//   - G > 1: wave 0 publishes the workgroup's (key, idx, count) as four tagged 8-byte granules
//     (write-through sc1 stores, epoch = pod + 1) and sweeps all G records until every tag matches
//     (MI355X_MICROARCH "handoff-1to1"/"allgather" R2 granules: no fences needed); every workgroup
//     then folds the same G records into the same decision;
//   - the owner lane of the winning node commits it in registers; nodes are written back at exit.
// ------------------------------------------------------------------------------------------------
template <int NPT, int PRIO, int DOM, bool LAB, bool F53>
__global__ __launch_bounds__(kExactBlock) void k_exact(ExactArgs A) {
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int g = blockIdx.x;
    const int64_t lo = (int64_t)g * A.per_wg;
    const int64_t hi = (lo + A.per_wg < A.n) ? lo + A.per_wg : A.n;
    const double y3 = recip(3.0);

    int64_t a0[NPT], a1[NPT], a2[NPT];
    double f0[NPT], f1[NPT], f2[NPT], y0[NPT], y1[NPT], y2[NPT];
    uint64_t lab[NPT];
    float pr[NPT];
    int32_t id[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        const int64_t j = lo + tid + (int64_t)k * kExactBlock;
        if (j < hi) {
            const NodeRec &nd = A.nodes[j];
            a0[k] = nd.a[0]; a1[k] = nd.a[1]; a2[k] = nd.a[2];
            f0[k] = nd.af[0]; f1[k] = nd.af[1]; f2[k] = nd.af[2];
            y0[k] = nd.y[0]; y1[k] = nd.y[1]; y2[k] = nd.y[2];
            lab[k] = nd.labels; pr[k] = nd.price; id[k] = (int32_t)j;
        } else {
            a0[k] = a1[k] = a2[k] = 0; f0[k] = f1[k] = f2[k] = 0.0; y0[k] = y1[k] = y2[k] = 0.0;
            lab[k] = 0; pr[k] = 0.f; id[k] = kNoIdx;
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
                if (pair_key_fast<PRIO, DOM, F53>(f, rc, rm, rp, rcf, rmf, rpf, a0[k], a1[k], a2[k], f0[k], f1[k],
                                                  f2[k], y0[k], y1[k], y2[k], y3, pr[k], &key) &&
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
            osc = PRIO == kPrioPrice ? 0.0 - gk : gk;
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                if (id[k] == gi) {  // commit: used += request, ONE pod (anchor/predicate.go:99-102)
                    a0[k] = wsub(a0[k], rc); a1[k] = wsub(a1[k], rm); a2[k] = wsub(a2[k], 1);
                    f0[k] = (double)a0[k]; f1[k] = (double)a1[k]; f2[k] = (double)a2[k];
                    y0[k] = recip_or_zero(a0[k], f0[k]); y1[k] = recip_or_zero(a1[k], f1[k]);
                    y2[k] = recip_or_zero(a2[k], f2[k]);
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
    for (int k = 0; k < NPT; ++k)
        if (id[k] != kNoIdx) set_node(A.nodes + id[k], a0[k], a1[k], a2[k]);
}

// ------------------------------------------------------------------------------------------------
// Exact mode on ONE workgroup (kExact1Block threads; n <= kExact1Block * NPT): every node lives in a register
// slot of this workgroup, so a pod is decided with one workgroup barrier and no cross-workgroup exchange (k_exact
// with G > 1 pays a round of tagged granules through L2 per pod, ~2.7 us on c2).  Thread t holds slots
// s = t + k * kExact1Block.
//   best-price: slot s is the node of rank s in (price asc, node index asc) -- the order of the reference's
//     argmax over -price with the lowest index on ties (README.md:37-64; price_key) -- so a pod's node is the
//     FIRST feasible slot: per wave one ballot per k (its lowest set bit), the minimum over the waves; the feasible
//     count is the sum of the ballots' popcounts.  No key is compared at all.
//   resource: slot s is node s; per pod every lane keys its slots, wave arg-best, the waves' bests through LDS.
// Restated by the same oracle as k_exact (oracle/cpu_ref.c or_schedule); results bit-identical.
// ------------------------------------------------------------------------------------------------
template <int NPT, int BS, int PRIO, int DOM, bool LAB, bool F53>
__global__ __launch_bounds__(BS) void k_exact1(ExactArgs A) {
    constexpr int kExact1Block = BS;
    constexpr int W = kExact1Block / 64;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const double y3 = recip(3.0);
    constexpr bool kRes = PRIO != kPrioPrice;
    int64_t a0[NPT], a1[NPT], a2[NPT];
    double f0[kRes ? NPT : 1], f1[kRes ? NPT : 1], f2[kRes ? NPT : 1];
    double yy0[kRes ? NPT : 1], yy1[kRes ? NPT : 1], yy2[kRes ? NPT : 1];
    uint64_t lab[NPT];
    float pr[NPT];
    int32_t id[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        const int64_t sl = tid + (int64_t)k * kExact1Block;
        id[k] = kNoIdx;
        a0[k] = a1[k] = a2[k] = 0; lab[k] = 0; pr[k] = 0.f;
        if constexpr (kRes) { f0[k] = f1[k] = f2[k] = 0.0; yy0[k] = yy1[k] = yy2[k] = 0.0; }
        if (sl < A.n) {
            const int32_t j = A.perm ? A.perm[sl] : (int32_t)sl;
            const NodeRec &nd = A.nodes[j];
            a0[k] = nd.a[0]; a1[k] = nd.a[1]; a2[k] = nd.a[2];
            lab[k] = nd.labels; pr[k] = nd.price; id[k] = j;
            if constexpr (kRes) {
                f0[k] = nd.af[0]; f1[k] = nd.af[1]; f2[k] = nd.af[2];
                yy0[k] = nd.y[0]; yy1[k] = nd.y[1]; yy2[k] = nd.y[2];
            }
        }
    }
    __shared__ int32_t s_cnt[2][W];
    __shared__ int32_t s_slot[2][W];  // best-price: the wave's first feasible slot (INT32_MAX: none)
    __shared__ double s_key[2][W];    // resource: the wave's best (key, node)
    __shared__ int32_t s_idx[2][W];
    // the next pod's request is loaded one pod ahead: its latency hides behind the current pod
    int64_t nrc = 0, nrm = 0, nrp = 0;
    uint64_t nsel = 0;
    if (A.pods.p > 0) { nrc = A.pods.rc[0]; nrm = A.pods.rm[0]; nrp = A.pods.rp[0]; nsel = LAB ? A.pods.sel[0] : 0; }
    for (int64_t i = 0; i < A.pods.p; ++i) {
        const int par = (int)(i & 1);
        const int64_t rc = nrc, rm = nrm, rp = nrp;
        const uint64_t sel = nsel;
        if (i + 1 < A.pods.p) {
            nrc = A.pods.rc[i + 1]; nrm = A.pods.rm[i + 1]; nrp = A.pods.rp[i + 1];
            nsel = LAB ? A.pods.sel[i + 1] : 0;
        }
        int32_t cnt = 0;
        int32_t oidx = -1;
        double osc = 0.0;
        if constexpr (!kRes) {
            int32_t first = 0x7fffffff;
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                const bool f = id[k] != kNoIdx && fits(rc, rm, rp, sel, a0[k], a1[k], a2[k], lab[k], LAB);
                const uint64_t m = __ballot(f);
                cnt += __popcll(m);
                if (first == 0x7fffffff && m) first = k * kExact1Block + wave * 64 + (int)__builtin_ctzll(m);
            }
            if (lane == 0) { s_slot[par][wave] = first; s_cnt[par][wave] = cnt; }
            __syncthreads();
            int32_t gs = s_slot[par][0], gc = s_cnt[par][0];
#pragma unroll
            for (int w = 1; w < W; ++w) { gs = s_slot[par][w] < gs ? s_slot[par][w] : gs; gc += s_cnt[par][w]; }
            // the first feasible slot's owner commits it and writes the pod's results; no feasible node: thread 0
            if (gc == 0) {
                if (tid == 0) { A.out.idx[i] = -1; A.out.score[i] = 0.0; A.out.feas[i] = 0; }  // NO_FIT
            } else if ((gs & (kExact1Block - 1)) == tid) {
#pragma unroll
                for (int k = 0; k < NPT; ++k) {
                    if (gs == k * kExact1Block + tid) {  // commit: used += request, ONE pod (anchor/predicate.go:99-102)
                        A.out.idx[i] = id[k];
                        A.out.score[i] = 0.0 - price_key(pr[k]);
                        A.out.feas[i] = gc;
                        a0[k] = wsub(a0[k], rc); a1[k] = wsub(a1[k], rm); a2[k] = wsub(a2[k], 1);
                    }
                }
            }
            (void)oidx; (void)osc;
        } else {
            const double rcf = (double)rc, rmf = (double)rm, rpf = (double)rp;
            double bk = -__builtin_inf();
            int32_t bi = kNoIdx;
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                if (id[k] != kNoIdx) {
                    const bool f = fits(rc, rm, rp, sel, a0[k], a1[k], a2[k], lab[k], LAB);
                    cnt += f;
                    double key;
                    if (pair_key_fast<PRIO, DOM, F53>(f, rc, rm, rp, rcf, rmf, rpf, a0[k], a1[k], a2[k], f0[k], f1[k],
                                                      f2[k], yy0[k], yy1[k], yy2[k], y3, pr[k], &key) &&
                        better(key, id[k], bk, bi)) {
                        bk = key;
                        bi = id[k];
                    }
                }
            }
            int32_t aux = 0;
            wave_argbest(bk, bi, aux);
            cnt = (int32_t)wave_sum_i64(cnt);
            if (lane == 0) { s_key[par][wave] = bk; s_idx[par][wave] = bi; s_cnt[par][wave] = cnt; }
            __syncthreads();
            double gk = s_key[par][0];
            int32_t gi = s_idx[par][0], gc = s_cnt[par][0];
#pragma unroll
            for (int w = 1; w < W; ++w) {
                gc += s_cnt[par][w];
                if (better(s_key[par][w], s_idx[par][w], gk, gi)) { gk = s_key[par][w]; gi = s_idx[par][w]; }
            }
            oidx = gc == 0 ? -1 : (gi == kNoIdx ? -2 : gi);  // NO_FIT / NO_POSITIVE_SCORE (anchor/schedule.go:74-76)
            osc = oidx >= 0 ? gk : 0.0;
            if (oidx >= 0) {
#pragma unroll
                for (int k = 0; k < NPT; ++k) {
                    if (id[k] == gi) {
                        a0[k] = wsub(a0[k], rc); a1[k] = wsub(a1[k], rm); a2[k] = wsub(a2[k], 1);
                        f0[k] = (double)a0[k]; f1[k] = (double)a1[k]; f2[k] = (double)a2[k];
                        yy0[k] = recip_or_zero(a0[k], f0[k]); yy1[k] = recip_or_zero(a1[k], f1[k]);
                        yy2[k] = recip_or_zero(a2[k], f2[k]);
                    }
                }
            }
            if (tid == 0) { A.out.idx[i] = oidx; A.out.score[i] = osc; A.out.feas[i] = gc; }
        }
    }
#pragma unroll
    for (int k = 0; k < NPT; ++k)
        if (id[k] != kNoIdx) set_node(A.nodes + id[k], a0[k], a1[k], a2[k]);
}

// ------------------------------------------------------------------------------------------------
// Batched mode, stage 1: fused predicate + score + top-KC per (pod, workgroup).  Lane = pod of the
// batch.  A workgroup is kScoreWaves waves; wave w of workgroup g scans sub-chunk s = g + G*w of the
// NSC = G*kScoreWaves sub-chunks, i.e. the nodes j with j mod NSC == s: workgroup g holds the nodes
// j = g (mod G), so the lowest-index members of a tie class land in different workgroups and short
// lists still merge into a long exact prefix.  Node rows are wave-uniform (scalar loads of the 96-B
// NodeRec, reciprocals included).
//   Each wave keeps a sorted top-KC per lane (branch-free register insert; nodes arrive in ascending
//   index, so a strict key compare keeps ties in index order).  The wave lists fold pairwise through
//   LDS into one list per (pod, workgroup): two lists that are each cut when full fold into the top-KC
//   of their union, again cut when full.
// ------------------------------------------------------------------------------------------------
template <int KC, int PRIO, int DOM, bool LAB, bool F53>
__device__ __forceinline__ void score_topk_body(const ScoreArgs &A) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double *s_key = reinterpret_cast<double *>(smem);                                   // [W/2][KC][64]
    int32_t *s_idx = reinterpret_cast<int32_t *>(smem + (size_t)(kScoreWaves / 2) * KC * 64 * 8);
    int32_t *s_cnt = s_idx + (size_t)(kScoreWaves / 2) * KC * 64;                        // [64]
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t G = gridDim.x;
    const int64_t NSC = G * kScoreWaves;
    const int64_t sub = (int64_t)blockIdx.x + G * wave;
    if (A.wait_committed) {
        // commit(b-2) published its plan for this batch, its commits (XBuf) and Ctl::committed with an
        // agent release: one lane polls (relaxed, s_sleep), one agent acquire, then plain loads
        __shared__ int s_late;
        if (threadIdx.x == 0) {
            const uint64_t t0 = wall_clock64();
            s_late = 0;
            while (__hip_atomic_load(A.wait_committed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < A.wait_target) {
                __builtin_amdgcn_s_sleep(1);
                if (wall_clock64() - t0 > 200000000ull) {  // 2 s: report instead of spinning forever
                    __hip_atomic_store(A.err, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    s_late = 1;
                    break;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        if (s_late) return;
    }
    // Batch b-2's commits (<= 128 nodes, two per lane): the wave whose sub-chunk holds a node writes it
    // back to the row (for the next launches) and overlays it on what it reads in this launch, so no
    // separate apply kernel has to run between commit(b-2) and score(b).
    int64_t pj0 = -1, pj1 = -1;  // local node index of entries lane and lane + 64, if in this sub-chunk
    {
        const int np = A.patch->count;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int e = h * 64 + lane;
            const int64_t j = e < np ? (int64_t)A.patch->e[e].idx - A.node_offset : -1;
            const bool mine = j >= 0 && j < A.n_local && (j % NSC) == sub;
            if (mine && blockIdx.y == 0) {
                const XRec &x = A.patch->e[e];
                set_node(A.nodes + j, x.cur[0], x.cur[1], x.cur[2]);
            }
            if (h == 0) pj0 = mine ? j : -1;
            else pj1 = mine ? j : -1;
        }
    }
    const bool anyp = __ballot(pj0 >= 0 || pj1 >= 0) != 0;
    if (threadIdx.x < 64) s_cnt[threadIdx.x] = 0;
    const int64_t p0 = *A.cursor;
    if (p0 < 0 || p0 >= A.pods.p) return;  // workgroup-uniform
    __syncthreads();
    const int b = blockIdx.y * 64 + lane;
    const int64_t pod = p0 + b;
    const bool active = (b < A.B) && (pod < A.pods.p);
    const int64_t rc = active ? A.pods.rc[pod] : 0;
    const int64_t rm = active ? A.pods.rm[pod] : 0;
    const int64_t rp = active ? A.pods.rp[pod] : 0;
    const uint64_t sel = (LAB && active) ? A.pods.sel[pod] : 0;
    const double rcf = (double)rc, rmf = (double)rm, rpf = (double)rp;
    const double y3 = recip(3.0);

    double key[KC];
    int32_t idx[KC];
#pragma unroll
    for (int q = 0; q < KC; ++q) { key[q] = -__builtin_inf(); idx[q] = kNoIdx; }
    int32_t cnt = 0;
    // one node against this lane's pod: predicate, key, sorted insert (strict '>': nodes arrive in
    // ascending index, so equal keys keep index order)
    auto visit = [&](int64_t j, int64_t ac, int64_t am, int64_t ap, double af0, double af1, double af2, double y0,
                     double y1, double y2, uint64_t lab, float price) {
        const bool f = fits(rc, rm, rp, sel, ac, am, ap, lab, LAB);
        cnt += f;
        double k;
        const bool el = pair_key_fast<PRIO, DOM, F53>(f, rc, rm, rp, rcf, rmf, rpf, ac, am, ap, af0, af1, af2, y0, y1,
                                                      y2, y3, price, &k);
        double ck = el ? k : -__builtin_inf();
        int32_t ci = (int32_t)(A.node_offset + j);
        bool moved = false;  // once placed, every later entry shifts down one slot
#pragma unroll
        for (int q = 0; q < KC; ++q) {
            const bool sw = moved || ck > key[q];
            moved = sw;
            const double tk = key[q];
            const int32_t ti = idx[q];
            key[q] = sw ? ck : tk; idx[q] = sw ? ci : ti;
            ck = sw ? tk : ck; ci = sw ? ti : ci;
        }
    };
    if (!anyp) {
        // Node rows are wave-uniform: read through the constant address space they arrive as scalar
        // loads (s_load_dwordx16 + x8) into SGPRs, one row ahead of its use -- row j + NSC is in flight
        // while row j is scored -- and feed the VALU as scalar operands (no row VGPRs).
        const NodeRecC *rows = (const NodeRecC *)(A.nodes);
        NodeRec nxt;
        if (sub < A.n_local) nxt = load_row(rows + sub);
        for (int64_t j = sub; j < A.n_local; j += NSC) {
            const NodeRec nd = nxt;
            const int64_t jn = j + NSC;
            if (jn < A.n_local) nxt = load_row(rows + jn);
            visit(j, nd.a[0], nd.a[1], nd.a[2], nd.af[0], nd.af[1], nd.af[2], nd.y[0], nd.y[1], nd.y[2], nd.labels,
                  nd.price);
        }
    } else {
        // this sub-chunk holds nodes committed by batch b-2 (~6 % of the waves at B = 64): their rows
        // are overlaid from the XBuf as they are reached (the write-back above may not be visible yet
        // to this launch's reads, and is not done at all by pod groups y > 0)
        for (int64_t j = sub; j < A.n_local; j += NSC) {
            const NodeRec &nd = A.nodes[j];
            int64_t ac = nd.a[0], am = nd.a[1], ap = nd.a[2];
            double af0 = nd.af[0], af1 = nd.af[1], af2 = nd.af[2], y0 = nd.y[0], y1 = nd.y[1], y2 = nd.y[2];
            const uint64_t hit = __ballot(pj0 == j || pj1 == j);
            if (hit) {
                const int src = __ffsll((unsigned long long)hit) - 1;
                const int e = __builtin_amdgcn_readlane(pj0 == j ? lane : lane + 64, src);
                const XRec &xr = A.patch->e[e];
                ac = xr.cur[0]; am = xr.cur[1]; ap = xr.cur[2];
                af0 = (double)ac; af1 = (double)am; af2 = (double)ap;
                y0 = recip_or_zero(ac, af0); y1 = recip_or_zero(am, af1); y2 = recip_or_zero(ap, af2);
            }
            visit(j, ac, am, ap, af0, af1, af2, y0, y1, y2, nd.labels, nd.price);
        }
    }
    if (cnt) atomicAdd(&s_cnt[lane], cnt);
    // fold the wave lists pairwise: W -> W/2 -> ... -> 1
#pragma unroll
    for (int half = kScoreWaves / 2; half >= 1; half >>= 1) {
        if (wave >= half && wave < 2 * half) {
#pragma unroll
            for (int q = 0; q < KC; ++q) {
                s_key[((wave - half) * KC + q) * 64 + lane] = key[q];
                s_idx[((wave - half) * KC + q) * 64 + lane] = idx[q];
            }
        }
        __syncthreads();
        if (wave < half) {
#pragma unroll
            for (int q = 0; q < KC; ++q) {
                const int32_t oi = s_idx[(wave * KC + q) * 64 + lane];
                if (oi == kNoIdx) break;
                list_insert_ordered<KC>(key, idx, s_key[(wave * KC + q) * 64 + lane], oi);
            }
        }
        __syncthreads();
    }
    if (wave == 0 && active) {
        Cand *dst = A.part + ((size_t)b * G + blockIdx.x) * KC;
#pragma unroll
        for (int q = 0; q < KC; ++q) { dst[q].key = key[q]; dst[q].idx = idx[q]; dst[q].pad = 0; }
        A.part_cnt[(size_t)b * G + blockIdx.x] = s_cnt[lane];
    }
}

template <int KC, int K>
__global__ __launch_bounds__(kMergeThreads) void k_merge_pod(MergeArgs A) {
    __shared__ MergeSmem<KC, K, kMergeThreads> sm;
    merge_pod_body<KC, K, false, kMergeThreads>(A, blockIdx.x, threadIdx.x, sm, BlockSync{});
}

// Score kernel (the merge waits on a stream event).
// <= 64 VGPRs (launch bound: 8 waves per SIMD): two score waves + two commit waves (190 VGPRs) must
// fit one SIMD, or the single-workgroup commit cannot dispatch beside the score grid.
template <int KC, int PRIO, int DOM, bool LAB, bool F53>
__global__ __launch_bounds__(kScoreThreads, 8) void k_score_topk(ScoreArgs A) {
    score_topk_body<KC, PRIO, DOM, LAB, F53>(A);
}

// ------------------------------------------------------------------------------------------------
// Merge: one wave per (pod, group of <= 64 sorted lists of KIN entries).  Each lane stages one list in
// LDS; K rounds of wave arg-best over the lanes' heads (the winning lane advances).  Final stage writes
// Rec entries carrying the node snapshot state; INPUT_REC merges the ranks' Rec lists.
// Exact prefix ("cut") rule: a cut input list has unlisted candidates, all ranking below its last
// entry.  The output keeps only entries ranking at or above the best such cutoff (anything below it
// could be preceded by an unlisted candidate) and is itself cut when any input was, or when entries
// were left over after K rounds.  The flag travels in entry 0's pad (Cand) / pad (Rec).
// ------------------------------------------------------------------------------------------------
template <int KIN, int K, bool INPUT_REC, bool FINAL>
__global__ __launch_bounds__(64) void k_merge(MergeArgs A) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical: win issue arbitration over co-resident score waves
    __shared__ double s_key[64 * KIN];
    __shared__ int32_t s_idx[64 * KIN];
    const int lane = threadIdx.x;
    const int grp = blockIdx.x;
    const int b = blockIdx.y;
    const int64_t p0 = *A.cursor;
    if (p0 < 0 || p0 >= A.P || b >= A.B || p0 + b >= A.P) return;
    const int list = grp * 64 + lane;
    const bool has = list < A.C_in;
    int64_t cnt = 0;
    int n = 0;          // valid entries of this lane's list
    bool cut = false;   // this lane's list is cut
    if (has) {
        if (INPUT_REC) {
            const char *blk = static_cast<const char *>(A.in) + (size_t)list * A.rank_stride;
            const Rec *src = reinterpret_cast<const Rec *>(blk) + (size_t)b * KIN;
#pragma unroll
            for (int q = 0; q < KIN; ++q) {
                const bool v = src[q].valid != 0;
                s_key[lane * KIN + q] = v ? src[q].key : -__builtin_inf();
                s_idx[lane * KIN + q] = v ? src[q].idx : kNoIdx;
                n += v;
            }
            cut = src[0].pad != 0;
            cnt = reinterpret_cast<const int64_t *>(blk + (size_t)A.B * KIN * sizeof(Rec))[b];
        } else {
            const Cand *src = static_cast<const Cand *>(A.in) + ((size_t)b * A.C_in + list) * KIN;
#pragma unroll
            for (int q = 0; q < KIN; ++q) {
                s_key[lane * KIN + q] = src[q].key;
                s_idx[lane * KIN + q] = src[q].idx;
                n += src[q].idx != kNoIdx;
            }
            // chunk lists (first stage): cut when full; merged lists carry the flag
            cut = A.chunk_input ? (n == KIN) : (src[0].pad != 0);
            cnt = A.in_cnt[(size_t)b * A.C_in + list];
        }
    }
    cnt = wave_sum_i64(cnt);
    // best cutoff over the cut lists (their last valid entry)
    double ck = (cut && n > 0) ? s_key[lane * KIN + n - 1] : -__builtin_inf();
    int32_t ci = (cut && n > 0) ? s_idx[lane * KIN + n - 1] : kNoIdx;
    const bool anycut = __ballot(cut) != 0;
    {
        int32_t aux = 0;
        wave_argbest(ck, ci, aux);
    }
    __syncthreads();
    int h = 0;
    double mk = -__builtin_inf();
    int32_t mi = kNoIdx, msrc = -1;
    for (int r = 0; r < K; ++r) {
        double k = (h < n) ? s_key[lane * KIN + h] : -__builtin_inf();
        int32_t ix = (h < n) ? s_idx[lane * KIN + h] : kNoIdx;
        int32_t src = lane * KIN + h;
        wave_argbest(k, ix, src);
        if (ix == kNoIdx) break;  // wave-uniform
        if (src == lane * KIN + h) ++h;
        if (lane == r) { mk = k; mi = ix; msrc = src; }
    }
    const bool left = __ballot(h < n) != 0;  // candidates beyond the K output entries
    // entries ranking below the best cutoff are not exact
    if (anycut && mi != kNoIdx && better(ck, ci, mk, mi)) { mk = -__builtin_inf(); mi = kNoIdx; }
    const int32_t cut_out = (anycut || left) ? 1 : 0;
    if (!FINAL) {
        if (lane < K) {
            Cand *dst = A.out + ((size_t)b * A.C_out + grp) * K + lane;
            dst->key = mk; dst->idx = mi; dst->pad = lane == 0 ? cut_out : 0;
        }
        if (lane == 0) A.out_cnt[(size_t)b * A.C_out + grp] = cnt;
    } else {
        if (lane < K) {
            Rec r{};
            if (mi != kNoIdx) {
                if (INPUT_REC) {
                    const int srcl = msrc / KIN, srcq = msrc % KIN;
                    const char *blk = static_cast<const char *>(A.in) + (size_t)(grp * 64 + srcl) * A.rank_stride;
                    r = reinterpret_cast<const Rec *>(blk)[(size_t)b * KIN + srcq];
                } else {
                    const NodeRec &nd = A.nodes[mi - A.node_offset];
                    r.key = mk; r.idx = mi; r.valid = 1;
                    r.a[0] = nd.a[0]; r.a[1] = nd.a[1]; r.a[2] = nd.a[2];
                    r.labels = nd.labels; r.price = nd.price;
                }
            } else {
                r.key = -__builtin_inf(); r.idx = kNoIdx; r.valid = 0;
            }
            r.pad = lane == 0 ? cut_out : 0;
            A.out_rec[(size_t)b * K + lane] = r;
        }
        if (lane == 0) A.out_fc[b] = cnt;
    }
}

// ------------------------------------------------------------------------------------------------
// Ordered commit of one batch: a single-wave sequencer.  For pod i of the batch, with T = nodes
// committed by pods < i of this batch (LDS table; s0 = snapshot state, cur = current state):
//   fc   = fc0[i] - sum_T fits(s0) + sum_T fits(cur)                          (predicate count)
//   t*   = best of T re-scored at cur;  u* = first list entry not in T (exact: untouched)
//   list full and all touched: t* must beat list[K-1] (every unlisted untouched node ranks below
//   it), otherwise the batch stops before pod i (overflow) and the next batch restarts there.
// One wave, no barriers: reductions are register butterflies (DPP + permlane swaps) and ballots;
// every lane evaluates the (wave-uniform) decision; requests and feasible counts are staged into LDS
// once; lane q < K holds candidate q of the current pod while the next pod's candidates load into
// the other register buffer (the loop is unrolled by two so the wait lands one pod later).
// ------------------------------------------------------------------------------------------------
constexpr int kMaxTouchedSlots = 4;  // touched nodes per lane -> 256 (previous batch's + this batch's, B <= 128)

struct CommitCtx {
    int32_t *hkey;       // open-addressing set of touched node indices (kTouchHash slots, -1 = empty)
    uint32_t *filt;      // 64K-bit filter: bit (idx & 0xffff) set once idx is touched
    Touched *T;
    const PodStage *PS;
    const CandStage *CS; // [B][K] staged candidate lists
    int nT;
    int64_t placed;
    double y3;
    int lane;
    int64_t p0;
};

__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

__device__ __forceinline__ uint32_t thash(int32_t idx) { return ((uint32_t)idx * 2654435761u) >> (32 - kTouchHashBits); }

__device__ __forceinline__ bool touched_has(const CommitCtx &cx, int32_t idx) {
    if (!(cx.filt[((uint32_t)idx & 0xffffu) >> 5] & (1u << ((uint32_t)idx & 31)))) return false;
    for (uint32_t h = thash(idx);; h = (h + 1) & (kTouchHash - 1)) {
        const int32_t k = cx.hkey[h];
        if (k == idx) return true;
        if (k < 0) return false;
    }
}

__device__ __forceinline__ void touched_insert(CommitCtx &cx, int32_t idx) {
    uint32_t h = thash(idx);
    while (cx.hkey[h] >= 0) h = (h + 1) & (kTouchHash - 1);
    cx.hkey[h] = idx;
    cx.filt[((uint32_t)idx & 0xffffu) >> 5] |= 1u << ((uint32_t)idx & 31);
}

// Touched-node re-scoring, filtered: an upper bound (reciprocal multiplies, no corrections) per slot
// decides which touched nodes could beat the threshold (thk, thi); only those are scored exactly.
// Non-candidates provably rank below the threshold, so the decision is unchanged.
// Feasibility deltas (exact integer compares) come through ballots.
template <int NS, int PRIO, int DOM, bool LAB, bool F53>
__device__ __forceinline__ void rescore_touched(const CommitCtx &cx, int64_t rc, int64_t rm, int64_t rp, uint64_t sel,
                                                double rcf, double rmf, double rpf, double thk, int32_t thi,
                                                int64_t &df, double &tk, int32_t &ti, int32_t &ts, bool &any) {
    bool cand[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int t = cx.lane + 64 * s;
        const bool in = t < cx.nT;
        const Touched &x = cx.T[in ? t : 0];
        const bool f0 = in && fits(rc, rm, rp, sel, x.s0[0], x.s0[1], x.s0[2], x.labels, LAB);
        const bool f1 = in && fits(rc, rm, rp, sel, x.cur[0], x.cur[1], x.cur[2], x.labels, LAB);
        df += (int64_t)__popcll(__ballot(f1)) - (int64_t)__popcll(__ballot(f0));
        bool c;
        if (PRIO == kPrioPrice) {
            c = f1 && better(price_key(x.price), x.idx, thk, thi);
        } else {
            bool near1;
            const double hi = resource_score_upper<F53>(rc, rm, rp, rcf, rmf, rpf, x.cur[0], x.cur[1], x.cur[2],
                                                        x.curf[0], x.curf[1], x.curf[2], x.cury[0], x.cury[1],
                                                        x.cury[2], cx.y3, &near1);
            c = in && (DOM == kDomAll || f1) && (near1 || (hi > 0.0 && hi >= thk));
        }
        cand[s] = c;
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        if (__ballot(cand[s]) == 0) continue;  // wave-uniform: nothing to score exactly in this slot
        any = true;
        if (cand[s]) {
            const int t = cx.lane + 64 * s;
            const Touched &x = cx.T[t];
            const bool f1 = fits(rc, rm, rp, sel, x.cur[0], x.cur[1], x.cur[2], x.labels, LAB);
            double k;
            if (pair_key_fast<PRIO, DOM, F53>(f1, rc, rm, rp, rcf, rmf, rpf, x.cur[0], x.cur[1], x.cur[2], x.curf[0],
                                              x.curf[1], x.curf[2], x.cury[0], x.cury[1], x.cury[2], cx.y3, x.price,
                                              &k) &&
                better(k, x.idx, tk, ti)) {
                tk = k; ti = x.idx; ts = t;
            }
        }
    }
}

template <int K, int PRIO, int DOM, bool LAB, bool F53, bool ST>
__device__ __forceinline__ bool commit_step(const CommitArgs &A, CommitCtx &cx, int i, const PodStage &ps,
                                            const CandStage &my, uint64_t *ph) {
    const int lane = cx.lane;
    uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
    if (ST) t0 = stamp();
    const int64_t rc = ps.rc, rm = ps.rm, rp = ps.rp;
    const uint64_t sel = ps.sel;
    const double rcf = (double)rc, rmf = (double)rm, rpf = (double)rp;
    // candidate list: valid prefix, first entry not committed in this batch
    const bool valid = lane < K && my.idx != kNoIdx;
    const bool untouched = valid && (cx.nT == 0 || !touched_has(cx, my.idx));
    const uint64_t vmask = __ballot(valid);
    const uint64_t umask = __ballot(untouched);
    const int cv = __popcll(vmask);
    const int uq = umask ? __ffsll((unsigned long long)umask) - 1 : K;
    const bool cut = ps.cut != 0;  // unlisted candidates exist, all ranking below the last valid entry
    // threshold a touched node must beat to matter: u*, else the last valid entry (cut list), else anything
    double thk = -__builtin_inf();
    int32_t thi = kNoIdx;
    if (uq < cv) { thk = readlane_f64(my.key, uq); thi = __builtin_amdgcn_readlane(my.idx, uq); }
    else if (cut && cv > 0) { thk = readlane_f64(my.key, cv - 1); thi = __builtin_amdgcn_readlane(my.idx, cv - 1); }
    // re-score the nodes already committed (this batch's and the previous batch's)
    int64_t df = 0;
    double tk = -__builtin_inf();
    int32_t ti = kNoIdx, ts = -1;
    bool any = false;
    if (cx.nT > 0) {
        if (cx.nT <= 64)
            rescore_touched<1, PRIO, DOM, LAB, F53>(cx, rc, rm, rp, sel, rcf, rmf, rpf, thk, thi, df, tk, ti, ts, any);
        else if (cx.nT <= 128)
            rescore_touched<2, PRIO, DOM, LAB, F53>(cx, rc, rm, rp, sel, rcf, rmf, rpf, thk, thi, df, tk, ti, ts, any);
        else
            rescore_touched<kMaxTouchedSlots, PRIO, DOM, LAB, F53>(cx, rc, rm, rp, sel, rcf, rmf, rpf, thk, thi, df, tk,
                                                                   ti, ts, any);
    }
    if (ST) { asm volatile("" ::"v"(tk), "v"(ti), "v"(ts)); t1 = stamp(); }
    if (any) wave_argbest_fast(tk, ti, ts);
    if (ST) { asm volatile("" ::"v"(tk), "v"(ti), "v"(ts)); t2 = stamp(); }
    const int64_t fc = ps.fc0 + df;
    int32_t oidx = -1;
    double osc = 0.0;
    int kind = 0;  // 0 none, 1 winner from list (new touch), 2 winner already touched, 3 overflow
    double wk = 0.0;
    int32_t wi = kNoIdx;
    if (fc != 0) {
        if (uq < cv) {
            const double uk = readlane_f64(my.key, uq);
            const int32_t ui = __builtin_amdgcn_readlane(my.idx, uq);
            if (ti != kNoIdx && better(tk, ti, uk, ui)) { kind = 2; wk = tk; wi = ti; }
            else { kind = 1; wk = uk; wi = ui; }
        } else if (!cut) {
            if (ti != kNoIdx) { kind = 2; wk = tk; wi = ti; }
        } else if (cv > 0) {
            const double lk = readlane_f64(my.key, cv - 1);
            const int32_t li = __builtin_amdgcn_readlane(my.idx, cv - 1);
            if (ti != kNoIdx && better(tk, ti, lk, li)) { kind = 2; wk = tk; wi = ti; }
            else kind = 3;
        } else {
            kind = 3;  // unreachable: a cut list keeps at least its cutoff entry
        }
    }
    if (ST) t3 = stamp();
    if (kind == 3) return true;  // overflow: stop before pod i (wave-uniform)
    if (fc != 0) {
        if (kind == 0) {
            oidx = -2;
        } else {
            oidx = wi;
            osc = PRIO == kPrioPrice ? 0.0 - wk : wk;
            ++cx.placed;
            int slot = ts;
            int writer = 0;
            int64_t b0, b1, b2;
            if (kind == 1) {  // first touch: the holder of the candidate opens the slot
                slot = cx.nT++;
                writer = uq;
                b0 = my.a[0]; b1 = my.a[1]; b2 = my.a[2];
                if (lane == uq) {
                    Touched &x = cx.T[slot];
                    x.idx = my.idx; x.mine = 1;
                    x.s0[0] = b0; x.s0[1] = b1; x.s0[2] = b2;
                    x.sb[0] = b0; x.sb[1] = b1; x.sb[2] = b2;  // untouched by the previous batch
                    x.labels = my.labels; x.price = my.price; x.pad2 = 0;
                    touched_insert(cx, my.idx);
                }
            } else {
                b0 = cx.T[slot].cur[0]; b1 = cx.T[slot].cur[1]; b2 = cx.T[slot].cur[2];
            }
            if (lane == writer) {
                Touched &x = cx.T[slot];
                x.mine = 1;
                const int64_t c0 = wsub(b0, rc), c1 = wsub(b1, rm), c2 = wsub(b2, 1);
                x.cur[0] = c0; x.cur[1] = c1; x.cur[2] = c2;
                x.curf[0] = (double)c0; x.curf[1] = (double)c1; x.curf[2] = (double)c2;
                x.cury[0] = recip_or_zero(c0, x.curf[0]);
                x.cury[1] = recip_or_zero(c1, x.curf[1]);
                x.cury[2] = recip_or_zero(c2, x.curf[2]);
            }
        }
    }
    if (lane == 0) {
        const int64_t pod = cx.p0 + i;
        A.out.idx[pod] = oidx;
        A.out.score[pod] = osc;
        A.out.feas[pod] = (int32_t)fc;
    }
    if (ST) {
        const uint64_t t4 = stamp();
        ph[0] += t1 - t0; ph[1] += t2 - t1; ph[2] += t3 - t2; ph[3] += t4 - t3;
    }
    return false;
}

template <int K, int PRIO, int DOM, bool LAB, bool F53, bool ST>
__device__ __forceinline__ int commit_loop(const CommitArgs &A, CommitCtx &cx, int nb, uint64_t *ph) {
    // pod i+1's staged request and candidates are read from LDS while pod i is being decided
    PodStage ps = cx.PS[0];
    CandStage my;
    if (cx.lane < K) my = cx.CS[cx.lane];
    else { my.idx = kNoIdx; my.key = -__builtin_inf(); }
    for (int i = 0; i < nb; ++i) {
        PodStage ps_n = ps;
        CandStage my_n = my;
        if (i + 1 < nb) {
            ps_n = cx.PS[i + 1];
            if (cx.lane < K) my_n = cx.CS[(i + 1) * K + cx.lane];
        }
        if (commit_step<K, PRIO, DOM, LAB, F53, ST>(A, cx, i, ps, my, ph)) return i;
        ps = ps_n;
        my = my_n;
    }
    return nb;
}

template <int K, int PRIO, int DOM, bool LAB, bool F53>
__global__ __launch_bounds__(64) void k_commit(CommitArgs A) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical: win issue arbitration over co-resident score waves
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x;
    const int64_t p0 = *A.plan;
    const int64_t cursor = A.ctl->cursor;
    if (p0 < 0 || p0 >= A.pods.p || p0 != cursor) {
        // nothing to do, or a speculative batch invalidated by an earlier truncation: skip it
        if (lane == 0) {
            A.xout->count = 0;
            if (p0 >= 0 && p0 < A.pods.p) A.ctl->stats[3] += 1;
            plan_after_commit(A, false, cursor);
        }
        publish_committed(A);
        return;
    }
    CommitCtx cx;
    cx.hkey = reinterpret_cast<int32_t *>(smem);
    char *p = smem + kTouchHash * sizeof(int32_t);
    cx.filt = reinterpret_cast<uint32_t *>(p);
    p += kTouchFilterWords * sizeof(uint32_t);
    cx.T = reinterpret_cast<Touched *>(p);
    p += (size_t)2 * A.B * sizeof(Touched);
    PodStage *PS = reinterpret_cast<PodStage *>(p);
    p += (size_t)A.B * sizeof(PodStage);
    CandStage *CS = reinterpret_cast<CandStage *>(p);
    cx.PS = PS;
    cx.CS = CS;
    cx.lane = lane;
    cx.placed = 0;
    cx.p0 = p0;
    const int nb = (int)((A.pods.p - p0 < A.B) ? A.pods.p - p0 : A.B);
    cx.y3 = recip(3.0);
    for (int w = lane; w < kTouchHash; w += 64) cx.hkey[w] = -1;
    for (int w = lane; w < kTouchFilterWords; w += 64) cx.filt[w] = 0;
    for (int b = lane; b < nb; b += 64) {
        PodStage s;
        s.rc = A.pods.rc[p0 + b]; s.rm = A.pods.rm[p0 + b]; s.rp = A.pods.rp[p0 + b];
        s.sel = LAB ? A.pods.sel[p0 + b] : 0;
        s.fc0 = A.fc0[b];
        s.cut = A.lists[(size_t)b * K].pad;
        s.pad = 0;
        PS[b] = s;
    }
    for (int e = lane; e < nb * K; e += 64) {
        const Rec r = A.lists[e];
        CandStage c;
        c.key = r.key; c.idx = r.valid ? r.idx : kNoIdx; c.price = r.price;
        c.a[0] = r.a[0]; c.a[1] = r.a[1]; c.a[2] = r.a[2]; c.labels = r.labels;
        CS[e] = c;
    }
    __syncthreads();
    // inherit the nodes the previous batch committed: this batch was scored before those commits
    const int nin = A.xin->count;
    for (int e = lane; e < nin; e += 64) {
        const XRec &xi = A.xin->e[e];
        Touched &x = cx.T[e];
        x.idx = xi.idx; x.mine = 0;
        for (int r = 0; r < 3; ++r) {
            x.s0[r] = xi.sb[r];
            x.sb[r] = xi.cur[r];
            x.cur[r] = xi.cur[r];
            x.curf[r] = (double)xi.cur[r];
            x.cury[r] = recip_or_zero(xi.cur[r], x.curf[r]);
        }
        x.labels = xi.labels; x.price = xi.price; x.pad2 = 0;
        uint32_t h = thash(xi.idx);
        while (atomicCAS(&cx.hkey[h], -1, xi.idx) != -1) h = (h + 1) & (kTouchHash - 1);
        atomicOr(&cx.filt[((uint32_t)xi.idx & 0xffffu) >> 5], 1u << ((uint32_t)xi.idx & 31));
    }
    cx.nT = nin;
    __syncthreads();

    uint64_t ph[4] = {0, 0, 0, 0};
    int done;
    if (A.dbg) {
        const uint64_t tl0 = stamp();
        done = commit_loop<K, PRIO, DOM, LAB, F53, true>(A, cx, nb, ph);
        const uint64_t tl1 = stamp();
        if (lane == 0) {
            A.dbg[0] += ph[0]; A.dbg[1] += ph[1]; A.dbg[2] += ph[2]; A.dbg[3] += ph[3];
            A.dbg[4] += tl1 - tl0; A.dbg[5] += done; A.dbg[6] += cx.nT; A.dbg[7] += 1;
        }
    } else {
        done = commit_loop<K, PRIO, DOM, LAB, F53, false>(A, cx, nb, ph);
    }
    __syncthreads();
    // export this batch's commits (wave-ordered compaction)
    int base = 0;
    for (int t0 = 0; t0 < cx.nT; t0 += 64) {
        const int t = t0 + lane;
        const bool m = t < cx.nT && cx.T[t].mine;
        const uint64_t mask = __ballot(m);
        if (m) {
            const Touched &x = cx.T[t];
            XRec &o = A.xout->e[base + __popcll(mask & ((1ull << lane) - 1))];
            o.idx = x.idx; o.pad = 0;
            o.sb[0] = x.sb[0]; o.sb[1] = x.sb[1]; o.sb[2] = x.sb[2];
            o.cur[0] = x.cur[0]; o.cur[1] = x.cur[1]; o.cur[2] = x.cur[2];
            o.labels = x.labels; o.price = x.price; o.pad2 = 0;
        }
        base += __popcll(mask);
    }
    if (lane == 0) {
        A.xout->count = base;
        A.ctl->cursor = p0 + done;
        A.ctl->stats[0] += 1;
        A.ctl->stats[1] += (done < nb) ? 1 : 0;
        A.ctl->stats[2] += cx.placed;
        plan_after_commit(A, done < nb, p0 + done);
    }
    publish_committed(A);
}

// Pipeline control at the start of a batched call: batch 0 starts at pod 0, batch 1 speculatively at B;
// every later plan is written by the commit two batches earlier (plan_after_commit).
__global__ void k_ctl_init(Ctl *ctl, int B, int64_t P, int lag) {
    if (threadIdx.x != 0) return;
    ctl->cursor = 0; ctl->spec_next = 0; ctl->resync = 0;
    for (int i = 0; i < 5; ++i) ctl->stats[i] = 0;
    ctl->scored = 0;
    ctl->committed = 0;
    for (int i = 0; i < 4; ++i) { ctl->arrive[i].v = 0; ctl->merged[i].v = 0; }
    for (int i = 0; i < kCtlReplicas; ++i) ctl->committed_x[i].v = 0;
    ctl->rescue_req.v = 0;
    ctl->rescue_done.v = 0;
    for (int i = 0; i < 16; ++i) (&ctl->hrec.v)[i] = 0;  // (v and pad: the two hand-off granules)
    ctl->polls_rmw = 0;
    for (int i = 0; i < kPlanRing; ++i) ctl->cursor_at[i] = 0;
    ctl->nact = 0;
    for (int i = 0; i < kPlanRing; ++i) ctl->plan[i] = -1;
    // the first `lag` plans (batch b's commit plans batch b + lag)
    for (int i = 0; i < lag; ++i) ctl->plan[i] = (int64_t)i * B < P ? (int64_t)i * B : -1;
}

// Write one batch's committed nodes into this rank's node rows.
__global__ void k_apply_batch(const XBuf *x, NodeRec *nodes, int64_t node_lo, int64_t n_local) {
    const int n = x->count;
    for (int e = threadIdx.x; e < n; e += blockDim.x) {
        const XRec &r = x->e[e];
        const int64_t j = (int64_t)r.idx - node_lo;
        if (j >= 0 && j < n_local) set_node(nodes + j, r.cur[0], r.cur[1], r.cur[2]);
    }
}

__global__ void k_apply_delta(NodeRec *nodes, int64_t n, int64_t k, const int32_t *idx, const int64_t *d) {
    // Sequential in one lane: deltas may repeat a node and must apply in order (wrapping adds).
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    for (int64_t i = 0; i < k; ++i) {
        const int64_t j = idx[i];
        if (j < 0 || j >= n) continue;
        NodeRec *nd = nodes + j;
        set_node(nd, (int64_t)((uint64_t)nd->a[0] + (uint64_t)d[i]), (int64_t)((uint64_t)nd->a[1] + (uint64_t)d[k + i]),
                 (int64_t)((uint64_t)nd->a[2] + (uint64_t)d[2 * k + i]));
    }
}

// FailedScheduling reasons of one pod against the current node state (anchor/predicate.go:134-148,
// the failures list of :157): per node the FIRST failing check in the reference's order -- CPU,
// Memory, Pod -- then the build-defined label check; 0 = fits.  Lane = node, coalesced u8 stores,
// per-wave ballot counts folded with one vector atomic per reason per wave.
__global__ void k_explain(const NodeRec *nodes, int64_t n, int64_t rc, int64_t rm, int64_t rp, uint64_t sel,
                          int use_labels, uint8_t *reason, unsigned long long *counts) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int r = -1;
    if (j < n) {
        const NodeRec &nd = nodes[j];
        r = nd.a[0] < rc ? 1 : nd.a[1] < rm ? 2 : nd.a[2] < rp ? 3 : (use_labels && (nd.labels & sel) != sel) ? 4 : 0;
        if (reason) reason[j] = (uint8_t)r;
    }
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < kNumReasons; ++k) {
        const unsigned long long m = __ballot(r == k);
        if (lane == 0 && m) atomicAdd(counts + k, (unsigned long long)__popcll(m));
    }
}

__global__ void k_selftest_div(int64_t n, const double *a, const double *b, double *native, double *fast) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = a[i], y = b[i];
    native[i] = x / y;
    fast[i] = qdiv(x, y, recip(y));
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
namespace {

template <int NPT, int PRIO, int DOM, bool LAB, bool F53>
hipError_t exact_one(const ExactArgs &a, int block, bool coop, hipStream_t s) {
    auto fn = k_exact<NPT, PRIO, DOM, LAB, F53>;
    if (coop && a.G > 1) {
        ExactArgs copy = a;
        void *args[] = {&copy};
        return hipLaunchCooperativeKernel((const void *)fn, dim3(a.G), dim3(block), args, 0, s);
    }
    hipLaunchKernelGGL(fn, dim3(a.G), dim3(block), 0, s, a);
    return hipGetLastError();
}

template <int PRIO, int DOM, bool LAB, bool F53>
hipError_t exact_npt(int npt, const ExactArgs &a, int block, bool coop, hipStream_t s) {
    switch (npt) {
        case 1: return exact_one<1, PRIO, DOM, LAB, F53>(a, block, coop, s);
        case 2: return exact_one<2, PRIO, DOM, LAB, F53>(a, block, coop, s);
        case 4: return exact_one<4, PRIO, DOM, LAB, F53>(a, block, coop, s);
        case 8: return exact_one<8, PRIO, DOM, LAB, F53>(a, block, coop, s);
        default: return hipErrorInvalidValue;
    }
}

template <int NPT, int BS, int PRIO, int DOM, bool LAB, bool F53>
hipError_t exact1_one(const ExactArgs &a, hipStream_t s) {
    hipLaunchKernelGGL((k_exact1<NPT, BS, PRIO, DOM, LAB, F53>), dim3(1), dim3(BS), 0, s, a);
    return hipGetLastError();
}
// (npt, block): resource slots <= 4 per thread of 1024 (registers); best-price more
template <int PRIO, int DOM, bool LAB, bool F53>
hipError_t exact1_npt(int npt, int bs, const ExactArgs &a, hipStream_t s) {
    if (bs == 1024) {
        switch (npt) {
            case 1: return exact1_one<1, 1024, PRIO, DOM, LAB, F53>(a, s);
            case 2: return exact1_one<2, 1024, PRIO, DOM, LAB, F53>(a, s);
            case 3: return exact1_one<3, 1024, PRIO, DOM, LAB, F53>(a, s);
            case 4: return exact1_one<4, 1024, PRIO, DOM, LAB, F53>(a, s);
            default: break;
        }
        if constexpr (PRIO == kPrioPrice) {
            switch (npt) {
                case 5: return exact1_one<5, 1024, PRIO, DOM, LAB, F53>(a, s);
                case 6: return exact1_one<6, 1024, PRIO, DOM, LAB, F53>(a, s);
                case 8: return exact1_one<8, 1024, PRIO, DOM, LAB, F53>(a, s);
                case 12: return exact1_one<12, 1024, PRIO, DOM, LAB, F53>(a, s);
                case 16: return exact1_one<16, 1024, PRIO, DOM, LAB, F53>(a, s);
                default: return hipErrorInvalidValue;
            }
        }
        return hipErrorInvalidValue;
    }
    if constexpr (PRIO == kPrioPrice) {
        if (bs == 512 && npt == 10) return exact1_one<10, 512, PRIO, DOM, LAB, F53>(a, s);
        if (bs == 256 && npt == 20) return exact1_one<20, 256, PRIO, DOM, LAB, F53>(a, s);
    }
    return hipErrorInvalidValue;
}

template <int KC, int PRIO, int DOM, bool LAB, bool F53>
hipError_t score_one(const ScoreArgs &a, int pod_groups, hipStream_t s) {
    const size_t lds = score_lds_bytes(KC);
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void *)k_score_topk<KC, PRIO, DOM, LAB, F53>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    dim3 grid((unsigned)(a.n_chunks / kScoreWaves), pod_groups);
    hipLaunchKernelGGL((k_score_topk<KC, PRIO, DOM, LAB, F53>), grid, dim3(kScoreThreads), lds, s, a);
    return hipGetLastError();
}

template <int PRIO, int DOM, bool LAB, bool F53>
hipError_t score_k(int KC, const ScoreArgs &a, int pg, hipStream_t s) {
    switch (KC) {
        case 2: return score_one<2, PRIO, DOM, LAB, F53>(a, pg, s);
        case 4: return score_one<4, PRIO, DOM, LAB, F53>(a, pg, s);
        case 8: return score_one<8, PRIO, DOM, LAB, F53>(a, pg, s);
        case 16: return score_one<16, PRIO, DOM, LAB, F53>(a, pg, s);
        default: return hipErrorInvalidValue;
    }
}

template <int KIN, int K>
hipError_t merge_kk(bool rec, bool fin, const MergeArgs &a, hipStream_t s) {
    dim3 grid(a.C_out, a.B);
    if (rec) {
        if (!fin) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_merge<KIN, K, true, true>), grid, dim3(64), 0, s, a);
    } else if (fin) {
        hipLaunchKernelGGL((k_merge<KIN, K, false, true>), grid, dim3(64), 0, s, a);
    } else {
        hipLaunchKernelGGL((k_merge<KIN, K, false, false>), grid, dim3(64), 0, s, a);
    }
    return hipGetLastError();
}

template <int K>
hipError_t merge_k(int KIN, bool rec, bool fin, const MergeArgs &a, hipStream_t s) {
    if (KIN == K) return merge_kk<K, K>(rec, fin, a, s);
    if (rec) return hipErrorInvalidValue;  // rank lists always hold K entries
    switch (KIN) {
        case 2: return merge_kk<2, K>(false, fin, a, s);
        case 4: return K > 4 ? merge_kk<(K > 4 ? 4 : K), K>(false, fin, a, s) : hipErrorInvalidValue;
        case 8: return K > 8 ? merge_kk<(K > 8 ? 8 : K), K>(false, fin, a, s) : hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
}

template <int K, int PRIO, int DOM, bool LAB, bool F53>
hipError_t commit_one(const CommitArgs &a, size_t lds, hipStream_t s) {
    static bool attr_set = false;
    const void *fn = (const void *)k_commit<K, PRIO, DOM, LAB, F53>;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 4096);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    hipLaunchKernelGGL((k_commit<K, PRIO, DOM, LAB, F53>), dim3(1), dim3(64), lds, s, a);
    return hipGetLastError();
}

template <int PRIO, int DOM, bool LAB, bool F53>
hipError_t commit_k(int K, const CommitArgs &a, size_t lds, hipStream_t s) {
    switch (K) {
        case 4: return commit_one<4, PRIO, DOM, LAB, F53>(a, lds, s);
        case 8: return commit_one<8, PRIO, DOM, LAB, F53>(a, lds, s);
        case 16: return commit_one<16, PRIO, DOM, LAB, F53>(a, lds, s);
        default: return hipErrorInvalidValue;
    }
}


}  // namespace

namespace {
template <int PRIO, int DOM, bool LAB, bool F53>
hipError_t score_attr_k(int KC, hipFuncAttributes *at) {
    switch (KC) {
        case 2: return hipFuncGetAttributes(at, (const void *)k_score_topk<2, PRIO, DOM, LAB, F53>);
        case 4: return hipFuncGetAttributes(at, (const void *)k_score_topk<4, PRIO, DOM, LAB, F53>);
        case 8: return hipFuncGetAttributes(at, (const void *)k_score_topk<8, PRIO, DOM, LAB, F53>);
        case 16: return hipFuncGetAttributes(at, (const void *)k_score_topk<16, PRIO, DOM, LAB, F53>);
        default: return hipErrorInvalidValue;
    }
}
template <int K, int PRIO, int DOM, bool LAB, bool F53>
hipError_t commit_attr_one(hipFuncAttributes *at) {
    return hipFuncGetAttributes(at, (const void *)k_commit<K, PRIO, DOM, LAB, F53>);
}
template <int PRIO, int DOM, bool LAB, bool F53>
hipError_t commit_attr_k(int K, hipFuncAttributes *at) {
    switch (K) {
        case 4: return commit_attr_one<4, PRIO, DOM, LAB, F53>(at);
        case 8: return commit_attr_one<8, PRIO, DOM, LAB, F53>(at);
        case 16: return commit_attr_one<16, PRIO, DOM, LAB, F53>(at);
        default: return hipErrorInvalidValue;
    }
}
hipError_t score_attributes(int KC, int prio, int dom, bool lab, bool f53, hipFuncAttributes *at) {
    KSCHED_DISPATCH(prio, dom, lab, f53, (score_attr_k<P_, D_, L_, F_>(KC, at)));
}
hipError_t seq_commit_attributes(int K, int prio, int dom, bool lab, bool f53, hipFuncAttributes *at) {
    KSCHED_DISPATCH(prio, dom, lab, f53, (commit_attr_k<P_, D_, L_, F_>(K, at)));
}
int alloc_vgprs(int n) { return (n + 7) / 8 * 8; }
}  // namespace

bool commit_fits_beside_score(int KC, int K, int B, bool spc, int prio, int dom, bool lab, bool f53) {
    hipFuncAttributes sa{}, ca{};
    size_t commit_lds = 0;
    if (score_attributes(KC, prio, dom, lab, f53, &sa) != hipSuccess) return false;
    if (spc) {
        if (commit_spc_attributes(K, prio, dom, lab, f53, &ca, &commit_lds) != hipSuccess) return false;
    } else {
        if (seq_commit_attributes(K, prio, dom, lab, f53, &ca) != hipSuccess) return false;
        commit_lds = commit_lds_bytes(B, K);
    }
    const int score_waves_per_simd = kScoreThreads / 64 / 4;
    const int commit_waves_per_simd = spc ? kSpcThreads / 64 / 4 : 1;
    const int vgpr = score_waves_per_simd * alloc_vgprs(sa.numRegs) + commit_waves_per_simd * alloc_vgprs(ca.numRegs);
    const size_t lds = sa.sharedSizeBytes + score_lds_bytes(KC) + ca.sharedSizeBytes + commit_lds;
    const int waves = kScoreThreads / 64 + (spc ? kSpcThreads / 64 : 1);
    return vgpr <= 512 && lds <= 160 * 1024 && waves <= 32;
}

hipError_t launch_prep_nodes(NodeRec *nodes, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_prep_nodes, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, nodes, n);
    return hipGetLastError();
}

hipError_t launch_exact(int npt, int prio, int dom, bool lab, bool f53, const ExactArgs &a, int block, bool coop,
                        hipStream_t s) {
    KSCHED_DISPATCH(prio, dom, lab, f53, (exact_npt<P_, D_, L_, F_>(npt, a, block, coop, s)));
}

hipError_t launch_exact1(int npt, int bs, int prio, int dom, bool lab, bool f53, const ExactArgs &a, hipStream_t s) {
    KSCHED_DISPATCH(prio, dom, lab, f53, (exact1_npt<P_, D_, L_, F_>(npt, bs, a, s)));
}

hipError_t launch_score_topk(int KC, int prio, int dom, bool lab, bool f53, const ScoreArgs &a, int pod_groups,
                             hipStream_t s) {
    KSCHED_DISPATCH(prio, dom, lab, f53, (score_k<P_, D_, L_, F_>(KC, a, pod_groups, s)));
}

hipError_t launch_merge(int KIN, int K, bool input_rec, bool final_stage, const MergeArgs &a, hipStream_t s) {
    switch (K) {
        case 4: return merge_k<4>(KIN, input_rec, final_stage, a, s);
        case 8: return merge_k<8>(KIN, input_rec, final_stage, a, s);
        case 16: return merge_k<16>(KIN, input_rec, final_stage, a, s);
        default: return hipErrorInvalidValue;
    }
}

namespace {
template <int K>
hipError_t merge_pod_k(int KC, const MergeArgs &a, hipStream_t s) {
    switch (KC) {
        case 2: hipLaunchKernelGGL((k_merge_pod<2, K>), dim3(a.B), dim3(kMergeThreads), 0, s, a); break;
        case 4: hipLaunchKernelGGL((k_merge_pod<4, K>), dim3(a.B), dim3(kMergeThreads), 0, s, a); break;
        case 8: hipLaunchKernelGGL((k_merge_pod<8, K>), dim3(a.B), dim3(kMergeThreads), 0, s, a); break;
        case 16: hipLaunchKernelGGL((k_merge_pod<16, K>), dim3(a.B), dim3(kMergeThreads), 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
}  // namespace

hipError_t launch_merge_pod(int KC, int K, const MergeArgs &a, hipStream_t s) {
    if (a.C_in > kMergeThreads || KC > K) return hipErrorInvalidValue;
    switch (K) {
        case 4: return merge_pod_k<4>(KC, a, s);
        case 8: return merge_pod_k<8>(KC, a, s);
        case 16: return merge_pod_k<16>(KC, a, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_commit(int K, int prio, int dom, bool lab, bool f53, const CommitArgs &a, size_t lds_bytes,
                         hipStream_t s) {
    KSCHED_DISPATCH(prio, dom, lab, f53, (commit_k<P_, D_, L_, F_>(K, a, lds_bytes, s)));
}

hipError_t launch_apply_delta(NodeRec *nodes, int64_t n, int64_t k, const int32_t *idx, const int64_t *d,
                              hipStream_t s) {
    hipLaunchKernelGGL(k_apply_delta, dim3(1), dim3(64), 0, s, nodes, n, k, idx, d);
    return hipGetLastError();
}

hipError_t launch_explain(const NodeRec *nodes, int64_t n, int64_t rc, int64_t rm, int64_t rp, uint64_t sel,
                          bool use_labels, uint8_t *reason, unsigned long long *counts, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_explain, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, nodes, n, rc, rm, rp, sel,
                       (int)use_labels, reason, counts);
    return hipGetLastError();
}

hipError_t launch_ctl_init(Ctl *ctl, int B, int64_t P, int lag, hipStream_t s) {
    hipLaunchKernelGGL(k_ctl_init, dim3(1), dim3(64), 0, s, ctl, B, P, lag);
    return hipGetLastError();
}

__global__ void k_zero_sys(uint64_t *p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        __hip_atomic_store(p + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_zero_sys(void *p, size_t bytes, hipStream_t s) {
    const int64_t n = (int64_t)(bytes / 8);
    if (n <= 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(k_zero_sys, dim3((unsigned)blocks), dim3(256), 0, s, static_cast<uint64_t *>(p), n);
    return hipGetLastError();
}

hipError_t launch_apply_batch(const XBuf *x, NodeRec *nodes, int64_t node_lo, int64_t n_local, hipStream_t s) {
    hipLaunchKernelGGL(k_apply_batch, dim3(1), dim3(256), 0, s, x, nodes, node_lo, n_local);
    return hipGetLastError();
}

hipError_t launch_selftest_div(int64_t n, const double *a, const double *b, double *native, double *fast,
                               hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_selftest_div, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, a, b, native, fast);
    return hipGetLastError();
}

}  // namespace ksched
