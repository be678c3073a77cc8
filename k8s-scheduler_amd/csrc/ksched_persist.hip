// ksched_persist.hip -- the single-rank batched pipeline as two resident kernels.
//
// The stream pipeline (ksched_engine.hip enqueue_batched) launches three kernels per batch and links
// them with stream events; on MI355X every cross-queue event costs ~13 us and every launch a few more,
// which is half of a 64-pod batch's wall.  Here the whole call is two launches:
//
//   k_persist_score  G = CUs - 1 workgroups, one per CU (its LDS request excludes a second one).  Each
//                    holds ITS node rows (j = g mod G) in LDS for the whole call -- the score scan never
//                    touches HBM for a node -- and loops over batches:
//                      wait Ctl::committed >= b - 1      (commit(b-2) done: plan(b), XBuf(b-2) final)
//                      apply XBuf(b-2) to its LDS rows   (+ sc1 write-back of a[] for the mergers)
//                      score 64 pods x its rows -> per-pod top-KC list (sc1 stores), arrive
//                      the last B arrivals each merge one pod's G lists into its Rec list (sc1)
//   k_persist_commit one workgroup (ksched_commit_spc.hip) on the CU the grid leaves free: waits for
//                    the B merges of batch b, commits it, publishes Ctl::committed = b + 1.
//
// Every hand-off is MI355X_MICROARCH "valid forms" row 1: sc1 stores of the handed-off bytes, every
// storing wave drained, ONE lane's counter update (atomic add / flag store), sc1 loads after the poll
// -- no L2 write-back fences.  Every wait is bounded (KSCHED_PERSIST_TIMEOUT_MS, default 10 s -> error words 5..9).
// Snapshot semantics are the stream pipeline's (score(b) sees every commit up to b-2, commit(b)
// inherits b-1's), so results are bit-identical; tests/test_gpu_parity.py runs both.
#include <hip/hip_runtime.h>

#include "ksched_kernels.h"
#include "ksched_merge.h"

namespace ksched {

namespace {

constexpr int kPW = 8;                     // score waves per workgroup
constexpr int kPThreads = kPW * 64;
#ifndef KSCHED_PERSIST_PU
#define KSCHED_PERSIST_PU 4
#endif
constexpr int kPU = KSCHED_PERSIST_PU;     // rows per score step (independent key chains)        // == kMergeThreads: a merger runs merge_pod_body as is
constexpr size_t kExclusiveLds = 81 * 1024;  // > 160 KiB / 2: one score workgroup per CU

__device__ __forceinline__ bool spin_ge(const unsigned long long *p, unsigned long long v, int64_t limit) {
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < v) {
        if ((int64_t)(wall_clock64() - t0) > limit) return false;
        __builtin_amdgcn_s_sleep(1);
    }
    return true;
}

// the first failure names the wait that timed out (ksched_sync reports it)
__device__ __forceinline__ void set_err(int32_t *err, int32_t code) { atomicCAS(err, 0, code); }

__device__ __forceinline__ void set_row(NodeRec *nd, int64_t a0, int64_t a1, int64_t a2) {
    nd->a[0] = a0; nd->a[1] = a1; nd->a[2] = a2;
    const double f0 = (double)a0, f1 = (double)a1, f2 = (double)a2;
    nd->af[0] = f0; nd->af[1] = f1; nd->af[2] = f2;
    nd->y[0] = recip_or_zero(a0, f0); nd->y[1] = recip_or_zero(a1, f1); nd->y[2] = recip_or_zero(a2, f2);
}

}  // namespace

template <int KC, int K, int PRIO, int DOM, bool LAB, bool F53>
__global__ __launch_bounds__(kPThreads) void k_persist_score(PersistArgs P) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    NodeRec *rows = reinterpret_cast<NodeRec *>(smem);                    // [rows_per_wg]
    char *fold = smem + (size_t)P.rows_per_wg * sizeof(NodeRec);
    double *s_key = reinterpret_cast<double *>(fold);                     // [W/2][KC][64]
    int32_t *s_idx = reinterpret_cast<int32_t *>(fold + (size_t)(kPW / 2) * KC * 64 * 8);
    int32_t *s_cnt = s_idx + (size_t)(kPW / 2) * KC * 64;                 // [64]
    __shared__ int64_t s_p0, s_done;
    __shared__ int s_stop;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int G = gridDim.x, g = blockIdx.x;
    const int64_t n = P.n_local, NP = P.pods.p;
    const int R = P.rows_per_wg;
    Ctl *ctl = P.ctl;
    // this workgroup's rows j = g + r * G, resident in LDS for the whole call
    for (int e = tid; e < R * 6; e += kPThreads) {
        const int r = e / 6, piece = e % 6;
        const int64_t j = g + (int64_t)r * G;
        if (j < n) reinterpret_cast<int4 *>(rows + r)[piece] = reinterpret_cast<const int4 *>(P.nodes + j)[piece];
    }
    __syncthreads();
    const double y3 = recip(3.0);
    int64_t nact = 0;
    int idle = 0;
    for (int64_t b = 0;; ++b) {
        // ---- wait for commit(b-2): its plan for b, its exported commits, the cursor after it ----
        if (tid == 0) {
            int stop = 0;
            if (b >= 2 && !spin_ge(&ctl->committed, (unsigned long long)(b - 1), P.timeout_ticks)) {
                set_err(P.err, 6);
                stop = 2;
            }
            if (g == 0) trace_at(P, b, 6);
            s_p0 = (int64_t)ld_coh(&ctl->plan[b % kPlanRing]);
            s_done = b >= 2 ? (int64_t)ld_coh(&ctl->cursor_at[(b - 2) % kPlanRing]) : 0;
            // a failed peer (the commit timed out) ends the call for everyone
            if (__hip_atomic_load(P.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) stop = 3;
            s_stop = stop;
        }
        __syncthreads();
        if (s_stop) return;
        const int64_t p0 = s_p0;
        // ---- apply commit(b-2)'s exported nodes to the rows this workgroup owns ----
        if (b >= 2) {
            const XBuf *xb = reinterpret_cast<const XBuf *>(P.xring + (size_t)((b - 2) % 4) * P.xbuf_bytes);
            const int nx = (int)(uint32_t)ld_coh(&xb->count);
            for (int e = tid; e < nx; e += kPThreads) {
                const uint64_t *w = reinterpret_cast<const uint64_t *>(&xb->e[e]);
                const int64_t j = (int64_t)(int32_t)(uint32_t)ld_coh(w);
                if (j % G != g) continue;
                const int64_t c0 = (int64_t)ld_coh(w + 4), c1 = (int64_t)ld_coh(w + 5), c2 = (int64_t)ld_coh(w + 6);
                set_row(rows + j / G, c0, c1, c2);
                // the mergers read a candidate's state from its HBM row (sc1)
                st_coh(&P.nodes[j].a[0], (uint64_t)c0);
                st_coh(&P.nodes[j].a[1], (uint64_t)c1);
                st_coh(&P.nodes[j].a[2], (uint64_t)c2);
            }
        }
        __syncthreads();
        if (s_done >= NP) break;                  // every pod resolved by commit(b-2) or earlier
        if (p0 < 0 || p0 >= NP) {                 // nothing planned for batch b (identical on every WG)
            // a truncation re-plans within two batches; a longer run of empty plans is a protocol error
            if (++idle > kPlanRing) {
                if (tid == 0) set_err(P.err, 8);
                return;
            }
            continue;
        }
        idle = 0;
        ++nact;
        if (g == 0 && tid == 0) trace_at(P, b, 0);
        // ---- score: lane = pod, wave w scans rows r = w, w + W, ... (nodes j = g + r G) ----
        if (tid < 64) s_cnt[tid] = 0;
        const int64_t pod = p0 + lane;
        const bool active = (lane < P.B) && (pod < NP);
        const int64_t rc = active ? P.pods.rc[pod] : 0;
        const int64_t rm = active ? P.pods.rm[pod] : 0;
        const int64_t rp = active ? P.pods.rp[pod] : 0;
        const uint64_t sel = (LAB && active) ? P.pods.sel[pod] : 0;
        const double rcf = (double)rc, rmf = (double)rm, rpf = (double)rp;
        double key[KC];
        int32_t idx[KC];
#pragma unroll
        for (int q = 0; q < KC; ++q) { key[q] = -__builtin_inf(); idx[q] = kNoIdx; }
        int32_t cnt = 0;
        // kPU rows per step: their keys are independent f64 chains the scheduler interleaves (two waves
        // per SIMD hide little latency on their own); inserted in ascending node order afterwards
        for (int r0 = wave; r0 < R; r0 += kPW * kPU) {
            double ks[kPU];
#pragma unroll
            for (int u = 0; u < kPU; ++u) {
                const int r = r0 + u * kPW;
                const int64_t j = g + (int64_t)r * G;
                ks[u] = -__builtin_inf();
                if (r < R && j < n) {  // wave-uniform
                    const NodeRec &nd = rows[r];
                    const int64_t ac = nd.a[0], am = nd.a[1], ap = nd.a[2];
                    const bool f = fits(rc, rm, rp, sel, ac, am, ap, nd.labels, LAB);
                    cnt += f;
                    double k;
                    const bool el = pair_key_fast<PRIO, DOM, F53>(f, rc, rm, rp, rcf, rmf, rpf, ac, am, ap, nd.af[0],
                                                                  nd.af[1], nd.af[2], nd.y[0], nd.y[1], nd.y[2], y3,
                                                                  nd.price, &k);
                    ks[u] = el ? k : -__builtin_inf();
                }
            }
#pragma unroll
            for (int u = 0; u < kPU; ++u) {
                double ck = ks[u];
                int32_t ci = (int32_t)(g + (int64_t)(r0 + u * kPW) * G);
                bool moved = false;  // nodes arrive in ascending index: strict '>' keeps ties in index order
#pragma unroll
                for (int q = 0; q < KC; ++q) {
                    const bool sw = moved || ck > key[q];
                    moved = sw;
                    const double tk = key[q];
                    const int32_t ti = idx[q];
                    key[q] = sw ? ck : tk; idx[q] = sw ? ci : ti;
                    ck = sw ? tk : ck; ci = sw ? ti : ci;
                }
            }
        }
        if (g == 0 && tid == 0) trace_at(P, b, 8);
        __syncthreads();  // s_cnt zeroed before any wave adds
        if (g == 0 && tid == 0) trace_at(P, b, 9);
        if (cnt) atomicAdd(&s_cnt[lane], cnt);
        // fold the wave lists pairwise: W -> W/2 -> ... -> 1 (a list that is cut when full folds into
        // the top-KC of the union, again cut when full: DESIGN.md section 4)
#pragma unroll
        for (int half = kPW / 2; half >= 1; half >>= 1) {
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
        if (g == 0 && tid == 0) trace_at(P, b, 10);
        const size_t part_elems = (size_t)P.B * G;
        Cand *part = P.part + (size_t)(b % 2) * part_elems * KC;
        int64_t *part_cnt = P.part_cnt + (size_t)(b % 2) * part_elems;
        if (wave == 0 && active) {
            Cand *dst = part + ((size_t)lane * G + g) * KC;
#pragma unroll
            for (int q = 0; q < KC; ++q) {
                st_coh(&dst[q].key, (uint64_t)__double_as_longlong(key[q]));
                st_coh(&dst[q].idx, (uint64_t)(uint32_t)idx[q]);  // idx + pad (0)
            }
            st_coh(part_cnt + (size_t)lane * G + g, (uint64_t)(int64_t)s_cnt[lane]);
        }
        drain_stores();
        __syncthreads();
        // ---- arrive (the merger workgroups, k_persist_merge, wait for all G) ----
        const int slot = (int)((nact - 1) % 4);
        if (tid == 0) {
            if (g == 0) trace_at(P, b, 5);
            const unsigned long long old = __hip_atomic_fetch_add(&ctl->arrive[slot], 1ull, __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long use = (unsigned long long)((nact - 1) / 4);
            if (old + 1 == (use + 1) * (unsigned long long)G) trace_at(P, b, 1);
        }
    }
    // every pod is resolved: this workgroup's rows go back to HBM whole (allocatable, cached doubles,
    // reciprocals) for the next call and for ksched_read_nodes
    for (int e = tid; e < R * 6; e += kPThreads) {
        const int r = e / 6, piece = e % 6;
        const int64_t j = g + (int64_t)r * G;
        if (j < n) reinterpret_cast<int4 *>(P.nodes + j)[piece] = reinterpret_cast<const int4 *>(rows + r)[piece];
    }
}

// The merge side: B workgroups, one per pod slot of a batch, resident beside the score grid (small LDS).
// Per active batch: wait for the G arrivals, merge pod m's G lists into its K-entry Rec list (sc1),
// count the merge.  The score workgroups never merge, so a merge never delays the next batch's scan.
template <int KC, int K>
__global__ __launch_bounds__(kMergeThreads) void k_persist_merge(PersistArgs P) {
    __shared__ int64_t s_p0, s_done;
    __shared__ int s_stop;
    const int tid = threadIdx.x;
    const int m = blockIdx.x;
    const int G = P.G;
    const int64_t NP = P.pods.p;
    Ctl *ctl = P.ctl;
    int64_t nact = 0;
    int idle = 0;
    for (int64_t b = 0;; ++b) {
        if (tid == 0) {
            int stop = 0;
            if (b >= 2 && !spin_ge(&ctl->committed, (unsigned long long)(b - 1), P.timeout_ticks)) {
                set_err(P.err, 6);
                stop = 2;
            }
            s_p0 = (int64_t)ld_coh(&ctl->plan[b % kPlanRing]);
            s_done = b >= 2 ? (int64_t)ld_coh(&ctl->cursor_at[(b - 2) % kPlanRing]) : 0;
            if (__hip_atomic_load(P.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) stop = 3;
            s_stop = stop;
        }
        __syncthreads();
        if (s_stop) return;
        const int64_t p0 = s_p0;
        if (s_done >= NP) return;
        if (p0 < 0 || p0 >= NP) {
            if (++idle > kPlanRing) {
                if (tid == 0) set_err(P.err, 8);
                return;
            }
            __syncthreads();  // s_p0 / s_done are rewritten next iteration
            continue;
        }
        idle = 0;
        ++nact;
        const int slot = (int)((nact - 1) % 4);
        const unsigned long long use = (unsigned long long)((nact - 1) / 4);
        if (tid == 0) {
            s_stop = spin_ge(&ctl->arrive[slot], (use + 1) * (unsigned long long)G, P.timeout_ticks) ? 0 : 1;
            if (s_stop) set_err(P.err, 7);
            if (m == 0) trace_at(P, b, 7);
        }
        __syncthreads();
        if (s_stop) return;
        const size_t part_elems = (size_t)P.B * G;
        char *lb = P.lring + (size_t)(b % 4) * P.lists_bytes;
        MergeArgs ma{};
        ma.in = P.part + (size_t)(b % 2) * part_elems * KC;
        ma.in_cnt = P.part_cnt + (size_t)(b % 2) * part_elems;
        ma.C_in = G; ma.C_out = 1; ma.chunk_input = 1;
        ma.cursor = &ctl->plan[b % kPlanRing]; ma.P = NP; ma.B = P.B;
        ma.p0_known = 1; ma.p0v = p0;
        ma.nodes = P.nodes; ma.node_offset = 0;
        ma.dbg = P.mdbg;
        ma.out_rec = reinterpret_cast<Rec *>(lb);
        ma.out_fc = reinterpret_cast<int64_t *>(lb + (size_t)P.B * K * sizeof(Rec));
        merge_pod_body<KC, K, true>(ma, m);
        drain_stores();
        __syncthreads();
        if (tid == 0) {
            const unsigned long long d =
                __hip_atomic_fetch_add(&ctl->merged[slot], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (d + 1 == (use + 1) * (unsigned long long)P.B) trace_at(P, b, 2);
        }
    }
}

size_t persist_score_lds(int KC, int rows_per_wg) {
    // a merger workgroup (merge_pod_body's static arrays: 512 lists x KC x 12 B + ~4 KiB) must fit beside
    const size_t need = (size_t)rows_per_wg * sizeof(NodeRec) + (size_t)(kPW / 2) * KC * 64 * 12 + 64 * 4;
    const size_t static_merge = (size_t)kMergeThreads * KC * 12 + 4096;
    if (need + static_merge > 160 * 1024) return 0;
    return need < kExclusiveLds ? kExclusiveLds : need;
}

namespace {

template <int KC, int K, int PRIO, int DOM, bool LAB, bool F53>
hipError_t persist_one(const PersistArgs &a, size_t lds, hipStream_t s, hipStream_t sm, bool launch) {
    auto fn = k_persist_score<KC, K, PRIO, DOM, LAB, F53>;
    auto fm = k_persist_merge<KC, K>;
    hipFuncAttributes at{}, am{};
    hipError_t e = hipFuncGetAttributes(&at, (const void *)fn);
    if (e != hipSuccess) return e;
    e = hipFuncGetAttributes(&am, (const void *)fm);
    if (e != hipSuccess) return e;
    // one score workgroup + one merger workgroup per CU: LDS, and two waves per SIMD of each in the
    // 512-entry VGPR file (granule 8) -- otherwise the caller falls back to the stream pipeline
    auto vg = [](int r) { return (r + 7) / 8 * 8; };
    if (at.sharedSizeBytes + lds + am.sharedSizeBytes > 160 * 1024) return hipErrorInvalidValue;
    if (2 * vg(at.numRegs) + 2 * vg(am.numRegs) > 512) return hipErrorInvalidValue;
    if (!launch) return hipSuccess;
    e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    // plain launches: G <= CUs - 8 score workgroups that each exclude a second one from their CU are
    // all resident beside the commit workgroup; the B mergers fit beside them (a cooperative launch
    // would wait for the running commit kernel to drain first -- measured: it never starts)
    hipLaunchKernelGGL(fn, dim3(a.G), dim3(kPThreads), lds, s, a);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(fm, dim3(a.B), dim3(kMergeThreads), 0, sm, a);
    return hipGetLastError();
}

template <int KC, int PRIO, int DOM, bool LAB, bool F53>
hipError_t persist_k(int K, const PersistArgs &a, size_t lds, hipStream_t s, hipStream_t sm, bool launch) {
    switch (K) {
        case 4: return KC <= 4 ? persist_one<(KC <= 4 ? KC : 4), 4, PRIO, DOM, LAB, F53>(a, lds, s, sm, launch) : hipErrorInvalidValue;
        case 8: return KC <= 8 ? persist_one<(KC <= 8 ? KC : 8), 8, PRIO, DOM, LAB, F53>(a, lds, s, sm, launch) : hipErrorInvalidValue;
        case 16: return persist_one<KC, 16, PRIO, DOM, LAB, F53>(a, lds, s, sm, launch);
        default: return hipErrorInvalidValue;
    }
}

template <int PRIO, int DOM, bool LAB, bool F53>
hipError_t persist_kc(int KC, int K, const PersistArgs &a, size_t lds, hipStream_t s, hipStream_t sm, bool launch) {
    switch (KC) {
        case 2: return persist_k<2, PRIO, DOM, LAB, F53>(K, a, lds, s, sm, launch);
        case 4: return persist_k<4, PRIO, DOM, LAB, F53>(K, a, lds, s, sm, launch);
        case 8: return persist_k<8, PRIO, DOM, LAB, F53>(K, a, lds, s, sm, launch);
        default: return hipErrorInvalidValue;
    }
}

hipError_t persist_grid(int KC, int K, int prio, int dom, bool lab, bool f53, const PersistArgs &a, size_t lds,
                        hipStream_t s, hipStream_t sm, bool launch) {
    KSCHED_DISPATCH(prio, dom, lab, f53, (persist_kc<P_, D_, L_, F_>(KC, K, a, lds, s, sm, launch)));
}

}  // namespace

hipError_t launch_persist(int KC, int K, int prio, int dom, bool lab, bool f53, const PersistArgs &a, size_t lds,
                          hipStream_t score_stream, hipStream_t commit_stream, hipStream_t merge_stream) {
    if (a.B > 64 || a.G < 1) return hipErrorInvalidValue;
    // check the residency budget before anything is launched (InvalidValue: the caller falls back)
    hipError_t e = persist_grid(KC, K, prio, dom, lab, f53, a, lds, score_stream, merge_stream, false);
    if (e != hipSuccess) return e;
    // the commit workgroup first: it must be resident before the score grid fills the other CUs
    e = launch_persist_commit(K, prio, dom, lab, f53, a, commit_stream);
    if (e != hipSuccess) return e;
    return persist_grid(KC, K, prio, dom, lab, f53, a, lds, score_stream, merge_stream, true);
}

}  // namespace ksched
