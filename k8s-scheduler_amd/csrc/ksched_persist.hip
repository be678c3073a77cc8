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
// -- no L2 write-back fences.  Every wait is bounded (2 s -> error word 5).
// Snapshot semantics are the stream pipeline's (score(b) sees every commit up to b-2, commit(b)
// inherits b-1's), so results are bit-identical; tests/test_gpu_parity.py runs both.
#include <hip/hip_runtime.h>

#include "ksched_kernels.h"
#include "ksched_merge.h"

namespace ksched {

namespace {

constexpr int kPW = 8;                     // score waves per workgroup
constexpr int kPThreads = kPW * 64;        // == kMergeThreads: a merger runs merge_pod_body as is
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
    __shared__ int s_stop, s_rank;
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
        for (int r = wave; r < R; r += kPW) {
            const int64_t j = g + (int64_t)r * G;
            if (j >= n) break;
            const NodeRec &nd = rows[r];
            const int64_t ac = nd.a[0], am = nd.a[1], ap = nd.a[2];
            const bool f = fits(rc, rm, rp, sel, ac, am, ap, nd.labels, LAB);
            cnt += f;
            double k;
            const bool el = pair_key_fast<PRIO, DOM, F53>(f, rc, rm, rp, rcf, rmf, rpf, ac, am, ap, nd.af[0], nd.af[1],
                                                          nd.af[2], nd.y[0], nd.y[1], nd.y[2], y3, nd.price, &k);
            double ck = el ? k : -__builtin_inf();
            int32_t ci = (int32_t)j;
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
        __syncthreads();  // s_cnt zeroed before any wave adds
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
        // ---- arrive; the last B arrivals of the batch merge one pod each ----
        const int slot = (int)((nact - 1) % 4);
        const unsigned long long use = (unsigned long long)((nact - 1) / 4);  // earlier uses of the slot
        if (tid == 0) {
            if (g == 0) trace_at(P, b, 5);
            const unsigned long long old = __hip_atomic_fetch_add(&ctl->arrive[slot], 1ull, __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT);
            s_rank = (int)(old - use * (unsigned long long)G);
        }
        __syncthreads();
        const int rank = s_rank;
        if (rank == G - 1 && tid == 0) trace_at(P, b, 1);
        if (rank >= G - P.B) {
            if (tid == 0) {
                s_stop = spin_ge(&ctl->arrive[slot], (use + 1) * (unsigned long long)G, P.timeout_ticks) ? 0 : 1;
                if (s_stop) set_err(P.err, 7);
            }
            __syncthreads();
            if (s_stop) return;
            if (rank == G - 1 && tid == 0) trace_at(P, b, 7);
            char *lb = P.lring + (size_t)(b % 4) * P.lists_bytes;
            MergeArgs ma{};
            ma.in = part; ma.in_cnt = part_cnt; ma.C_in = G; ma.C_out = 1; ma.chunk_input = 1;
            ma.cursor = &ctl->plan[b % kPlanRing]; ma.P = NP; ma.B = P.B;
            ma.nodes = P.nodes; ma.node_offset = 0;
            ma.out_rec = reinterpret_cast<Rec *>(lb);
            ma.out_fc = reinterpret_cast<int64_t *>(lb + (size_t)P.B * K * sizeof(Rec));
            merge_pod_body<KC, K, true>(ma, rank - (G - P.B));
            drain_stores();
            __syncthreads();
            if (tid == 0) {
                const unsigned long long m =
                    __hip_atomic_fetch_add(&ctl->merged[slot], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (m + 1 == (use + 1) * (unsigned long long)P.B) trace_at(P, b, 2);
            }
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

size_t persist_score_lds(int KC, int rows_per_wg) {
    // merge_pod_body's static arrays come on top: 512 lists x KC x 12 B + ~4 KiB
    const size_t need = (size_t)rows_per_wg * sizeof(NodeRec) + (size_t)(kPW / 2) * KC * 64 * 12 + 64 * 4;
    const size_t static_merge = (size_t)kMergeThreads * KC * 12 + 4096;
    if (need + static_merge > 160 * 1024) return 0;
    return need < kExclusiveLds ? kExclusiveLds : need;
}

namespace {

template <int KC, int K, int PRIO, int DOM, bool LAB, bool F53>
hipError_t persist_one(const PersistArgs &a, size_t lds, hipStream_t s) {
    auto fn = k_persist_score<KC, K, PRIO, DOM, LAB, F53>;
    hipFuncAttributes at{};
    hipError_t e = hipFuncGetAttributes(&at, (const void *)fn);
    if (e != hipSuccess) return e;
    if (at.sharedSizeBytes + lds > 160 * 1024) return hipErrorInvalidValue;  // caller falls back
    e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    // a plain launch: G <= CUs - 1 workgroups that each exclude a second one from their CU are all
    // resident beside the commit workgroup (a cooperative launch would wait for the running commit
    // kernel to drain first -- measured: it never starts)
    hipLaunchKernelGGL(fn, dim3(a.G), dim3(kPThreads), lds, s, a);
    return hipGetLastError();
}

template <int KC, int PRIO, int DOM, bool LAB, bool F53>
hipError_t persist_k(int K, const PersistArgs &a, size_t lds, hipStream_t s) {
    switch (K) {
        case 4: return KC <= 4 ? persist_one<(KC <= 4 ? KC : 4), 4, PRIO, DOM, LAB, F53>(a, lds, s) : hipErrorInvalidValue;
        case 8: return KC <= 8 ? persist_one<(KC <= 8 ? KC : 8), 8, PRIO, DOM, LAB, F53>(a, lds, s) : hipErrorInvalidValue;
        case 16: return persist_one<KC, 16, PRIO, DOM, LAB, F53>(a, lds, s);
        default: return hipErrorInvalidValue;
    }
}

template <int PRIO, int DOM, bool LAB, bool F53>
hipError_t persist_kc(int KC, int K, const PersistArgs &a, size_t lds, hipStream_t s) {
    switch (KC) {
        case 2: return persist_k<2, PRIO, DOM, LAB, F53>(K, a, lds, s);
        case 4: return persist_k<4, PRIO, DOM, LAB, F53>(K, a, lds, s);
        case 8: return persist_k<8, PRIO, DOM, LAB, F53>(K, a, lds, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

hipError_t launch_persist(int KC, int K, int prio, int dom, bool lab, bool f53, const PersistArgs &a, size_t lds,
                          hipStream_t score_stream, hipStream_t commit_stream) {
    if (a.B > 64 || a.B > a.G || a.G < 1) return hipErrorInvalidValue;
    // the commit workgroup first: it must be resident before the score grid fills the other CUs
    hipError_t e = launch_persist_commit(K, prio, dom, lab, f53, a, commit_stream);
    if (e != hipSuccess) return e;
    KSCHED_DISPATCH(prio, dom, lab, f53, (persist_kc<P_, D_, L_, F_>(KC, K, a, lds, score_stream)));
}

}  // namespace ksched
