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

#include <cstdio>
#include <cstdlib>

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

__device__ __forceinline__ bool spin_ge(const PersistArgs &P, int slot, const unsigned long long *p,
                                        unsigned long long v, unsigned long long *seen) {
    return poll_ge(p, v, P.timeout_ticks, &P.ctl->polls_rmw, seen, P.prog ? P.prog + kProgWords * slot + 2 : nullptr);
}

// the first failure names the wait that timed out (ksched_sync reports it)
__device__ __forceinline__ void set_err(int32_t *err, int32_t code) { atomicCAS(err, 0, code); }

// Cross-device granules: system-scope relaxed 8-byte accesses (global_store/load ... sc0 sc1) on the
// uncached receive rings; an 8-byte store arrives whole, so a granule whose tag matches holds its word.
__device__ __forceinline__ void st_sys(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld_sys(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// poll one granule until it carries `tag` (false: timed out)
__device__ __forceinline__ bool granule_wait(const uint64_t *p, uint32_t tag, int64_t limit, uint32_t *word) {
    uint64_t v = ld_sys(p);
    if ((uint32_t)(v >> 32) != tag) {
        const uint64_t t0 = wall_clock64();
        do {
            if ((int64_t)(wall_clock64() - t0) > limit) return false;
            __builtin_amdgcn_s_sleep(1);
            v = ld_sys(p);
        } while ((uint32_t)(v >> 32) != tag);
    }
    *word = (uint32_t)v;
    return true;
}

// Rank merge of pod m's R exchanged lists (wave 0, lane = source rank; the stream pipeline's
// k_merge<INPUT_REC> rule): K rounds of wave arg-best over the lists' heads, entries ranking below the
// best cutoff of a cut list dropped, cut when any input was cut or entries were left over.
template <int K>
__device__ __forceinline__ void rank_merge_msgs(const uint32_t *all, int R, Rec *out, int64_t *out_fc) {
    constexpr int MW = msg_words(K);
    const int lane = threadIdx.x & 63;
    const bool has = lane < R;
    const uint32_t *msg = all + (has ? lane : 0) * MW;
    auto rec_key = [&](int q) {
        return __longlong_as_double((long long)(((uint64_t)msg[q * kRecWords + 1] << 32) | msg[q * kRecWords]));
    };
    int n = 0;
    if (has) {
#pragma unroll
        for (int q = 0; q < K; ++q) n += msg[q * kRecWords + 3] != 0;  // valid entries form a prefix
    }
    const bool cut = has && msg[13] != 0;  // entry 0's pad (Rec word 13)
    int64_t cnt = has ? (int64_t)(((uint64_t)msg[K * kRecWords + 1] << 32) | msg[K * kRecWords]) : 0;
    cnt = wave_sum_i64(cnt);
    double ck = (cut && n > 0) ? rec_key(n - 1) : -__builtin_inf();
    int32_t ci = (cut && n > 0) ? (int32_t)msg[(n - 1) * kRecWords + 2] : kNoIdx;
    const bool anycut = __ballot(cut) != 0;
    {
        int32_t aux = 0;
        wave_argbest(ck, ci, aux);
    }
    int h = 0;
    double mk = -__builtin_inf();
    int32_t mi = kNoIdx, msrc = -1;
    for (int r = 0; r < K; ++r) {
        double k = (h < n) ? rec_key(h) : -__builtin_inf();
        int32_t ix = (h < n) ? (int32_t)msg[h * kRecWords + 2] : kNoIdx;
        int32_t src = lane * K + h;
        wave_argbest(k, ix, src);
        if (ix == kNoIdx) break;  // wave-uniform
        if (src == lane * K + h) ++h;
        if (lane == r) { mk = k; mi = ix; msrc = src; }
    }
    const bool left = __ballot(h < n) != 0;
    if (anycut && mi != kNoIdx && better(ck, ci, mk, mi)) { mk = -__builtin_inf(); mi = kNoIdx; }
    const int32_t cut_out = (anycut || left) ? 1 : 0;
    if (lane < K) {
        Rec r{};
        if (mi != kNoIdx) {
            uint32_t *w = reinterpret_cast<uint32_t *>(&r);
            const uint32_t *sw = all + (msrc / K) * MW + (msrc % K) * kRecWords;
#pragma unroll
            for (int x = 0; x < kRecWords; ++x) w[x] = sw[x];
        } else {
            r.key = -__builtin_inf(); r.idx = kNoIdx; r.valid = 0;
        }
        r.pad = lane == 0 ? cut_out : 0;
        store_rec<true>(out + lane, r);
    }
    if (lane == 0) store_i64<true>(out_fc, cnt);
}

__device__ __forceinline__ void set_row(NodeRec *nd, int64_t a0, int64_t a1, int64_t a2) {
    nd->a[0] = a0; nd->a[1] = a1; nd->a[2] = a2;
    const double f0 = (double)a0, f1 = (double)a1, f2 = (double)a2;
    nd->af[0] = f0; nd->af[1] = f1; nd->af[2] = f2;
    nd->y[0] = recip_or_zero(a0, f0); nd->y[1] = recip_or_zero(a1, f1); nd->y[2] = recip_or_zero(a2, f2);
}

}  // namespace

template <int KC, int K, int PRIO, int DOM, bool LAB, bool F53>
__global__ __launch_bounds__(kPThreads) __attribute__((amdgpu_num_vgpr(72))) void k_persist_score(PersistArgs P) {
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
        // ---- wave 0: wait for commit(b-2), then ONE round of loads -- its plan for b, the cursor after it,
        // its export (count and entries, lane = entry) -- and apply the exported nodes this workgroup owns
        // to its LDS rows before the barrier (the other waves never touch the export) ----
        if (wave == 0) {
            int stop = 0;
            if (lane == 0) {
                unsigned long long seen = 0;
                prog_at(P, g, b, kProgWaitCommit, 0);
                if (b >= 2 && !spin_ge(P, g, &ctl->committed_x[g % kCtlReplicas].v, (unsigned long long)(b - 1), &seen)) {
                    set_err(P.err, 6);
                    prog_at(P, g, b, kProgWaitCommit | kProgTimedOut, seen);
                    stop = 2;
                }
                if (g == 0) trace_at(P, b, 6);
            }
            stop = __builtin_amdgcn_readfirstlane(stop);
            wave_mark(P, g, 0, b, 0x10);  // wave 0: its poll ended
            int64_t p0v = 0, donev = 0;
            int errv = 0, nxv = 0;
            uint64_t w0 = 0, w4 = 0, w5 = 0, w6 = 0;
            const XBuf *xb = reinterpret_cast<const XBuf *>(P.xring + (size_t)((b >= 2 ? b - 2 : 0) % 4) * P.xbuf_bytes);
            if (lane == 0) {
                p0v = (int64_t)ld_coh(&ctl->plan[b % kPlanRing]);
                donev = b >= 2 ? (int64_t)ld_coh(&ctl->cursor_at[(b - 2) % kPlanRing]) : 0;
                // a failed peer (the commit timed out) ends the call for everyone
                errv = __hip_atomic_load(P.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (b >= 2) {
                nxv = (int)(uint32_t)ld_coh(&xb->count);  // one address: one request for the wave
                if (lane < 2 * P.B) {                      // speculative: entries past the count are ignored
                    const uint64_t *w = reinterpret_cast<const uint64_t *>(&xb->e[lane]);
                    w0 = ld_coh(w); w4 = ld_coh(w + 4); w5 = ld_coh(w + 5); w6 = ld_coh(w + 6);
                }
            }
            auto apply = [&](uint64_t x0, uint64_t x4, uint64_t x5, uint64_t x6) {
                const int64_t j = (int64_t)(int32_t)(uint32_t)x0 - P.node_offset;  // local row
                if (j < 0 || j >= n || j % G != g) return;  // another rank's node, or another workgroup's
                set_row(rows + j / G, (int64_t)x4, (int64_t)x5, (int64_t)x6);
                // the mergers read a candidate's state from its HBM row (sc1)
                st_coh(&P.nodes[j].a[0], x4);
                st_coh(&P.nodes[j].a[1], x5);
                st_coh(&P.nodes[j].a[2], x6);
            };
            if (lane < nxv) apply(w0, w4, w5, w6);
            for (int e = 64 + lane; e < nxv; e += 64) {  // exports beyond 64 entries (B > 64 only)
                const uint64_t *w = reinterpret_cast<const uint64_t *>(&xb->e[e]);
                apply(ld_coh(w), ld_coh(w + 4), ld_coh(w + 5), ld_coh(w + 6));
            }
            if (lane == 0) {
                s_p0 = p0v;
                s_done = donev;
                s_stop = errv != 0 ? 3 : stop;
            }
        } else {
            wave_mark(P, g, wave, b, 0x01);  // at barrier 1
        }
        __syncthreads();
        wave_mark(P, g, wave, b, 0x02);  // past barrier 1 (rows up to date)
        if (s_stop) return;
        const int64_t p0 = s_p0;
        if (s_done >= NP) break;                  // every pod resolved by commit(b-2) or earlier
        if (p0 < 0 || p0 >= NP) {                 // nothing planned for batch b (identical on every WG)
            if (tid == 0) prog_at(P, g, b, kProgIdle, (uint64_t)p0);
            // a truncation re-plans within two batches; a longer run of empty plans is a protocol error
            if (++idle > kPlanRing) {
                if (tid == 0) set_err(P.err, 8);
                return;
            }
            __syncthreads();  // every wave has read s_done before thread 0 rewrites it
            continue;
        }
        idle = 0;
        ++nact;
        if (tid == 0) {
            if (g == 0) trace_at(P, b, 0);
            prog_at(P, g, b, kProgScan, 0);
        }
        const uint64_t t_go = (P.trace && tid == 0) ? wall_clock64() : 0;
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
                int32_t ci = (int32_t)(P.node_offset + g + (int64_t)(r0 + u * kPW) * G);  // global index
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
        wave_mark(P, g, wave, b, 0x05);  // scanned
        if (g == 0 && tid == 0) trace_at(P, b, 8);
        const uint64_t t_scan = (P.trace && tid == 0) ? wall_clock64() : 0;
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
        wave_mark(P, g, wave, b, 0x06);  // folded and stored, at the arrive barrier
        __syncthreads();
        // ---- arrive (the merger workgroups, k_persist_merge, wait for all G) ----
        const int slot = (int)((nact - 1) % 4);
        if (tid == 0) {
            if (g == 0) trace_at(P, b, 5);
            const unsigned long long old = __hip_atomic_fetch_add(&ctl->arrive[slot].v, 1ull, __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long use = (unsigned long long)((nact - 1) / 4);
            if (old + 1 == (use + 1) * (unsigned long long)G) trace_at(P, b, 1);
            prog_at(P, g, b, kProgArrived, old + 1);
            if (P.trace) prog_add(P, g, t_scan - t_go, wall_clock64() - t_go);
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
// <= 112 VGPRs (amdgpu_num_vgpr counts half the unified gfx950 file): two merger waves per SIMD
// beside the score grid's two (up to 144 VGPRs at KC = 8)
template <int KC, int K>
__global__ __launch_bounds__(kMergeThreads) __attribute__((amdgpu_num_vgpr(56))) void k_persist_merge(PersistArgs P) {
    __shared__ int64_t s_p0, s_done;
    __shared__ int s_stop;
    __shared__ uint32_t s_msg[msg_words(K)];                  // this rank's list of pod m (R > 1)
    __shared__ uint32_t s_all[kMaxXchgRanks * msg_words(K)];  // every rank's list of pod m
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
            unsigned long long seen = 0;
            prog_at(P, P.G + m, b, kProgWaitCommit, 0);
            if (b >= 2 && !spin_ge(P, P.G + m, &ctl->committed_x[m % kCtlReplicas].v, (unsigned long long)(b - 1), &seen)) {
                set_err(P.err, 6);
                prog_at(P, P.G + m, b, kProgWaitCommit | kProgTimedOut, seen);
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
            if (tid == 0) prog_at(P, G + m, b, kProgIdle, (uint64_t)p0);
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
            unsigned long long seen = 0;
            prog_at(P, G + m, b, kProgWaitArrive, 0);
            s_stop = spin_ge(P, G + m, &ctl->arrive[slot].v, (use + 1) * (unsigned long long)G, &seen) ? 0 : 1;
            if (s_stop) {
                set_err(P.err, 7);
                prog_at(P, G + m, b, kProgWaitArrive | kProgTimedOut, seen);
            }
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
        ma.nodes = P.nodes; ma.node_offset = P.node_offset;
        ma.dbg = P.mdbg;
        ma.low_prio = P.merge_low_prio;
        ma.out_rec = reinterpret_cast<Rec *>(lb);
        ma.out_fc = reinterpret_cast<int64_t *>(lb + (size_t)P.B * K * sizeof(Rec));
        const bool xchg = P.R > 1 && p0 + m < NP;  // block-uniform
        if (xchg) ma.lds_msg = s_msg;
        merge_pod_body<KC, K, true>(ma, m);
        if (xchg) {
            // this rank's list of pod m -> slot (a % 4, rank, m) of every rank's ring; then the R lists of
            // pod m from this rank's ring -> rank merge -> the commit's list (lring)
            constexpr int MW = msg_words(K);
            const int R = P.R;
            const uint32_t tag = P.epoch0 + (uint32_t)nact;
            __syncthreads();
            for (int e = tid; e < MW * R; e += kMergeThreads) {
                const int r = e / MW, w = e % MW;
                uint64_t *dst = reinterpret_cast<uint64_t *>(
                    P.rx_peer[r] + ((size_t)(slot * R + P.rank) * P.B + m) * (size_t)P.xchg_stride);
                st_sys(dst + w, (uint64_t)s_msg[w] | ((uint64_t)tag << 32));
            }
            bool ok = true;
            const char *own = P.rx_peer[P.rank];
            for (int e = tid; e < MW * R; e += kMergeThreads) {
                const int r = e / MW, w = e % MW;
                const uint64_t *src = reinterpret_cast<const uint64_t *>(
                    own + ((size_t)(slot * R + r) * P.B + m) * (size_t)P.xchg_stride);
                uint32_t word = 0;
                if (ok && !granule_wait(src + w, tag, P.timeout_ticks, &word)) ok = false;
                s_all[e] = word;
            }
            if (!ok) set_err(P.err, 10);
            s_stop = 0;
            __syncthreads();
            if (!ok) s_stop = 1;
            __syncthreads();
            if (s_stop) return;
            if (tid < 64) rank_merge_msgs<K>(s_all, R, ma.out_rec + (size_t)m * K, ma.out_fc + m);
        }
        drain_stores();
        __syncthreads();
        if (tid == 0 && m == 0) st_coh(&ctl->nact, (uint64_t)nact);
        if (tid == 0) {
            const unsigned long long d =
                __hip_atomic_fetch_add(&ctl->merged[slot].v, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (d + 1 == (use + 1) * (unsigned long long)P.B) trace_at(P, b, 2);
            prog_at(P, G + m, b, kProgMerged, d + 1);
        }
    }
}

// All ranks meet on the device and agree on the minimum of `mine` (tag: this call's epoch0; the
// batches of the call use epoch0 + 1, ...).  One wave; lane r < R writes rank r's barrier granule.
__global__ __launch_bounds__(64) void k_xchg_min(PersistArgs P, int32_t mine, int32_t *out) {
    const int lane = threadIdx.x;
    const size_t off = (size_t)4 * P.R * P.B * (size_t)P.xchg_stride;
    const uint32_t tag = P.epoch0;
    if (lane < P.R) st_sys(reinterpret_cast<uint64_t *>(P.rx_peer[lane] + off) + P.rank, (uint64_t)(uint32_t)mine | ((uint64_t)tag << 32));
    int32_t v = 0x7fffffff;
    bool ok = true;
    if (lane < P.R) {
        uint32_t w = 0;
        ok = granule_wait(reinterpret_cast<const uint64_t *>(P.rx_peer[P.rank] + off) + lane, tag, P.timeout_ticks, &w);
        v = (int32_t)w;
    }
    v = wave_min_i32(v);
    const bool bad = __ballot(!ok) != 0;
    if (lane == 0) {
        if (bad) set_err(P.err, 11);
        *out = bad ? -1 : v;
    }
}

hipError_t launch_xchg_min(const PersistArgs &a, int32_t mine, int32_t *out, hipStream_t s) {
    if (a.R < 2 || a.R > kMaxXchgRanks) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_xchg_min, dim3(1), dim3(64), 0, s, a, mine, out);
    return hipGetLastError();
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
    if (std::getenv("KSCHED_DEBUG"))
        fprintf(stderr, "[ksched persist] score: %d VGPRs %zu+%zu B LDS; merger: %d VGPRs %zu B LDS\n", at.numRegs,
                (size_t)at.sharedSizeBytes, lds, am.numRegs, (size_t)am.sharedSizeBytes);
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
