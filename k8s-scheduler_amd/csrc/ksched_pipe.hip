// ksched_pipe.hip -- the batched pipeline as ONE persistent kernel.
//
// k_pipe, 1 + G + M workgroups of 768 threads, one per CU (its LDS request excludes a second one), every
// workgroup resident for the whole call -- guaranteed by the launch itself: a cooperative launch of a
// grid that the occupancy query admits (nothing of the call runs beside it), so no protocol below
// assumes a dispatch order, a co-location or a second kernel.  Roles come from blockIdx:
//
//   workgroup 0          the COMMIT (all 12 waves): per active batch, wait for its B merges, replay the
//                        batch in pod order against the exact current state (commit_spc_batch), export
//                        the touched nodes, plan batch b + kPipeLag, publish Ctl::committed = b + 1.
//   workgroup 1 + g      SCORE (g < G, 12 waves): the rows j = g (mod G) of this rank's nodes live in LDS
//                        for the whole call; per batch wait for commit(b - kPipeLag), apply its export to
//                        the rows, score 64 pods x the rows (lane = pod; the screened scan), fold the wave
//                        lists to one top-KC list per pod, store it, arrive.
//   workgroup 1 + G + i  MERGE (kMS slots of kMT threads): slot id merges pods id, id + kMS M, ... of
//                        every batch: wait for the G arrivals, merge the G lists into the pod's K-entry
//                        Rec list [R > 1: exchange with the peer ranks + rank merge], count the merge.
//
// The merger slots of a workgroup run independent loops, so they never meet at s_barrier: each slot
// synchronises its own waves through an LDS counter (role_sync).  Every cross-workgroup hand-off is
// MI355X_MICROARCH "valid forms" row 1 (sc1 stores, every storing wave drained, one lane's counter
// update; sc1 loads after the poll) and every wait is bounded (PersistArgs::timeout_ticks -> error words
// 5..11).  Snapshot semantics (lag kPipeLag = 3): score(b) sees every commit up to b - 3, commit(b)
// inherits the nodes b - 2 and b - 1 committed (oracle/cpu_ref.c or_schedule_lagged at lag 3).
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "ksched_commit.h"
#include "ksched_merge.h"

#ifndef KSCHED_PIPE_PART
#define KSCHED_PIPE_PART 0
#endif

namespace ksched {

namespace {

constexpr int kSW = kPipeScoreWaves;  // score waves per score workgroup
constexpr int kMT = kPipeMergeThreads; // threads of one pod merge: one per score workgroup's list (G <= kMT)
constexpr int kMW = kMT / 64;          // waves of one pod merge
constexpr int kMS = kPipeMergeSlots;   // pod merges per merger workgroup
constexpr int kPU = 4;                 // rows per score step (independent key chains)
#ifndef KSCHED_XCHG_DEBUG
#define KSCHED_XCHG_DEBUG 0
#endif
constexpr int kSPU = 4;  // rows per step of the screened scan's passes
// The screened scan's exact phase over (row, pod) pairs: each pod's needed rows (at most kPairCap; ~4-8 on c4) and
// the batch's pairs (at most kPairMax) -- past either the batch takes the row path (every needed row for every pod)
constexpr int kPairCap = 48;
constexpr int kPairMax = 1024;

// ds_bpermute: lane `src`'s value of v (every lane of the wave must be active)
__device__ __forceinline__ int bperm(int v, int src) { return __builtin_amdgcn_ds_bpermute(src << 2, v); }
__device__ __forceinline__ int64_t bperm64(int64_t v, int src) {
    const uint32_t lo = (uint32_t)bperm((int)(uint32_t)(uint64_t)v, src);
    const uint32_t hi = (uint32_t)bperm((int)(uint32_t)((uint64_t)v >> 32), src);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
// inclusive prefix sum over the wave's lanes (Hillis-Steele; every lane active)
__device__ __forceinline__ int wave_incl_sum(int v) {
    const int lane = (int)__lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int t = bperm(v, lane >= d ? lane - d : 0);
        v += lane >= d ? t : 0;
    }
    return v;
}

// ---- barrier of ONE role's waves (LDS counter; s_barrier would wait for the other role too) ----------
__device__ __forceinline__ void role_sync(unsigned *ctr, unsigned &target, unsigned nwaves) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    target += nwaves;
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// per-workgroup control words (LDS offset 0 of a score workgroup)
struct alignas(16) PipeCtl {
    unsigned sbar, mbar;          // role barrier counters
    int32_t s_stop, m_stop;
    int64_t s_p0, s_done;         // score role: this batch's plan and the cursor after commit(b - kPipeLag)
    int64_t m_p0, m_done;         // merge role: the same, read by its own poll
    int32_t c_stop;               // commit workgroup
    int32_t s_ex;                 // score role: rows of this batch scored exactly (screened scan)
    int32_t s_scr;                // score role: this batch uses the screened scan
    int32_t s_pairs;              // score role: pairs scored exactly (pair lists), -1: the row path
    // score role: the next batch's loads and export apply, done by wave kSW - 1 during this batch's fold
    int32_t n_ok, n_err;          // n_ok: they were (commit(b + 1 - kPipeLag) was already published)
    int64_t n_p0, n_done;
};
constexpr size_t kPipeCtlBytes = 128;
static_assert(sizeof(PipeCtl) <= kPipeCtlBytes, "PipeCtl");

__device__ __forceinline__ bool spin_ge(const PersistArgs &P, int slot, const unsigned long long *p,
                                        unsigned long long v, unsigned long long *seen) {
    return poll_ge(p, v, P.timeout_ticks, &P.ctl->polls_rmw, seen, P.prog ? P.prog + kProgWords * slot + 2 : nullptr);
}

// the first failure names the wait that timed out (ksched_sync reports it)
__device__ __forceinline__ void set_err(int32_t *err, int32_t code) { atomicCAS(err, 0, code); }

// Cross-device granules: system-scope relaxed 8-byte accesses (global_store/load ... sc0 sc1) on the receive
// rings, the tag in both 32-bit halves (gran_enc): a granule is taken only when both halves are the writer's.
__device__ __forceinline__ void st_sys(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld_sys(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// poll one granule until both its halves carry `tag` (gran_dec; false: timed out)
__device__ __forceinline__ bool granule_wait(const uint64_t *p, uint32_t tag, int64_t limit, uint32_t *word) {
    const uint32_t t16 = gran_tag(tag);
    if (!gran_dec(ld_sys(p), t16, word)) {
        const uint64_t t0 = wall_clock64();
        do {
            if ((int64_t)(wall_clock64() - t0) > limit) return false;
            __builtin_amdgcn_s_sleep(1);
        } while (!gran_dec(ld_sys(p), t16, word));
    }
    return true;
}

// Rank merge of pod m's R exchanged lists (one wave, lane = source rank; the stream pipeline's
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
    const int32_t thr_bits = list_thr_bits(cut_out != 0, __ballot(lane < K && mi != kNoIdx), key_code(mk));
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
        r.pad = lane == 0 ? cut_out : (lane == 1 ? thr_bits : 0);  // entry 1: the screen threshold (list_thr_bits)
        store_rec<true>(out + lane, r);
    }
    if (lane == 0) store_i64<true>(out_fc, cnt);
}

__device__ __forceinline__ void set_row(NodeRec *nd, int64_t a0, int64_t a1, int64_t a2) {
    nd->a[0] = a0; nd->a[1] = a1; nd->a[2] = a2;
    const double f0 = (double)a0, f1 = (double)a1, f2 = (double)a2;
    nd->af[0] = f0; nd->af[1] = f1; nd->af[2] = f2;
    nd->y[0] = recip_or_zero(a0, f0); nd->y[1] = recip_or_zero(a1, f1); nd->y[2] = recip_or_zero(a2, f2);
    nd->ys[0] = screen_recip(a0); nd->ys[1] = screen_recip(a1); nd->ys[2] = screen_recip(a2);
}

// Pass 1's lower bounds of one step of kSPU rows into the wave's KC slots.  When kSPU is a multiple of KC,
// row u of the step goes to slot u % KC, which keeps the MAXIMUM of its rows (one v_max per pair instead of
// an insertion into a sorted list): the KC slots of a wave, and of the 12 waves, are lower bounds of keys of
// DISTINCT rows, so the KC-th largest of them is at most the KC-th largest key of the workgroup -- a valid
// L, at most slightly weaker than the KC-th largest of all the rows' bounds (tests/diag/screen_sim.py: c4 exact
// rows +4 %).  Otherwise a sorted top-KC insertion.
template <int KC, int SPU>
__device__ __forceinline__ void bound_slots(uint32_t (&t)[KC], const uint32_t (&xs)[SPU]) {
    if constexpr (SPU % KC == 0) {
#pragma unroll
        for (int u = 0; u < SPU; ++u) t[u % KC] = t[u % KC] > xs[u] ? t[u % KC] : xs[u];
    } else {
#pragma unroll
        for (int u = 0; u < SPU; ++u) {
            uint32_t xv = xs[u];
#pragma unroll
            for (int q = 0; q < KC; ++q) {
                const uint32_t hi = t[q] > xv ? t[q] : xv;
                xv = t[q] > xv ? xv : t[q];
                t[q] = hi;
            }
        }
    }
}

// descending order of KC values (once per batch, before the cross-wave merge)
template <int KC>
__device__ __forceinline__ void sort_desc_u32(uint32_t (&t)[KC]) {
#pragma unroll
    for (int i = 1; i < KC; ++i) {
#pragma unroll
        for (int j = i; j >= 1; --j) {
            const uint32_t a = t[j - 1], c = t[j];
            t[j - 1] = a > c ? a : c;
            t[j] = a > c ? c : a;
        }
    }
}

// t (sorted descending) <- the KC largest of t and u (both sorted descending): the element-wise max of t
// and reversed u holds them as a bitonic sequence, which half-cleaners sort
template <int KC>
__device__ __forceinline__ void topk_merge_u32(uint32_t (&t)[KC], const uint32_t (&u)[KC]) {
    uint32_t v[KC];
#pragma unroll
    for (int q = 0; q < KC; ++q) v[q] = t[q] > u[KC - 1 - q] ? t[q] : u[KC - 1 - q];
#pragma unroll
    for (int d = KC / 2; d >= 1; d >>= 1) {
#pragma unroll
        for (int i = 0; i < KC; ++i) {
            if ((i & d) == 0) {
                const uint32_t a = v[i], b = v[i + d];
                v[i] = a > b ? a : b;
                v[i + d] = a > b ? b : a;
            }
        }
    }
#pragma unroll
    for (int q = 0; q < KC; ++q) t[q] = v[q];
}

// One butterfly stage of the fold: this lane's sorted (key desc, idx asc) list and its DPP partner's (stage S
// of wpartner: lane ^ 1, lane ^ 2, mirror within 8 lanes) -> the top KC of both, sorted, identical in both
// lanes (bitonic: element-wise best of the list and the reversed partner list, then half-cleaners)
template <int S, int KC>
__device__ __forceinline__ void fold_stage(double (&k)[KC], int32_t (&ix)[KC]) {
    double ok[KC];
    int32_t oi[KC];
#pragma unroll
    for (int q = 0; q < KC; ++q) {
        ok[q] = wpartner_f64<S>(k[q]);
        oi[q] = (int32_t)wpartner<S>((uint32_t)ix[q]);
    }
    double vk[KC];
    int32_t vi[KC];
#pragma unroll
    for (int q = 0; q < KC; ++q) {
        const bool t = better(ok[KC - 1 - q], oi[KC - 1 - q], k[q], ix[q]);
        vk[q] = t ? ok[KC - 1 - q] : k[q];
        vi[q] = t ? oi[KC - 1 - q] : ix[q];
    }
#pragma unroll
    for (int d = KC / 2; d >= 1; d >>= 1) {
#pragma unroll
        for (int i = 0; i < KC; ++i) {
            if ((i & d) == 0) {
                const bool t = better(vk[i + d], vi[i + d], vk[i], vi[i]);
                const double a = vk[i], bb = vk[i + d];
                const int32_t ai = vi[i], bi = vi[i + d];
                vk[i] = t ? bb : a; vi[i] = t ? bi : ai;
                vk[i + d] = t ? a : bb; vi[i + d] = t ? ai : bi;
            }
        }
    }
#pragma unroll
    for (int q = 0; q < KC; ++q) { k[q] = vk[q]; ix[q] = vi[q]; }
}

// LDS layout of a score workgroup: PipeCtl | rows [R] | screen reciprocals [R] | fold lists | merge scratch |
// exchange messages | [screen records, when they fit]
template <int KC, int K>
struct ScoreLayout {
    static constexpr size_t fold_list_bytes = (size_t)kSW * KC * 64 * 12 + 64 * 4;  // every wave's lists + s_cnt
    // the screened scan's bound lists [kSW][KC][64] u32, queue counts [kSW] and row queue [kSW][ceil(R / kSW)] u16
    __host__ __device__ static size_t fold_bytes(int R) {
        const size_t scr = (size_t)kSW * KC * 64 * 4 + kSW * 4 + (size_t)2 * kSW * ((R + kSW - 1) / kSW) * 2;
        return scr > fold_list_bytes ? scr : fold_list_bytes;
    }
    __host__ __device__ static size_t rows_off() { return kPipeCtlBytes; }
    __host__ __device__ static size_t fold_off(int R) { return kPipeCtlBytes + (size_t)R * sizeof(NodeRec); }
    __host__ __device__ static size_t total(int R) { return fold_off(R) + (fold_bytes(R) + 15) / 16 * 16; }
    // the screened scan (when it fits): its f32 reciprocals, one 16-byte record per row ...
    __host__ __device__ static size_t ysq_off(int R) { return total(R); }
    __host__ __device__ static size_t total_screen(int R) { return total(R) + (size_t)R * 16; }
    // ... and pass 1's per-pair records for pass 2: [kSW][ceil(R / kSW)][64] u16 (screen_rec)
    __host__ __device__ static size_t hrec_off(int R) { return total_screen(R); }
    // rows per wave, rounded up to pairs (pass 1 stores the records of two rows in one 32-bit word)
    __host__ __device__ static int hrec_qw(int R) { return ((R + kSW - 1) / kSW + 1) / 2 * 2; }
    __host__ __device__ static size_t hrec_bytes(int R) { return (size_t)kSW * hrec_qw(R) * 64 * 2; }
    __host__ __device__ static size_t total_with_hrec(int R) { return total_screen(R) + hrec_bytes(R); }
    // the pair lists (score_role's exact phase), inside the fold area after the screened scan's bound lists, queue
    // counts and row queues, in front of s_cnt: cnt[64] u32, nel[64] u32, key[kPairMax] f64, row[64][kPairCap] u16
    __host__ __device__ static size_t pair_off(int R) {
        const size_t QW = (size_t)(R + kSW - 1) / kSW;
        return ((size_t)kSW * KC * 64 * 4 + kSW * 4 + 4 * kSW * QW + 15) / 16 * 16;
    }
    static constexpr size_t pair_bytes = 64 * 4 * 2 + (size_t)kPairMax * 8 + (size_t)64 * kPairCap * 2;
    __host__ __device__ static bool pairs_fit(int R) { return pair_off(R) + pair_bytes <= (size_t)kSW * KC * 64 * 12; }
};
struct PairArea {
    uint32_t *cnt;  // [64] needed rows per pod (atomic; past kPairCap: the batch takes the row path)
    uint32_t *nel;  // [64] eligible keys per pod
    double *key;    // [kPairMax] the pairs' exact keys (-inf: no key), pod-major
    uint16_t *row;  // [64][kPairCap] the needed rows of each pod
};

// LDS of a merger workgroup: kMS slots of {control words | merge scratch | exchange messages}
struct alignas(16) MergeCtl {
    unsigned mbar;
    int32_t m_stop;
    int64_t m_p0, m_done;
    int32_t m_w, pad;             // mwait's outcome (0 held, 1 rescue pending, 2 timed out)
    unsigned long long m_q;       // the pending rescue request
};
template <int KC, int K>
struct MergeLayout {
    static constexpr size_t ctl_bytes = 64;
    static constexpr size_t merge_bytes = (sizeof(MergeSmem<KC, K, kMT>) + 15) / 16 * 16;
    static constexpr size_t msg_bytes = ((size_t)(1 + kMaxXchgRanks) * msg_words(K) * 4 + 15) / 16 * 16;
    static constexpr size_t slot_bytes = ctl_bytes + merge_bytes + msg_bytes;
    static constexpr size_t total = kMS * slot_bytes;
};
static_assert(sizeof(MergeCtl) <= 64, "MergeCtl");

// + kCanaryBytes between the control state and the commit's arrays (KSCHED_CANARY: checked every batch)
constexpr size_t kCanaryBytes = 128;
constexpr size_t commit_loc_bytes() { return (sizeof(PersistLocal) + 15) / 16 * 16 + kCanaryBytes; }
template <int K>
constexpr size_t commit_total_bytes() { return commit_loc_bytes() + spc_lds_bytes<K, kPipeThreads, true>(); }
static_assert(commit_total_bytes<16>() <= 160 * 1024, "the persistent commit's LDS (lag-3 slots)");
// (+ 256: the kernel's static LDS, placed in front of the dynamic block)
static_assert(commit_loc_bytes() + spc_small_bytes<16, kPipeThreads, true>() + 256 <= 65536,
              "the persistent commit's arrays in front of S reach LDS immediate offsets");

// ------------------------------------------------------------------------------------------------
// SCORE role (waves 0 .. kSW-1 of workgroup 1 + g)
// ------------------------------------------------------------------------------------------------
template <int KC, int K, int PRIO, int DOM, bool LAB, bool F53>
__device__ __forceinline__ void score_role(const PersistArgs &P, char *smem, const int g) {
    PipeCtl *pc = reinterpret_cast<PipeCtl *>(smem);
    const int R = P.rows_per_wg;
    NodeRec *rows = reinterpret_cast<NodeRec *>(smem + ScoreLayout<KC, K>::rows_off());
    char *fold = smem + ScoreLayout<KC, K>::fold_off(R);
    float4 *ysq = reinterpret_cast<float4 *>(smem + ScoreLayout<KC, K>::ysq_off(R));  // screen reciprocals, SoA rows
    uint16_t *hrec = reinterpret_cast<uint16_t *>(smem + ScoreLayout<KC, K>::hrec_off(R));  // [kSW][QW/2][64] u16 pairs (P.screen_h)
    int32_t *s_cnt = reinterpret_cast<int32_t *>(fold + (size_t)kSW * KC * 64 * 12);  // [64], after the fold lists
    PairArea pr;
    {
        char *pa = fold + ScoreLayout<KC, K>::pair_off(R);
        pr.cnt = reinterpret_cast<uint32_t *>(pa);
        pr.nel = pr.cnt + 64;
        pr.key = reinterpret_cast<double *>(pa + 512);
        pr.row = reinterpret_cast<uint16_t *>(pa + 512 + (size_t)kPairMax * 8);
    }
    constexpr int kST = kSW * 64;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int G = P.G;
    const int64_t n = P.n_local, NP = P.pods.p;
    Ctl *ctl = P.ctl;
    auto sync = [&]() { __syncthreads(); };  // a score workgroup has no other role: plain barriers
    // this workgroup's rows j = g + r * G, resident in LDS for the whole call
    for (int e = tid; e < R * 6; e += kST) {
        const int r = e / 6, piece = e % 6;
        const int64_t j = g + (int64_t)r * G;
        if (j < n) reinterpret_cast<int4 *>(rows + r)[piece] = reinterpret_cast<const int4 *>(P.nodes + j)[piece];
    }
    if (tid == 0) pc->n_ok = 0;
    sync();
    if (P.screen_ok) {
        for (int r = tid; r < R; r += kST) {  // the screen's f32 reciprocals, one 16-byte record per row
            const NodeRec &nd = rows[r];
            ysq[r] = make_float4(screen_recip(nd.a[0]), screen_recip(nd.a[1]), screen_recip(nd.a[2]), 0.0f);
        }
    }
    // (batch 0's first barrier orders these writes before any export apply or scan)
    const double y3 = recip(3.0);
    // The screened scan (resource priority with the FAST53 bound): a row is scored exactly only when, for
    // some pod of the batch, its f32 screen cannot prove the pair below the workgroup's KC-th best key;
    // each workgroup turns it off for a while when most of its rows need the exact score anyway
    constexpr bool kScreen = PRIO == kPrioResource && F53;
    // the exact phase over (row, pod) pairs (PairArea) when the lists fit the fold area; else every needed row is
    // scored for every pod (the row path)
    constexpr bool kPairs = kScreen;
    const bool pairs_ok = kPairs && !P.no_pairs && ScoreLayout<KC, K>::pairs_fit(R);
    constexpr int kScreenOffBatches = 16;
    constexpr bool kPrefetch = kSW > 8;  // wave kSW - 1 does not fold
    int64_t scr_off_until = 0;  // wave 0: batches before this one scan unscreened
    int64_t ex_rows = 0, scan_rows = 0;  // tid 0: rows scored exactly / rows scanned (progress words 4, 5)
    const int64_t Rvalid = (n - g + G - 1) / G;  // rows of this workgroup that hold a node
    int64_t nact = 0;
    int idle = 0;
    unsigned long long early_c = 0;  // wave 0 lane 0: Ctl::committed as read before the last fold
    unsigned long long pre_c = 0;    // wave kSW - 1 lane 0: the same, for the prefetch of the next batch
    // One wave's round of loads for batch bb -- lane 0: its plan, the cursor after commit(bb - kPipeLag), the
    // error word; every lane: that commit's export (count and entries, lane = entry) -- and the apply of the
    // exported nodes this workgroup owns to its LDS rows and their HBM rows (the mergers read a candidate's
    // state there, sc1).  The caller has seen commit(bb - kPipeLag) published (stop: it timed out instead).
    auto load_apply = [&](int64_t bb, int stop, int64_t *p0v, int64_t *donev, int *errv) {
        int nxv = 0;
        // entry chunks {tag, idx, cur0} {tag, cur1, cur2.lo} {tag, cur2.hi, -} (store_xrec's persistent layout)
        u32x4 x0 = {0u, 0u, 0u, 0u}, x1 = {0u, 0u, 0u, 0u}, x2 = {0u, 0u, 0u, 0u};
        const XBuf *xb =
            reinterpret_cast<const XBuf *>(P.xring + (size_t)((bb >= kPipeLag ? bb - kPipeLag : 0) % 4) * P.xbuf_bytes);
        if (lane == 0) {
            *p0v = (int64_t)ld_coh(&ctl->plan[bb % kPlanRing]);
            *donev = bb >= kPipeLag ? (int64_t)ld_coh(&ctl->cursor_at[(bb - kPipeLag) % kPlanRing]) : 0;
            // a failed peer (a wait timed out) ends the call for everyone
            *errv = __hip_atomic_load(P.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (bb >= kPipeLag && !stop) {
            // {count, batch tag} in one granule: an idle commit (plan -1) leaves its ring slot untouched,
            // so a slot still tagged with an older batch is an empty export (never a torn one)
            const uint64_t hdr = ld_coh(&xb->count);  // one address: one request for the wave
            nxv = (uint32_t)(hdr >> 32) == (uint32_t)(bb - kPipeLag) ? (int)(uint32_t)hdr : 0;
            if (lane < 2 * P.B) {                      // speculative: entries past the count are ignored
                const __amdgpu_buffer_rsrc_t rs = coh_rsrc(xb->e);  // uniform base, the lane's entry by offset
                const uint32_t o = (uint32_t)lane * kXRecPipe;
                x0 = ld_coh16(rs, o); x1 = ld_coh16(rs, o + 16); x2 = ld_coh16(rs, o + 32);
            }
        }
        auto apply = [&](const u32x4 &c0, const u32x4 &c1, const u32x4 &c2) {
            const int64_t j = (int64_t)(int32_t)c0.y - P.node_offset;  // local row
            if (j < 0 || j >= n || j % G != g) return;  // another rank's node, or another workgroup's
            const int64_t a0 = w64(c0.z, c0.w), a1 = w64(c1.y, c1.z), a2 = w64(c1.w, c2.y);
            set_row(rows + j / G, a0, a1, a2);
            if (P.screen_ok) ysq[j / G] = make_float4(screen_recip(a0), screen_recip(a1), screen_recip(a2), 0.0f);
            st_coh(&P.nodes[j].a[0], (uint64_t)a0);
            st_coh(&P.nodes[j].a[1], (uint64_t)a1);
            st_coh(&P.nodes[j].a[2], (uint64_t)a2);
        };
        if (lane < nxv) apply(x0, x1, x2);
        for (int e = 64 + lane; e < nxv; e += 64) {  // exports beyond 64 entries (B > 64 only)
            const __amdgpu_buffer_rsrc_t rs = coh_rsrc(xb->e);
            const uint32_t o = (uint32_t)e * kXRecPipe;
            apply(ld_coh16(rs, o), ld_coh16(rs, o + 16), ld_coh16(rs, o + 32));
        }
    };
    for (int64_t b = 0;; ++b) {
        // ---- wave 0: wait for commit(b - kPipeLag), then ONE round of loads and the export apply (load_apply),
        // before the barrier (the other waves never touch the export) -- unless wave kSW - 1 did both during
        // the previous batch's fold ----
        if (wave == 0) {
            if (kPrefetch && __builtin_amdgcn_readfirstlane(pc->n_ok)) {  // wave kSW - 1 did it during the last fold
                if (lane == 0) {
                    pc->s_p0 = pc->n_p0;
                    pc->s_done = pc->n_done;
                    pc->s_stop = pc->n_err != 0 ? 3 : 0;
                    pc->s_scr = kScreen && P.screen_ok && !P.no_screen && b >= scr_off_until;
                    pc->s_ex = 0;
                    pc->n_ok = 0;
                }
            } else {
                int stop = 0;
                jitter_at(P.jitter, b, 1);  // the score workgroup's wait and loads
                if (lane == 0) {
                    unsigned long long seen = 0;
                    const unsigned long long need = (unsigned long long)(b - kPipeLag + 1);
                    // the count read before the previous batch's fold (early_c) usually suffices: no wait, and no
                    // progress store ahead of this round of loads
                    if (b >= kPipeLag && early_c < need) {
                        prog_at(P, g, b, kProgWaitCommit, 0);
                        if (!spin_ge(P, g, &ctl->committed_x[g % kCtlReplicas].v, need, &seen)) {
                            set_err(P.err, 6);
                            prog_at(P, g, b, kProgWaitCommit | kProgTimedOut, seen);
                            stop = 2;
                        }
                    }
                    if (g == 0) trace_at(P, b, 6);
                }
                stop = __builtin_amdgcn_readfirstlane(stop);
                int64_t p0v = 0, donev = 0;
                int errv = 0;
                load_apply(b, stop, &p0v, &donev, &errv);
                if (lane == 0) {
                    pc->s_p0 = p0v;
                    pc->s_done = donev;
                    pc->s_stop = errv != 0 ? 3 : stop;
                    pc->s_scr = kScreen && P.screen_ok && !P.no_screen && b >= scr_off_until;
                    pc->s_ex = 0;
                }
            }
        }
        sync();
        // the prefetch's node-row stores are complete before this batch's arrival (the mergers read them)
        if (kPrefetch && wave == kSW - 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (pc->s_stop) return;
        const int64_t p0 = pc->s_p0;
        if (pc->s_done >= NP) break;  // every pod resolved by commit(b - kPipeLag) or earlier
        if (p0 < 0 || p0 >= NP) {     // nothing planned for batch b (identical on every workgroup)
            if (tid == 0) prog_at(P, g, b, kProgIdle, (uint64_t)p0);
            // a truncation re-plans within kPipeLag batches; a longer run of empty plans is a protocol error
            if (++idle > kPlanRing) {
                if (tid == 0) set_err(P.err, 8);
                return;
            }
            sync();  // every wave has read s_done before wave 0 rewrites it
            continue;
        }
        idle = 0;
        ++nact;
        if (tid == 0) {
            if (g == 0) trace_at(P, b, 0);
            prog_at(P, g, b, kProgScan, 0);
        }
        const uint64_t t_go = ((P.trace || P.trace_wg) && tid == 0) ? wall_clock64() : 0;
        // ---- score: lane = pod, wave w scans rows r = w, w + W, ... (nodes j = g + r G) ----
        if (tid < 64) s_cnt[tid] = 0;
        if (kPairs && tid < 64) { pr.cnt[tid] = 0; pr.nel[tid] = 0; }
        bool pairs = false;          // this batch's exact phase runs over the pair lists
        int pT = 0, pincl = 0, pexcl = 0;  // ... pairs in all, and lane (pod) p's range [pexcl, pincl)
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
        const bool scr = kScreen && pc->s_scr;  // workgroup-uniform
        if (scr) {
            // Bounds travel shifted by +1 as f32 bit patterns: every one is then 0 ("none") or a positive
            // float, whose bits order as unsigned integers (max/min without NaN canonicalisation).
            const float qc = screen_req(rc), qm = screen_req(rm), qp = screen_req(rp);
            const int Rv = (int)((n - g + G - 1) / G);  // rows of this workgroup that hold a node
            const int QW = (R + kSW - 1) / kSW;
            const bool keep_h = P.screen_h != 0;      // pass 1 leaves a record per pair for pass 2
            // the records of a wave's rows k (r = wave + k kSW): rows 2i and 2i + 1 share a 32-bit word per lane
            uint32_t *hw = reinterpret_cast<uint32_t *>(hrec) + (size_t)wave * (ScoreLayout<KC, K>::hrec_qw(R) / 2) * 64 + lane;
            // One row for every pod of the batch: the f32 fractions decide the predicate unless one lies
            // within 2^-20 of 1 or is NaN (then the int64 compares of the row decide, for every pod); the
            // screen value, whether it bounds an eligible key from below, and whether the pair has a key.
            auto row_screen = [&](int r, const float4 &y, bool valid, bool *f, bool *el, bool *lo_ok) {
                const float c = qc * y.x, m = qm * y.y, p = qp * y.z;
                bool okc = c < kFracLo, okm = m < kFracLo, okp = p < kFracLo;
                const bool amb = !(okc || c > kFracHi) || !(okm || m > kFracHi) || !(okp || p > kFracHi);
                uint64_t lab = 0;
                if (__ballot(valid && amb)) {  // wave-uniform, rare
                    const NodeRec &nd = rows[r];
                    okc = nd.a[0] >= rc; okm = nd.a[1] >= rm; okp = nd.a[2] >= rp;
                }
                if (LAB) lab = rows[r].labels;
                *f = okc & okm & okp & (!LAB || (lab & sel) == sel);
                *el = DOM == kDomAll || *f;
                return screen_q(c, m, p, okc, okm, okp, lo_ok);
            };
            // ---- pass 1: every row -- the predicate count, the KC largest lower bounds of this pod's eligible
            // keys, and (keep_h) the pair's upper bound as a 16-bit record for pass 2 ----
            uint32_t t[KC];
#pragma unroll
            for (int q = 0; q < KC; ++q) t[q] = 0u;
            uint32_t *sl = reinterpret_cast<uint32_t *>(fold);  // [kSW][KC][64] (the fold area is free until
            int32_t *qcnt = reinterpret_cast<int32_t *>(sl + kSW * KC * 64);  // [kSW]      the scan ends)
            uint16_t *qrow = reinterpret_cast<uint16_t *>(qcnt + kSW);         // [kSW][QW] rows for the exact phase
            uint16_t *arow = qrow + kSW * QW;                                  // [kSW][QW] rows with an ambiguous fraction
            int na = 0;
            if (keep_h) {
                // branch-free: a pair whose fraction is ambiguous (within 2^-20 of 1, or NaN) contributes no
                // bound, gets a NaN record (scored exactly if it can matter) and its predicate is counted
                // exactly after the loop, from its row's int64 values
                static_assert(kSPU % 2 == 0, "pass 1 stores the records of row pairs");
                for (int r0 = wave; r0 < Rv; r0 += kSW * kSPU) {
                    float4 yv[kSPU];
                    uint64_t lb[kSPU];
#pragma unroll
                    for (int u = 0; u < kSPU; ++u) {
                        const int r = r0 + u * kSW;
                        yv[u] = ysq[r < Rv ? r : r0];
                        lb[u] = LAB ? rows[r < Rv ? r : r0].labels : 0ull;
                    }
                    uint32_t xs[kSPU];
                    uint32_t hh[kSPU];
                    uint32_t ambm = 0;  // rows of this group with an ambiguous fraction for this lane's pod
                    float ww[kSPU];     // the record's w before its conversion: base - v (screen_rec / screen_rec_nf)
                    uint32_t nrm[kSPU]; // 0: the record is hh; 1: a resource-fitting record; 0x8000 | 1: non-fitting
#pragma unroll
                    for (int u = 0; u < kSPU; ++u) {
                        const int r = r0 + u * kSW;
                        const bool valid = r < Rv;
                        const ScreenV sv = screen_fast(qc * yv[u].x, qm * yv[u].y, qp * yv[u].z);
                        const float v = sv.v;
                        const bool amb = sv.amb, rf = sv.rf;
                        const bool f = rf && (!LAB || (lb[u] & sel) == sel);
                        const bool el = DOM == kDomAll || f;
                        // a lower bound only where the key is surely there: a resource-fitting pair whose largest fraction
                        // is below 0.999 (its balanced part cannot vanish), or a non-fitting one; and v > eps
                        const bool lo_ok = !(rf && sv.mx >= 0.999f) && v > kScreenEps;
                        cnt += (valid && f && !amb) ? 1 : 0;
                        xs[u] = (valid && active && el && lo_ok && !amb) ? __float_as_uint(v + (1.0f - kScreenEps)) : 0u;
                        // the pair's upper bound (screen_rec / screen_rec_nf by the screen's form): 0 (always needed)
                        // when ambiguous, 0xffff (never needed) without a key
                        ww[u] = __builtin_fmaxf((rf ? 10.0f : kNfBase) - v, 0.0f);
                        nrm[u] = (!amb && el) ? (rf ? 1u : 0x8001u) : 0u;
                        hh[u] = amb ? 0u : 0xffffu;
                        ambm |= (valid && amb) ? 1u << u : 0u;
                    }
                    // the records of rows k, k + 1 (k = (r0 - wave) / kSW + u, u even) in one store; a pair's second
                    // row past the wave's last is never read
#pragma unroll
                    for (int u = 0; u < kSPU; u += 2) {
                        // both rows' records in one conversion: round toward zero IS the records' round-down for w >= 0
                        const uint32_t rec = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(ww[u], ww[u + 1]));
                        const uint32_t w2 = (nrm[u] ? ((rec & 0xffffu) | (nrm[u] & 0x8000u)) : hh[u]) |
                                            ((nrm[u + 1] ? ((rec >> 16) | (nrm[u + 1] & 0x8000u)) : hh[u + 1]) << 16);
                        if (r0 + u * kSW < Rv) hw[(size_t)(((r0 - wave) / kSW + u) / 2) * 64] = w2;
                    }
                    if (__ballot(ambm != 0)) {  // wave-uniform, rare: queue the rows with an ambiguous pair
#pragma unroll
                        for (int u = 0; u < kSPU; ++u) {
                            const bool anya = __ballot((ambm >> u) & 1u) != 0;
                            if (lane == 0 && na < QW) arow[wave * QW + na] = (uint16_t)(r0 + u * kSW);  // kept when anya
                            na += anya ? 1 : 0;
                        }
                    }
                    bound_slots<KC>(t, xs);
                }
                // the ambiguous pairs' predicate, exactly
                for (int e = 0; e < na; ++e) {
                    const int r = arow[wave * QW + e];
                    const NodeRec &nd = rows[r];
                    const float4 y = ysq[r];
                    const float c = qc * y.x, m = qm * y.y, p = qp * y.z;
                    const bool amb = !(c < kFracLo || c > kFracHi) || !(m < kFracLo || m > kFracHi) ||
                                     !(p < kFracLo || p > kFracHi);
                    cnt += (amb && fits(rc, rm, rp, sel, nd.a[0], nd.a[1], nd.a[2], nd.labels, LAB)) ? 1 : 0;
                }
            } else {
                for (int r0 = wave; r0 < Rv; r0 += kSW * kSPU) {
                    float4 yv[kSPU];
#pragma unroll
                    for (int u = 0; u < kSPU; ++u) {
                        const int r = r0 + u * kSW;
                        yv[u] = ysq[r < Rv ? r : r0];
                    }
                    uint32_t xs[kSPU];
#pragma unroll
                    for (int u = 0; u < kSPU; ++u) {
                        const int r = r0 + u * kSW;
                        const bool valid = r < Rv;
                        bool f, el, lo_ok;
                        const float v = row_screen(valid ? r : r0, yv[u], valid, &f, &el, &lo_ok);
                        cnt += (valid && f) ? 1 : 0;
                        xs[u] = (valid && active && el && lo_ok) ? __float_as_uint(v + (1.0f - kScreenEps)) : 0u;
                    }
                    bound_slots<KC>(t, xs);
                }
            }
            if (g == 0 && tid == 0) trace_at(P, b, 11);
            // ---- the workgroup's bound: the KC-th largest lower bound over every wave's list (the fold
            // area is free until the scan ends) ----
            sort_desc_u32<KC>(t);
#pragma unroll
            for (int q = 0; q < KC; ++q) sl[(wave * KC + q) * 64 + lane] = t[q];
            sync();
            for (int w = 1; w < kSW; ++w) {
                const int ow = (wave + w) % kSW;
                uint32_t u[KC];
#pragma unroll
                for (int q = 0; q < KC; ++q) u[q] = sl[(ow * KC + q) * 64 + lane];
                topk_merge_u32<KC>(t, u);
            }
            const float L = __uint_as_float(t[KC - 1]);  // + 1; 0 = fewer than KC bounds: everything passes
            if (g == 0 && tid == 0) trace_at(P, b, 12);
            // the predicate counts (s_cnt was zeroed before pass 1, and that write is ordered by the barrier above)
            if (cnt) atomicAdd(&s_cnt[lane], cnt);
            // ---- pass 2: a row needs its exact scores when some pod's upper bound reaches L (a pair below
            // L is below KC eligible keys of this workgroup, so it is in no top-KC list the exact scan would
            // have produced); the wave queues such rows, and (pair lists) each needed (row, pod) pair in its
            // pod's list ----
            int qn = 0;
            // pod `lane` needs row r: one slot of its pair list (a count past kPairCap sends the batch to the row path)
            auto add_pair = [&](bool need, int r) {
                if (kPairs && need) {
                    const uint32_t s = atomicAdd(&pr.cnt[lane], 1u);
                    if (s < (uint32_t)kPairCap) pr.row[lane * kPairCap + s] = (uint16_t)r;
                }
            };
            if (keep_h) {
                const int nr = (Rv - wave + kSW - 1) / kSW;  // this wave's rows
                // in the records' own units: the pair is needed when its bound + 1 + eps reaches L; -1: an
                // inactive lane
                const int tq = active ? screen_rec_threshold(L) : -1;
                const int tqn = active ? screen_rec_threshold_nf(L) : -1;
                for (int i0 = 0; i0 < nr; i0 += 8) {
                    uint16_t hv[8];
#pragma unroll
                    for (int u = 0; u < 8; u += 2) {
                        const uint32_t x = hw[(size_t)((i0 + u < nr ? i0 + u : i0) / 2) * 64];
                        hv[u] = (uint16_t)x;
                        hv[u + 1] = (uint16_t)(x >> 16);
                    }
                    uint32_t grp = 0;   // wave-uniform: the group's rows some pod needs
                    uint32_t mine = 0;  // ... and the ones this lane's pod needs
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const bool nd = screen_rec_needed(hv[u], tq, tqn);
                        const uint64_t bm = __builtin_amdgcn_ballot_w64(nd);
                        grp |= (bm != 0 ? 1u : 0u) << u;
                        mine |= (nd ? 1u : 0u) << u;
                    }
                    if (nr - i0 < 8) grp &= (1u << (nr - i0)) - 1u;  // rows past the wave's last
                    // lanes 0..7 queue the group's needed rows in order, one store (a wave's rows fit its QW)
                    if (lane < 8 && ((grp >> lane) & 1u))
                        qrow[wave * QW + qn + __builtin_popcount(grp & ((1u << lane) - 1u))] =
                            (uint16_t)(wave + (i0 + lane) * kSW);
                    qn += __builtin_popcount(grp);
                    if (kPairs && grp) {  // one slot reservation per lane for the group's needed rows
                        uint32_t mm = mine & grp;
                        const int c = __builtin_popcount(mm);
                        uint32_t s = c ? atomicAdd(&pr.cnt[lane], (uint32_t)c) : 0u;
                        for (; mm; mm &= mm - 1u, ++s)
                            if (s < (uint32_t)kPairCap)
                                pr.row[lane * kPairCap + s] = (uint16_t)(wave + (i0 + __builtin_ctz(mm)) * kSW);
                    }
                }
            } else {
                for (int r0 = wave; r0 < Rv; r0 += kSW * kSPU) {
                    float4 yv[kSPU];
#pragma unroll
                    for (int u = 0; u < kSPU; ++u) {
                        const int r = r0 + u * kSW;
                        yv[u] = ysq[r < Rv ? r : r0];
                    }
#pragma unroll
                    for (int u = 0; u < kSPU; ++u) {
                        const int r = r0 + u * kSW;
                        const bool valid = r < Rv;
                        bool f, el, lo_ok;
                        const float v = row_screen(valid ? r : r0, yv[u], valid, &f, &el, &lo_ok);
                        const bool need = valid && active && el && !(v + (1.0f + kScreenEps) < L);  // NaN: needed
                        const bool any = __ballot(need) != 0;
                        if (lane == 0 && qn < QW) qrow[wave * QW + qn] = (uint16_t)r;  // kept when any
                        qn += any ? 1 : 0;
                        if (any) add_pair(need, r);
                    }
                }
            }
            if (lane == 0) qcnt[wave] = qn;
            if (g == 0 && tid == 0) trace_at(P, b, 14);
            sync();
            int base[kSW], tot = 0;
#pragma unroll
            for (int w = 0; w < kSW; ++w) { base[w] = tot; tot += qcnt[w]; }
            // ---- the pair lists (every wave computes the same prefix over the pods' counts, lane = pod): when
            // none overflowed, thread e scores the e-th needed (row, pod) pair exactly -- ~4-8 pairs per pod
            // instead of every pod against every needed row ----
            if (kPairs) {
                const int c = (int)pr.cnt[lane];
                pincl = wave_incl_sum(c);
                pexcl = pincl - c;
                pT = __builtin_amdgcn_readlane(pincl, 63);
                pairs = pairs_ok && __ballot(c > kPairCap) == 0 && pT <= kPairMax;  // workgroup-uniform
            }
            if (pairs) {
                for (int e0 = wave * 64; e0 < pT; e0 += kST) {  // wave-uniform trip count: every lane shuffles
                    const int e = e0 + lane;
                    const int ec = e < pT ? e : pT - 1;
                    int p = 0;  // the pod: how many lanes' inclusive counts are <= e
#pragma unroll
                    for (int st = 32; st; st >>= 1) p += bperm(pincl, p + st - 1) <= ec ? st : 0;
                    const int s = ec - bperm(pexcl, p);
                    const int64_t qc = bperm64(rc, p), qm = bperm64(rm, p), qp = bperm64(rp, p);
                    const uint64_t qs = LAB ? (uint64_t)bperm64((int64_t)sel, p) : 0ull;
                    if (e < pT) {
                        const int r = pr.row[p * kPairCap + s];
                        const NodeRec &nd = rows[r];
                        const int64_t ac = nd.a[0], am = nd.a[1], ap = nd.a[2];
                        const bool f = fits(qc, qm, qp, qs, ac, am, ap, nd.labels, LAB);
                        double k;
                        const bool el = pair_key_fast<PRIO, DOM, F53>(f, qc, qm, qp, (double)qc, (double)qm, (double)qp, ac,
                                                                      am, ap, nd.af[0], nd.af[1], nd.af[2], nd.y[0],
                                                                      nd.y[1], nd.y[2], y3, nd.price, &k);
                        pr.key[e] = el ? k : -__builtin_inf();
                        if (el) atomicAdd(&pr.nel[p], 1u);
                    }
                }
            } else
            // ---- the queued rows, dealt round-robin to the waves (balanced), scored exactly for every pod;
            // arrival order is not node order, so the insert ranks ties by node index ----
            for (int e = wave; e < tot; e += kSW) {
                int w = 0;
#pragma unroll
                for (int v = 1; v < kSW; ++v) w += e >= base[v] ? 1 : 0;
                const int r = qrow[w * QW + (e - base[w])];
                const NodeRec &nd = rows[r];
                const int64_t ac = nd.a[0], am = nd.a[1], ap = nd.a[2];
                const bool f = fits(rc, rm, rp, sel, ac, am, ap, nd.labels, LAB);
                double k;
                const bool el = pair_key_fast<PRIO, DOM, F53>(f, rc, rm, rp, rcf, rmf, rpf, ac, am, ap, nd.af[0], nd.af[1],
                                                              nd.af[2], nd.y[0], nd.y[1], nd.y[2], y3, nd.price, &k);
                if (el) list_insert_ordered<KC>(key, idx, k, (int32_t)(P.node_offset + g + (int64_t)r * G));
            }
            if (wave == 0 && lane == 0) { pc->s_ex = tot; pc->s_pairs = pairs ? pT : -1; }
        } else
        // kPU rows per step: their keys are independent f64 chains the scheduler interleaves; inserted
        // in ascending node order afterwards
        for (int r0 = wave; r0 < R; r0 += kSW * kPU) {
            double ks[kPU];
#pragma unroll
            for (int u = 0; u < kPU; ++u) {
                const int r = r0 + u * kSW;
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
                int32_t ci = (int32_t)(P.node_offset + g + (int64_t)(r0 + u * kSW) * G);  // global index
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
        const uint64_t t_scan = (P.trace && tid == 0) ? wall_clock64() : 0;
        // the commit count for the next batch's wait, read now: its latency hides behind the fold and stores
        if (tid == 0) early_c = __hip_atomic_load(&ctl->committed_x[g % kCtlReplicas].v, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
        if (kPrefetch && wave == kSW - 1 && lane == 0)
            pre_c = __hip_atomic_load(&ctl->committed_x[g % kCtlReplicas].v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sync();  // every wave's scan is done (the fold area is free); s_cnt was zeroed
        if (g == 0 && tid == 0) trace_at(P, b, 9);
        // ---- the next batch's loads and export apply by wave kSW - 1, while the others fold (or rank the pairs): a
        // workgroup still busy with this batch when commit(b + 1 - kPipeLag) is published starts the next scan right
        // after its arrival.  Only when that commit is already out: this wave never waits for it ----
        auto prefetch_next = [&]() {
            const unsigned long long need = (unsigned long long)(b + 1 - kPipeLag + 1);
            int ok = 0;
            if (lane == 0) {
                ok = b + 1 < kPipeLag || pre_c >= need;
                if (!ok) ok = __hip_atomic_load(&ctl->committed_x[g % kCtlReplicas].v, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT) >= need;
            }
            ok = __builtin_amdgcn_readfirstlane(ok);
            if (ok) {
                if (g == 0 && lane == 0) trace_at(P, b + 1, 6);
                int64_t p0v = 0, donev = 0;
                int errv = 0;
                load_apply(b + 1, 0, &p0v, &donev, &errv);
                if (lane == 0) { pc->n_p0 = p0v; pc->n_done = donev; pc->n_err = errv; }
            }
            if (lane == 0) pc->n_ok = ok;
        };
        const size_t part_elems = (size_t)P.B * G;
        Cand *part = P.part + (size_t)(b % kPipeLag) * part_elems * KC;  // merge(b) is done before score(b + kPipeLag)
        // entry q of pod pl's list as one 16-B record {key, idx, pad}, entry 0's pad carrying the workgroup's predicate
        // count for the pod; word 3: the batch's tag (bits 16..31) and, in entry 0, the count (< 2^16 rows per workgroup)
        auto store_entry = [&](int pl, int q, double kk, int32_t ii) {
            const uint64_t kb = (uint64_t)__double_as_longlong(kk);
            const uint32_t tag = (uint32_t)((b + 1) & 0xffff) << 16;
            const u32x4 v = {(uint32_t)kb, (uint32_t)(kb >> 32), (uint32_t)ii, tag | (q == 0 ? (uint32_t)s_cnt[pl] : 0u)};
            st_coh16(coh_rsrc(part), (uint32_t)((((size_t)pl * G + g) * KC + q) * sizeof(Cand)), v);
        };
        if (pairs) {
            // ---- pair lists: each scored pair's rank among its pod's pairs (key desc, node index asc -- rows are in
            // node order within the workgroup) is its slot; the KC best are stored, wave 0 fills the empty slots ----
            if (kPrefetch && wave == kSW - 1) {
                prefetch_next();
            } else {
                constexpr int RW = kPrefetch ? kSW - 1 : kSW;  // the ranking waves
                for (int e0 = wave * 64; e0 < pT; e0 += RW * 64) {  // wave-uniform trip count: every lane shuffles
                    const int e = e0 + lane;
                    const int ec = e < pT ? e : pT - 1;
                    int p = 0;
#pragma unroll
                    for (int st = 32; st; st >>= 1) p += bperm(pincl, p + st - 1) <= ec ? st : 0;
                    const int ex = bperm(pexcl, p), in = bperm(pincl, p);
                    if (e < pT) {
                        const double k = pr.key[e];
                        if (k != -__builtin_inf()) {
                            const uint16_t *prow = pr.row + p * kPairCap;
                            const int r = prow[e - ex];
                            int rank = 0;
                            int e2 = ex;
                            for (; e2 + 4 <= in; e2 += 4) {  // four loads in flight
                                double k2[4];
                                int r2[4];
#pragma unroll
                                for (int u = 0; u < 4; ++u) { k2[u] = pr.key[e2 + u]; r2[u] = prow[e2 + u - ex]; }
#pragma unroll
                                for (int u = 0; u < 4; ++u) rank += (k2[u] > k || (k2[u] == k && r2[u] < r)) ? 1 : 0;
                            }
                            for (; e2 < in; ++e2) {
                                const double k2 = pr.key[e2];
                                const int r2 = prow[e2 - ex];
                                rank += (k2 > k || (k2 == k && r2 < r)) ? 1 : 0;
                            }
                            if (rank < KC && p < P.B && p0 + p < NP)
                                store_entry(p, rank, k, (int32_t)(P.node_offset + g + (int64_t)r * G));
                        }
                    }
                }
                if (wave == 0 && lane < P.B && p0 + lane < NP) {
                    for (int q = (int)pr.nel[lane]; q < KC; ++q) store_entry(lane, q, -__builtin_inf(), kNoIdx);
                }
            }
            if (g == 0 && tid == 0) trace_at(P, b, 10);
            // Wave 0's export apply (the node rows the mergers read for the candidates' state) complete before the
            // arrival, independent of what follows
            if (wave == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
        if (!scr && cnt) atomicAdd(&s_cnt[lane], cnt);  // (screened batches counted after pass 1)
        // ---- fold: every wave's lists to LDS; then wave w merges pods 8w .. 8w+7 for all 8 source waves at
        // once (lane = pod x source wave; three 8-lane butterfly merges of sorted lists) and stores them.  A
        // list that is cut when full folds into the top-KC of the union, again cut when full.
        double *fk = reinterpret_cast<double *>(fold);                                  // [kSW][KC][64]
        int32_t *fi = reinterpret_cast<int32_t *>(fold + (size_t)kSW * KC * 64 * 8);    // [kSW][KC][64]
#pragma unroll
        for (int q = 0; q < KC; ++q) {
            fk[(wave * KC + q) * 64 + lane] = key[q];
            fi[(wave * KC + q) * 64 + lane] = idx[q];
        }
        sync();
        static_assert(kSW >= 8 && kSW <= 16, "the fold deals 8 pods to each of the first 8 waves");
        const int pl = wave * 8 + (lane >> 3);  // this lane's pod of the batch (waves 0..7)
        const int src = lane & 7;               // ... and source wave (plus src + 8 when that exists)
        const bool folds = wave < 8;
        if (kPrefetch && wave == kSW - 1) prefetch_next();
        if (folds) {
#pragma unroll
            for (int q = 0; q < KC; ++q) {
                key[q] = fk[(src * KC + q) * 64 + pl];
                idx[q] = fi[(src * KC + q) * 64 + pl];
            }
            if (src + 8 < kSW) {
#pragma unroll
                for (int q = 0; q < KC; ++q) {
                    const int32_t oi = fi[((src + 8) * KC + q) * 64 + pl];
                    if (oi == kNoIdx) break;
                    list_insert_ordered<KC>(key, idx, fk[((src + 8) * KC + q) * 64 + pl], oi);
                }
            }
            fold_stage<0, KC>(key, idx);
            fold_stage<1, KC>(key, idx);
            fold_stage<2, KC>(key, idx);
        }
        if (g == 0 && tid == 0) trace_at(P, b, 10);
        // Wave 0's export apply (the node rows the mergers read for the candidates' state) complete before the
        // arrival: drained here, a whole scan after it was issued (free by now), independent of what follows
        if (wave == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (folds && pl < P.B && p0 + pl < NP && src < KC) {
            // every lane of the group holds the pod's list: lane src stores entry src
            double kk = key[0];
            int32_t ii = idx[0];
#pragma unroll
            for (int q = 1; q < KC; ++q) {
                kk = src == q ? key[q] : kk;
                ii = src == q ? idx[q] : ii;
            }
            store_entry(pl, src, kk, ii);
        }
        }
        // The records need no drain (the mergers read them again until their tags are this batch's)
        sync();  // every wave's record stores issued
        if (wave == 0) {
            // most rows needed the exact score: the screen only costs here -- scan unscreened for a while
            if (scr && 2 * pc->s_ex > R) scr_off_until = b + 1 + kScreenOffBatches;
            if (scr && g == 0 && lane == 0 && P.trace && b < P.trace_cap)  // rows | pairs << 32 (0xffffffff: row path)
                P.trace[b * kTraceCols + 13] = (uint64_t)(uint32_t)pc->s_ex | (uint64_t)(uint32_t)pc->s_pairs << 32;
            if (lane == 0) { ex_rows += scr ? pc->s_ex : Rvalid; scan_rows += Rvalid; }
            // ---- arrive (the merge waves of workgroups 1 .. B wait for all G) ----
            jitter_at(P.jitter, b, 2);
            const int slot = (int)((nact - 1) % 4);
            if (lane == 0) {
                if (g == 0) trace_at(P, b, 5);
                const unsigned long long old = __hip_atomic_fetch_add(&ctl->arrive[slot].v, 1ull, __ATOMIC_RELAXED,
                                                                      __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long use = (unsigned long long)((nact - 1) / 4);
                if (old + 1 == (use + 1) * (unsigned long long)G) trace_at(P, b, 1);
                prog_at(P, g, b, kProgArrived, old + 1);
                if (P.trace) prog_add(P, g, t_scan - t_go, wall_clock64() - t_go);
                if (P.trace_wg && b < P.trace_cap)
                    P.trace_wg[b * G + g] = (t_go & 0xffffffffull) | (wall_clock64() << 32);
            }
        }
        // the next batch's first barrier orders s_cnt / fold reuse after wave 0's reads
    }
    if (tid == 0 && P.prog) { P.prog[kProgWords * g + 4] = (uint64_t)ex_rows; P.prog[kProgWords * g + 5] = (uint64_t)scan_rows; }
    // every pod is resolved: this workgroup's rows go back to HBM whole (allocatable, cached doubles,
    // reciprocals) for the next call and for ksched_read_nodes
    for (int e = tid; e < R * 6; e += kST) {
        const int r = e / 6, piece = e % 6;
        const int64_t j = g + (int64_t)r * G;
        if (j < n) reinterpret_cast<int4 *>(P.nodes + j)[piece] = reinterpret_cast<const int4 *>(rows + r)[piece];
    }
}

// ------------------------------------------------------------------------------------------------
// The rescue of an exhausted candidate list, merger side (commit side: commit_rescue, ksched_commit.h)
// ------------------------------------------------------------------------------------------------
// mtid 0 of a merger slot: wait for *p >= v like poll_ge, serving rescues meanwhile.  0: it holds; 1: a
// rescue request newer than `served` is pending (*q); 2: timed out (*seen = the last value read).
__device__ __forceinline__ int poll_ge_or_rescue(const PersistArgs &P, int slot, const unsigned long long *p,
                                                 unsigned long long v, unsigned long long served,
                                                 unsigned long long *q, unsigned long long *seen) {
    const unsigned long long *rq = &P.ctl->rescue_req.v;
    const bool resc = P.rescue != nullptr;
    unsigned long long x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (x >= v) { *seen = x; return 0; }
    const uint64_t t0 = wall_clock64();
    for (int it = 1;; ++it) {
        if (resc) {
            const unsigned long long r = (it & 1023) == 0 ? (unsigned long long)ld_rmw(rq)
                                                          : __hip_atomic_load(rq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (r > served) { *q = r; *seen = x; return 1; }
        }
        __builtin_amdgcn_s_sleep(1);
        if ((it & 1023) == 0) {
            if (P.prog) __hip_atomic_store(P.prog + kProgWords * slot + 2, (uint64_t)it, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            x = (unsigned long long)ld_rmw(p);
            if (x >= v) {
                __hip_atomic_fetch_add(&P.ctl->polls_rmw, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                *seen = x;
                return 0;
            }
            if ((int64_t)(wall_clock64() - t0) > P.timeout_ticks) { *seen = x; return 2; }
        } else {
            x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (x >= v) { *seen = x; return 0; }
        }
    }
}

// One rescue request, by every thread of merger slot `id` (< B): the slot's share of this rank's node rows,
// [id * chunk, (id + 1) * chunk), at their current state -- the HBM rows, read sc1 (a score workgroup's export
// apply writes them) -- except the nodes of the request's touched set T, which the commit evaluates itself.
// Nodes outside T are untouched since the batch's score snapshot (commit(b - 3)); every score workgroup
// applied that commit's export to HBM before the batch's merges completed, which the commit waited for.  The
// slot's best eligible (key desc, idx asc) goes to res[id] (sc1, drained) and is counted in Ctl::rescue_done.
// LDS: the slot's merge scratch, free between merges.  Restated by oracle/cpu_ref.c or_rescue.
template <int PRIO, int DOM, bool LAB, bool F53, typename Sync>
__device__ __forceinline__ void serve_rescue(const PersistArgs &P, int id, int mtid, char *scratch, Sync sync) {
    constexpr int kRH = 1024;  // open-addressed set of T's node indices (|T| <= kRescueMaxT)
    static_assert(kRH >= 2 * kRescueMaxT, "rescue set");
    const RescueReq *rq = reinterpret_cast<const RescueReq *>(P.rescue);
    int32_t *hs = reinterpret_cast<int32_t *>(scratch);
    double *wk = reinterpret_cast<double *>(scratch + kRH * 4);
    int32_t *wi = reinterpret_cast<int32_t *>(wk + kMW);
    const int64_t rc = (int64_t)ld_coh(&rq->rc), rm = (int64_t)ld_coh(&rq->rm), rp = (int64_t)ld_coh(&rq->rp);
    const uint64_t sel = LAB ? ld_coh(&rq->sel) : 0;
    const int nT = (int)ld_coh(&rq->nT);
    auto slot_of = [](int32_t x) { return (int)(((uint32_t)x * 2654435761u) >> 22); };  // log2(kRH) = 10
    for (int e = mtid; e < kRH; e += kMT) hs[e] = -1;
    sync();
    for (int t = mtid; t < nT; t += kMT) {
        const int32_t x = (int32_t)ld_coh(&rq->ti[t]);
        for (int h = slot_of(x);; h = (h + 1) & (kRH - 1)) {
            const int32_t prev = atomicCAS(&hs[h], -1, x);
            if (prev == -1 || prev == x) break;
        }
    }
    sync();
    const int64_t n = P.n_local;
    const int64_t chunk = (n + P.B - 1) / P.B;
    const int64_t lo = (int64_t)id * chunk, hi = lo + chunk < n ? lo + chunk : n;
    const double rcf = (double)rc, rmf = (double)rm, rpf = (double)rp, y3 = recip(3.0);
    double bk = -__builtin_inf();
    int32_t bi = kNoIdx;
    for (int64_t j = lo + mtid; j < hi; j += kMT) {
        const int32_t gj = (int32_t)(P.node_offset + j);
        bool in_t = false;
        for (int h = slot_of(gj);; h = (h + 1) & (kRH - 1)) {
            const int32_t x = hs[h];
            if (x == gj) { in_t = true; break; }
            if (x == -1) break;
        }
        if (in_t) continue;
        const NodeRec &nd = P.nodes[j];
        const int64_t a0 = (int64_t)ld_coh(&nd.a[0]), a1 = (int64_t)ld_coh(&nd.a[1]), a2 = (int64_t)ld_coh(&nd.a[2]);
        const uint64_t lab = LAB ? nd.labels : 0ull;  // labels and prices never change during a call
        const bool f = fits(rc, rm, rp, sel, a0, a1, a2, lab, LAB);
        const double f0 = (double)a0, f1 = (double)a1, f2 = (double)a2;
        double k;
        if (pair_key_fast<PRIO, DOM, F53>(f, rc, rm, rp, rcf, rmf, rpf, a0, a1, a2, f0, f1, f2, recip_or_zero(a0, f0),
                                          recip_or_zero(a1, f1), recip_or_zero(a2, f2), y3, nd.price, &k) &&
            better(k, gj, bk, bi)) {
            bk = k;
            bi = gj;
        }
    }
    int32_t aux = 0;
    wave_argbest(bk, bi, aux);
    if ((mtid & 63) == 0) { wk[mtid >> 6] = bk; wi[mtid >> 6] = bi; }
    sync();
    if (mtid == 0) {
        for (int w = 1; w < kMW; ++w)
            if (wi[w] != kNoIdx && better(wk[w], wi[w], bk, bi)) { bk = wk[w]; bi = wi[w]; }
        Rec r{};
        if (bi != kNoIdx) {
            const NodeRec &nd = P.nodes[bi - P.node_offset];
            r.key = bk; r.idx = bi; r.valid = 1;
            r.a[0] = (int64_t)ld_coh(&nd.a[0]); r.a[1] = (int64_t)ld_coh(&nd.a[1]); r.a[2] = (int64_t)ld_coh(&nd.a[2]);
            r.labels = nd.labels; r.price = nd.price;
        } else {
            r.key = -__builtin_inf(); r.idx = kNoIdx; r.valid = 0;
        }
        store_rec<true>(reinterpret_cast<Rec *>(P.rescue + kRescueResOff) + id, r);
        drain_stores();
        __hip_atomic_fetch_add(&P.ctl->rescue_done.v, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Pod m of batch b (p0 + m) against the nodes batch b - 2 committed (its export, ring slot (b - 2) % 4): the
// keys at their current state, the predicate deltas since b's snapshot and the best entry -- what commit(b)
// would otherwise compute for those inherited slots on its own critical path (commit_spc_batch, LAG3).  Wave 0
// of the merger slot, lane = export entry; commit(b - 2) is done (the caller waited).  The key column goes to
// inh keys[b % 4][m][0, n2), the summary to inh summary[b % 4][m]: {sum of deltas, best key, best idx | entry
// << 32} (entry -1: none eligible).  Restated by oracle/cpu_ref.c commit_inherit (the two exports' deltas add).
template <int PRIO, int DOM, bool LAB, bool F53>
__device__ __forceinline__ void inherit_x2_keys(const PersistArgs &P, int64_t b, int m, int64_t pod, int mtid) {
    if (mtid >= 64) return;
    const int lane = mtid;
    const XBuf *xb = reinterpret_cast<const XBuf *>(P.xring + (size_t)((b - 2) % 4) * P.xbuf_bytes);
    const uint64_t hdr = ld_coh(&xb->count);
    const int n2 = (uint32_t)(hdr >> 32) == (uint32_t)(b - 2) ? (int)(uint32_t)hdr : 0;
    const int64_t rc = P.pods.rc[pod], rm = P.pods.rm[pod], rp = P.pods.rp[pod];
    const uint64_t sel = LAB ? P.pods.sel[pod] : 0ull;
    double k = -__builtin_inf();
    int32_t ix = kNoIdx;
    int64_t d = 0;
    double *keys = reinterpret_cast<double *>(P.inh + (size_t)4 * P.B * 32) + ((size_t)(b % 4) * P.B + m) * 64;
    if (lane < n2) {
        const XRec x = load_xrec<true>(xb->e, lane);
        const bool f0 = fits(rc, rm, rp, sel, x.sb[0], x.sb[1], x.sb[2], x.labels, LAB);
        const bool f1 = fits(rc, rm, rp, sel, x.cur[0], x.cur[1], x.cur[2], x.labels, LAB);
        d = (int64_t)f1 - (int64_t)f0;
        const double c0 = (double)x.cur[0], c1 = (double)x.cur[1], c2 = (double)x.cur[2];
        double kk;
        if (pair_key_fast<PRIO, DOM, F53>(f1, rc, rm, rp, (double)rc, (double)rm, (double)rp, x.cur[0], x.cur[1],
                                          x.cur[2], c0, c1, c2, recip_or_zero(x.cur[0], c0), recip_or_zero(x.cur[1], c1),
                                          recip_or_zero(x.cur[2], c2), recip(3.0), x.price, &kk)) {
            k = kk;
            ix = x.idx;
        }
    }
    // pairs of keys as 16-byte sc1 stores (entries >= n2 are never read)
    const double kn = __shfl_down(k, 1);
    if (lane < n2 && (lane & 1) == 0)
        st_coh16(coh_rsrc(keys), (uint32_t)(8 * lane),
                 u32x4{(uint32_t)__double_as_longlong(k), (uint32_t)((uint64_t)__double_as_longlong(k) >> 32),
                       (uint32_t)__double_as_longlong(kn), (uint32_t)((uint64_t)__double_as_longlong(kn) >> 32)});
    d = wave_sum_i64(d);
    int32_t src = lane;
    wave_argbest(k, ix, src);
    if (lane == 0) {
        uint64_t *sm = reinterpret_cast<uint64_t *>(P.inh + ((size_t)(b % 4) * P.B + m) * 32);
        const uint64_t kb = (uint64_t)__double_as_longlong(k);
        st_coh16(coh_rsrc(sm), 0, u32x4{(uint32_t)(uint64_t)d, (uint32_t)((uint64_t)d >> 32), (uint32_t)kb, (uint32_t)(kb >> 32)});
        st_coh(sm + 2, (uint64_t)(uint32_t)ix | (uint64_t)(uint32_t)(ix == kNoIdx ? -1 : src) << 32);
    }
}

// ------------------------------------------------------------------------------------------------
// MERGE role (slot id = kMS * merger workgroup + slot, id < B; kMT threads): pods m = id, id + kMS * M, ...
// of every batch
// ------------------------------------------------------------------------------------------------
template <int KC, int K, int PRIO, int DOM, bool LAB, bool F53>
__device__ __forceinline__ void merge_role(const PersistArgs &P, char *sbase, const int g) {
    using ML = MergeLayout<KC, K>;
    static_assert(sizeof(MergeSmem<KC, K, kMT>) >= 1024 * 4 + kMW * 12, "serve_rescue's scratch");
    MergeCtl *pc = reinterpret_cast<MergeCtl *>(sbase);
    MergeSmem<KC, K, kMT> &ms = *reinterpret_cast<MergeSmem<KC, K, kMT> *>(sbase + ML::ctl_bytes);
    uint32_t *s_msg = reinterpret_cast<uint32_t *>(sbase + ML::ctl_bytes + ML::merge_bytes);  // this rank's list
    uint32_t *s_all = s_msg + msg_words(K);                                                     // every rank's list
    const int mtid = threadIdx.x % kMT;
    const int G = P.G;
    const int slot_prog = G + g;
    const int64_t NP = P.pods.p;
    Ctl *ctl = P.ctl;
    unsigned bar = 0;
    auto sync = [&]() { role_sync(&pc->mbar, bar, kMW); };
    int64_t nact = 0;
    int idle = 0;
    unsigned long long served = 0;  // rescue requests this slot has served
    // a wait of the slot (mtid 0 polls) that serves the commit's rescue requests while it waits; false: timed
    // out (error errc).  Every path from the read of pc->m_w to its next write passes a role_sync.
    auto mwait = [&](int64_t b, const unsigned long long *p, unsigned long long v, int errc, int phase) -> bool {
        for (;;) {
            if (mtid == 0) {
                unsigned long long seen = 0, q = 0;
                prog_at(P, slot_prog, b, phase, 0);
                const int w = poll_ge_or_rescue(P, slot_prog, p, v, served, &q, &seen);
                if (w == 2) {
                    set_err(P.err, errc);
                    prog_at(P, slot_prog, b, phase | kProgTimedOut, seen);
                }
                pc->m_w = w;
                pc->m_q = q;
            }
            sync();
            const int w = pc->m_w;
            if (w == 0) return true;
            if (w == 2) return false;
            if (mtid == 0) prog_at(P, slot_prog, b, kProgRescue, pc->m_q);
            served = pc->m_q;
            serve_rescue<PRIO, DOM, LAB, F53>(P, g, mtid, reinterpret_cast<char *>(&ms), sync);
        }
    };
    for (int64_t b = 0;; ++b) {
        if (b >= kPipeLag && !mwait(b, &ctl->committed_x[g % kCtlReplicas].v, (unsigned long long)(b - kPipeLag + 1), 6,
                                    kProgWaitCommit))
            return;
        if (mtid == 0) {
            pc->m_p0 = (int64_t)ld_coh(&ctl->plan[b % kPlanRing]);
            pc->m_done = b >= kPipeLag ? (int64_t)ld_coh(&ctl->cursor_at[(b - kPipeLag) % kPlanRing]) : 0;
            pc->m_stop = __hip_atomic_load(P.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ? 3 : 0;
        }
        sync();
        if (pc->m_stop) return;
        const int64_t p0 = pc->m_p0;
        if (pc->m_done >= NP) return;
        if (p0 < 0 || p0 >= NP) {
            if (mtid == 0) prog_at(P, slot_prog, b, kProgIdle, (uint64_t)p0);
            if (++idle > kPlanRing) {
                if (mtid == 0) set_err(P.err, 8);
                return;
            }
            sync();  // m_p0 / m_done are rewritten next iteration
            continue;
        }
        idle = 0;
        ++nact;
        const int slot = (int)((nact - 1) % 4);
        const unsigned long long use = (unsigned long long)((nact - 1) / 4);
        // the pods' keys against the older inherited export, while the score workgroups still scan the batch: off
        // the merge -> commit path (after the merge instead, c4 measured 10 % slower: the merges then end later)
        if (P.inh && b >= 2) {
            if (!mwait(b, &ctl->committed_x[g % kCtlReplicas].v, (unsigned long long)(b - 1), 6, kProgWaitCommit)) return;
            jitter_at(P.jitter, b, 3);
            for (int m = g; m < P.B; m += kMS * P.M)
                if (p0 + m < NP) inherit_x2_keys<PRIO, DOM, LAB, F53>(P, b, m, p0 + m, mtid);
        }
        if (!mwait(b, &ctl->arrive[slot].v, (use + 1) * (unsigned long long)G, 7, kProgWaitArrive)) return;
        if (mtid == 0 && g == 0) trace_at(P, b, 7);
        const size_t part_elems = (size_t)P.B * G;
        char *lb = P.lring + (size_t)(b % 4) * P.lists_bytes;
        MergeArgs ma{};
        ma.in = P.part + (size_t)(b % kPipeLag) * part_elems * KC;
        ma.in_cnt = nullptr;  // the counts travel in entry 0's pad
        ma.C_in = G; ma.C_out = 1; ma.chunk_input = 1;
        ma.cursor = &ctl->plan[b % kPlanRing]; ma.P = NP; ma.B = P.B;
        ma.p0_known = 1; ma.p0v = p0;
        ma.tag = (uint32_t)((b + 1) & 0xffff);
        ma.err = P.err;
        ma.nodes = P.nodes; ma.node_offset = P.node_offset;
        ma.dbg = P.mdbg;
        ma.out_rec = reinterpret_cast<Rec *>(lb);
        ma.out_fc = reinterpret_cast<int64_t *>(lb + (size_t)P.B * K * sizeof(Rec));
        for (int m = g; m < P.B; m += kMS * P.M) {
            const bool xchg = P.R > 1 && p0 + m < NP;  // uniform over the merge waves
            // the pod's list is staged in LDS (the message the exchange sends, or the commit's list), so that it
            // leaves as 16-byte sc1 stores (an 8-byte sc1 store costs a whole memory write request)
            ma.lds_msg = p0 + m < NP ? s_msg : nullptr;
            merge_pod_fast<KC, K, true, kMT>(ma, m, mtid, ms, sync);
            if (!xchg && p0 + m < NP) {
                static_assert(K * sizeof(Rec) % 16 == 0, "a list is whole 16-byte chunks");
                constexpr int kChunks = K * (int)sizeof(Rec) / 16;
                sync();
                if (mtid < kChunks) {
                    const uint32_t *w = s_msg + 4 * mtid;
                    st_coh16(coh_rsrc(ma.out_rec + (size_t)m * K), (uint32_t)(16 * mtid), u32x4{w[0], w[1], w[2], w[3]});
                }
                if (mtid == kChunks)
                    st_coh(ma.out_fc + m, (uint64_t)s_msg[K * kRecWords] | (uint64_t)s_msg[K * kRecWords + 1] << 32);
            }
            if (xchg) {
                // this rank's list of pod m -> slot (a % 4, rank, m) of every rank's ring; then the R lists of
                // pod m from this rank's ring -> rank merge -> the commit's list (lring)
                constexpr int MW = msg_words(K);
                const int RR = P.R;
                const uint32_t tag = P.epoch0 + (uint32_t)nact;
                sync();
                for (int e = mtid; e < MW * RR; e += kMT) {
                    const int r = e / MW, w = e % MW;
                    uint64_t *dst = reinterpret_cast<uint64_t *>(
                        P.rx_peer[r] + ((size_t)(slot * RR + P.rank) * P.B + m) * (size_t)P.xchg_stride);
                    st_sys(dst + w, gran_enc(s_msg[w], gran_tag(tag)));
                }
                bool ok = true;
                const char *own = P.rx_peer[P.rank];
                for (int e = mtid; e < MW * RR; e += kMT) {
                    const int r = e / MW, w = e % MW;
                    const uint64_t *src = reinterpret_cast<const uint64_t *>(
                        own + ((size_t)(slot * RR + r) * P.B + m) * (size_t)P.xchg_stride);
                    uint32_t word = 0;
                    if (ok && !granule_wait(src + w, tag, P.timeout_ticks, &word)) ok = false;
                    s_all[e] = word;
                }
                if (!ok) { set_err(P.err, 10); pc->m_stop = 1; }
                sync();
                if (pc->m_stop) return;
#if KSCHED_XCHG_DEBUG  // diagnostics build (tests/diag/xchg_ring_experiment.py): message hashes and the first messages
                if (P.xdbg && mtid <= RR && nact - 1 < P.xdbg_cap) {  // diagnostics: the messages as received / sent
                    const uint32_t *msg = mtid < RR ? s_all + mtid * MW : s_msg;
                    uint64_t h = 0x9e3779b97f4a7c15ull;
                    for (int w = 0; w < MW; ++w) h = (h ^ msg[w]) * 0x100000001b3ull;
                    P.xdbg[((size_t)(nact - 1) * P.B + m) * (RR + 1) + mtid] = h;
                }
                if (P.xdbg && nact - 1 < 16) {  // diagnostics: the first 16 active batches' sent messages, whole
                    uint32_t *xm = reinterpret_cast<uint32_t *>(P.xdbg + (size_t)P.xdbg_cap * P.B * (RR + 1)) +
                                   ((size_t)(nact - 1) * P.B + m) * MW;
                    for (int w = mtid; w < MW; w += kMT) xm[w] = s_msg[w];
                }
#endif
                if (mtid < 64) rank_merge_msgs<K>(s_all, RR, ma.out_rec + (size_t)m * K, ma.out_fc + m);
            }
            jitter_at(P.jitter, b, 4 + m);
            drain_stores();
            sync();  // every merge wave's stores drained before the count; LDS free for the next pod
#if KSCHED_XCHG_DEBUG
            if (P.xdbg && mtid < 64 && nact - 1 < P.xdbg_cap && p0 + m < NP) {  // diagnostics: the list as written
                const uint64_t *w = reinterpret_cast<const uint64_t *>(ma.out_rec + (size_t)m * K + (mtid < K ? mtid : 0));
                int64_t x = mtid < K ? (int64_t)dbg_mix(ld_coh(w), ld_coh(w + 1), mtid) : 0;
                x = wave_sum_i64(x);
                if (mtid == 0)
                    P.xdbg[xdbg_sums_off(P.xdbg_cap, P.B, P.R, K) + ((size_t)(nact - 1) * P.B + m) * 2] = (uint64_t)x;
            }
#endif
            if (mtid == 0) {
                if (m == 0) st_coh(&ctl->nact, (uint64_t)nact);
                const unsigned long long d =
                    __hip_atomic_fetch_add(&ctl->merged[slot].v, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (d + 1 == (use + 1) * (unsigned long long)P.B) trace_at(P, b, 2);
                prog_at(P, slot_prog, b, kProgMerged, d + 1);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------
// COMMIT role (workgroups 0 and 1, all kPipeWaves = 12 waves each): workgroup `par` commits the batches
// b = par, par + 2, ... .  Per batch: the work that does not depend on commit(b - 1) -- tables, the slots of
// export(b - 2), the wait for the batch's B merges (Ctl::merged), its lists, the mergers' keys -- runs while the
// other workgroup commits b - 1; then the hand-off (Ctl::committed >= b: commit(b - 1) published its cursor,
// plans and export), the rest of the commit (commit_spc_batch), Ctl::committed = b + 1.  The plans, the cursor
// and the export travel through global memory (sc1), so the two workgroups share no LDS state.  Once every pod
// is resolved, the workgroup that resolved the last one publishes a committed count no wait can exceed, so
// every workgroup still waiting -- the other commit workgroup included -- sees the end.
// ------------------------------------------------------------------------------------------------
template <int K, int PRIO, int DOM, bool LAB, bool F53>
__device__ __forceinline__ void commit_role(const PersistArgs &P, char *smem, const int par) {
    __builtin_amdgcn_s_setprio(3);
    PersistLocal &loc = *reinterpret_cast<PersistLocal *>(smem);
    char *cs = smem + commit_loc_bytes();
    uint32_t *canary = reinterpret_cast<uint32_t *>(cs - kCanaryBytes);
    if (threadIdx.x < kCanaryBytes / 4) canary[threadIdx.x] = 0xA5A5A5A5u ^ threadIdx.x;
    __shared__ int s_stop;
    __shared__ HandoffRes s_ho;
    __shared__ int s_hr;
    Ctl *ctl = P.ctl;
    // k_ctl_init ran before this kernel on the stream: the call's initial cursor
    if (threadIdx.x == 0) {
        loc.cursor = (int64_t)ld_rmw(&ctl->cursor);
        for (int i = 0; i < 5; ++i) loc.stats[i] = 0;
        loc.xcount = 0;
        loc.xcount2 = 0;
        loc.rseq = 0;
        loc.rescue_credit = 4 * P.rescue_cap;
    }
    __syncthreads();
    const int64_t cursor0 = loc.cursor;
    const int cslot = P.G + P.B + par;  // progress slot
    constexpr int kPoller = 128;  // the merges' wait: wave 2 lane 0 (its wave loads nothing else in the prologue)
    const int rep = (par + kCtlReplicas - 1) % kCtlReplicas;  // the committed replica this workgroup polls
    int64_t nact = 0;  // active batches among 0 .. b (both workgroups' batches)
    int idle = 0;
    for (int64_t b = par;; b += 2) {
        // the plans of b - 1 and b were set by commits b - 4 and b - 3 (or k_ctl_init).  Both are in this
        // workgroup's LDS copy already: plan(b - 1) from its own commit(b - 4) (persist_plan), plan(b) from the
        // hand-off record commit(b - 2) received (commit(b - 3) drains nothing in front of the record, so its
        // store to Ctl::plan may still be in flight here).  Only the plans k_ctl_init set come from memory.
        const int64_t p0 = b >= 2 ? loc.plan[b % kPlanRing] : (int64_t)ld_coh(&ctl->plan[b % kPlanRing]);
        const int64_t pm = b >= 4 ? loc.plan[(b - 1) % kPlanRing] : b >= 1 ? (int64_t)ld_coh(&ctl->plan[(b - 1) % kPlanRing]) : -1;
        const bool act = p0 >= 0 && p0 < P.pods.p;
        nact += ((b >= 1 && pm >= 0 && pm < P.pods.p) ? 1 : 0) + (act ? 1 : 0);
        jitter_at(P.jitter, b, 100);  // the commit workgroup's loop top
        if (b < 2) {
            // the first two plans reach the LDS copy here; every wave reads it (commit_spc_batch) only after this
            // barrier -- without it a wave could read the copy before thread 0 wrote it: an LDS word left by an
            // earlier kernel (round 5: a fresh engine then took the idle path on some waves only)
            if (threadIdx.x == 0) loc.plan[b % kPlanRing] = p0;
            __syncthreads();
        }
        if (!act && ++idle > kPlanRing) {
            // pods remain but nothing is planned: a truncation re-plans within kPipeLag batches, so this is a
            // protocol error -- stop everyone instead of spinning
            if (threadIdx.x == 0) atomicCAS(P.err, 0, 9);
            if (threadIdx.x < 64) publish_committed_all(ctl, 1ull << 62);
            return;
        }
        if (threadIdx.x == 0) trace_at(P, b, 15);
        LanePods pre{0, 0, 0, 0};
        unsigned long long early_m = 0;
        if (act) {
            idle = 0;
            // the pods' requests: their loads overlap the prologue (a batch voided by commit(b - 1) discards them)
            pre = load_lane_pods<LAB>(P.pods, p0, (int)(P.pods.p - p0 < P.B ? P.pods.p - p0 : P.B));
            // the merge count, read now: its latency hides behind the prologue (the merges are usually done)
            if (threadIdx.x == kPoller)
                early_m = __hip_atomic_load(&ctl->merged[(nact - 1) % 4].v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // the batch's merges (everything of the commit that needs no candidate list runs before this)
        auto wait_merged = [&]() -> bool {
            if (act) {
                const uint64_t tw0 = P.cdbg ? __builtin_amdgcn_s_memtime() : 0;
                if (threadIdx.x == kPoller) {
                    const int slot = (int)((nact - 1) % 4);
                    const unsigned long long want = (unsigned long long)((nact - 1) / 4 + 1) * (unsigned long long)P.B;
                    unsigned long long seen = 0;
                    s_stop = 0;
                    if (P.cdbg && early_m >= want) P.cdbg[15] += 1;  // diagnostics: the early read sufficed
                    if (early_m < want) {
                        prog_at(P, cslot, b, kProgWaitMerged, 0);
                        s_stop = poll_ge(&ctl->merged[slot].v, want, P.timeout_ticks, &ctl->polls_rmw, &seen) ? 0 : 1;
                        if (s_stop) prog_at(P, cslot, b, kProgWaitMerged | kProgTimedOut, seen);
                    }
                    if (P.cdbg) P.cdbg[10] += __builtin_amdgcn_s_memtime() - tw0;  // the poll
                }
                __syncthreads();
                if (P.cdbg && threadIdx.x == 0) P.cdbg[11] += __builtin_amdgcn_s_memtime() - tw0;  // poll + barrier
                if (s_stop) return false;
            }
            if (threadIdx.x == 0) trace_at(P, b, 3);
            return true;
        };
        // commit(b - 1) -> commit(b): the two hand-off granules tagged b (Ctl::hrec, put_handoff) and the n1 entries of
        // export(b - 1), every 16-byte chunk tagged b (store_xrec), polled together by wave 0 (lane = entry) -- one
        // round of loads shows the record and the export, and commit(b - 1) drains nothing in front of them -- or the
        // end of the call (Ctl::committed >= 2^62: the last pod resolved, or an error elsewhere)
        const XRec *xin_e = reinterpret_cast<const XBuf *>(P.xring + (size_t)(b >= 1 ? (b - 1) % 4 : 4) * P.xbuf_bytes)->e;
        auto handoff = [&](HandoffRes *r, XRec *xo) -> int {
            if (threadIdx.x < 64) {
                const int lane = (int)threadIdx.x;
                int st = 0;
                HandoffRes h{};
                if (b == 0) {
                    h.cursor = cursor0;
                    h.plan_next = (int64_t)ld_coh(&ctl->plan[(kPipeLag - 1) % kPlanRing]);
                } else {
                    if (lane == 0) prog_at(P, cslot, b, kProgWaitCommit, 0);
                    const __amdgpu_buffer_rsrc_t hr = coh_rsrc(&ctl->hrec);
                    const uint32_t tag = (uint32_t)b;
                    const uint64_t t0 = wall_clock64();
                    for (int it = 1;; ++it) {
                        const u32x4 c0 = ld_coh16(hr, 0), c1 = ld_coh16(hr, 16);  // one address: one request
                        // (lanes past the export slot's 2B entries load nothing: the buffer resource does not bound them)
                        const bool eok = lane < 2 * P.B ? load_xrec_pipe(xin_e, lane, tag, xo) : true;
                        const bool hok = __builtin_amdgcn_readfirstlane((int)(c0.x == tag && c1.x == tag)) != 0;
                        const int n1 = hok ? (int)__builtin_amdgcn_readfirstlane((int)c0.y) : 64;
                        if (hok && __ballot(lane < n1 && !eok) == 0) {
                            h.n1 = n1;
                            h.cursor = (int64_t)((uint64_t)c0.w << 32 | c0.z);
                            h.rseq = (int64_t)c1.y;
                            h.plan_next = (int64_t)((uint64_t)c1.w << 32 | c1.z);
                            break;
                        }
                        if ((it & 63) == 0) {
                            int end = 0;
                            if (lane == 0) {
                                const unsigned long long cm =
                                    __hip_atomic_load(&ctl->committed_x[rep].v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                if (cm >= (1ull << 62)) {
                                    end = 1;
                                } else if ((int64_t)(wall_clock64() - t0) > P.timeout_ticks) {
                                    prog_at(P, cslot, b, kProgWaitCommit | kProgTimedOut, cm);
                                    end = -1;
                                }
                            }
                            end = __builtin_amdgcn_readfirstlane(end);
                            if (end) { st = end; break; }
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
                if (lane == 0) {
                    s_ho = h;
                    s_hr = st;
                }
            }
            __syncthreads();
            *r = s_ho;
            if (threadIdx.x == 0) trace_at(P, b, 22);  // past the hand-off
            return s_hr;
        };
        CommitArgs ca{};
        char *lb = P.lring + (size_t)(b % 4) * P.lists_bytes;
        ca.lists = reinterpret_cast<const Rec *>(lb);
        ca.fc0 = reinterpret_cast<const int64_t *>(lb + (size_t)P.B * K * sizeof(Rec));
        ca.pods = P.pods; ca.ctl = ctl; ca.B = P.B;
        ca.plan = &ctl->plan[b % kPlanRing];
        ca.plan1 = &ctl->plan[(b + kPipeLag - 1) % kPlanRing];
        ca.plan2 = &ctl->plan[(b + kPipeLag) % kPlanRing];
        // exports of b - 1 and b - 2 (ring slot 4 stays empty: the batches before the first)
        ca.xin = reinterpret_cast<const XBuf *>(P.xring + (size_t)(b >= 1 ? (b - 1) % 4 : 4) * P.xbuf_bytes);
        ca.xin2 = reinterpret_cast<const XBuf *>(P.xring + (size_t)(b >= 2 ? (b - 2) % 4 : 4) * P.xbuf_bytes);
        ca.xout = reinterpret_cast<XBuf *>(P.xring + (size_t)(b % 4) * P.xbuf_bytes);
        ca.out = P.out;
        ca.batch = b;
        ca.cursor_at = &ctl->cursor_at[b % kPlanRing];
        ca.dbg = P.cdbg;
        ca.trace_row = (P.trace && b < P.trace_cap) ? P.trace + b * kTraceCols : nullptr;
        ca.loc = &loc;
        ca.rescue = P.rescue;  // null: an exhausted list truncates its batch (KSCHED_RESCUE_MAX=0)
        ca.xp = &P;            // R > 1: the rescue's rank fold
        ca.dbg_act = nact - 1;
        ca.rescue_n = P.B;
        ca.rescue_max = P.rescue_max;
        ca.rescue_rate = P.rescue_rate;
        ca.rescue_look = P.rescue_look;
        ca.rescue_cap = P.rescue_cap;
        ca.rescue_low = P.rescue_low;
        ca.touch_screen = P.touch_screen;
        ca.inh = P.inh;
        ca.timeout_ticks = P.timeout_ticks;
        ca.err = P.err;
        const int rc = commit_spc_batch<K, PRIO, DOM, LAB, F53, true, kPipeThreads>(ca, cs, &pre, wait_merged, handoff);
        if (rc == 2) return;  // the call ended (or failed) elsewhere
        if (rc == 0) {
            if (threadIdx.x == 0) atomicCAS(P.err, 0, 5);
            if (threadIdx.x < 64) publish_committed_all(ctl, 1ull << 62);
            return;
        }
        __syncthreads();
        if (threadIdx.x < kCanaryBytes / 4 && canary[threadIdx.x] != (0xA5A5A5A5u ^ threadIdx.x)) {
            // an LDS write below the commit's arrays: report which word, once
            if (atomicCAS(P.err, 0, 15) == 0 && P.prog)
                P.prog[kProgWords * cslot + 2] = (uint64_t)b << 32 | (uint64_t)threadIdx.x << 16 | (canary[threadIdx.x] & 0xffffu);
        }
        if (threadIdx.x == 0) {
            trace_at(P, b, 4);
            prog_at(P, cslot, b, kProgCommitted, 0);
        }
        if (loc.cursor >= P.pods.p) {
            if (threadIdx.x < 64) publish_committed_all(ctl, 1ull << 62);
            return;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// The kernel.  <= 128 VGPRs (1024 threads: four waves per SIMD).
// ------------------------------------------------------------------------------------------------
template <int KC, int K, int PRIO, int DOM, bool LAB, bool F53>
__global__ __launch_bounds__(kPipeThreads) void k_pipe(PipeLaunch L) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // this workgroup's rank (ranks of one process sharing the device run as one launch; R = 1 otherwise)
    int r = 0;
#pragma unroll
    for (int i = 1; i < kMaxLocalRanks; ++i) r += (i < L.R && (int)blockIdx.x >= L.base[i]) ? 1 : 0;
    const PersistArgs &P = L.P[r];
    const int blk = (int)blockIdx.x - L.base[r];
    if (P.poison_lds) {  // diagnostics: any LDS read before its write then sees the fill, not a predecessor's data
        const int role = blk < kCommitWGs ? 1 : (blk < kCommitWGs + P.G ? 2 : 4);
        // role bit 8: a distinct pattern per role (the fill ^ role * 0x01010101), so a value read before its write
        // names the role whose LDS it came from
        const uint32_t fill = (P.lds_fill_role & 8) ? P.lds_fill ^ ((uint32_t)role * 0x01010101u) : P.lds_fill;
        if (P.lds_fill_role & role)
            for (int i = (int)threadIdx.x; i < P.poison_lds / 4; i += kPipeThreads)
                if (4 * i >= P.lds_fill_lo && 4 * i < P.lds_fill_hi) reinterpret_cast<uint32_t *>(smem)[i] = fill;
        __syncthreads();
    }
    if (blk < kCommitWGs) {
        commit_role<K, PRIO, DOM, LAB, F53>(P, smem, blk);
        return;
    }
    if (blk < kCommitWGs + P.G) {
        PipeCtl *pc = reinterpret_cast<PipeCtl *>(smem);
        if (threadIdx.x == 0) { pc->sbar = 0; pc->mbar = 0; }
        __syncthreads();
        score_role<KC, K, PRIO, DOM, LAB, F53>(P, smem, blk - kCommitWGs);
        return;
    }
    // a merger workgroup: kMS independent pod slots of kMT threads
    const int slot = (int)threadIdx.x / kMT;
    const int id = (blk - kCommitWGs - P.G) * kMS + slot;
    char *sbase = smem + (size_t)slot * MergeLayout<KC, K>::slot_bytes;
    if (threadIdx.x % kMT == 0) reinterpret_cast<MergeCtl *>(sbase)->mbar = 0;
    __syncthreads();  // the only workgroup-wide barrier: before the slots part
    if (id < P.B) merge_role<KC, K, PRIO, DOM, LAB, F53>(P, sbase, id);
}

template <int KC, int K, int PRIO, int DOM, bool LAB, bool F53>
hipError_t pipe_one(const PipeLaunch &L0, int launch, PipeInfo *info, hipStream_t s) {
    auto fn = k_pipe<KC, K, PRIO, DOM, LAB, F53>;
    PipeLaunch L = L0;
    // the screened scan when its reciprocals fit beside everything else, keeping pass 1's per-pair records
    // when those fit too (every rank of a launch has the same geometry up to one row)
    constexpr size_t kLds = (size_t)160 * 1024;
    int R = 0;
    for (int r = 0; r < L.R; ++r) R = L.P[r].rows_per_wg > R ? L.P[r].rows_per_wg : R;
    const int sh = ScoreLayout<KC, K>::total_with_hrec(R) <= kLds ? 1 : 0;
    const int so = ScoreLayout<KC, K>::total_screen(R) <= kLds ? 1 : 0;
    for (int r = 0; r < L.R; ++r) { L.P[r].screen_h = sh; L.P[r].screen_ok = so; }
    const size_t sl = sh ? ScoreLayout<KC, K>::total_with_hrec(R)
                         : (so ? ScoreLayout<KC, K>::total_screen(R) : ScoreLayout<KC, K>::total(R));
    const size_t cl = commit_total_bytes<K>(), ml = MergeLayout<KC, K>::total;
    const size_t lds = sl > cl ? (sl > ml ? sl : ml) : (cl > ml ? cl : ml);
    if (info) {
        hipFuncAttributes at{};
        hipError_t e = hipFuncGetAttributes(&at, (const void *)fn);
        if (e != hipSuccess) return e;
        info->lds = lds;
        info->static_lds = at.sharedSizeBytes;
        info->vgprs = at.numRegs;
        info->spill = at.localSizeBytes;
        info->occ = 0;
        if (lds + at.sharedSizeBytes <= kLds) {
            e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&info->occ, fn, kPipeThreads, lds);
            if (e != hipSuccess) return e;
        }
    }
    if (!launch) return hipSuccess;
    if (L.R < 1 || L.R > kMaxLocalRanks || L.base[0] != 0) return hipErrorInvalidValue;
    for (int r = 0; r < L.R; ++r) {
        const PersistArgs &a = L.P[r];
        if (a.G > kMT || a.B > 64 || a.M * kMS < a.B || L.base[r + 1] - L.base[r] != kCommitWGs + a.G + a.M ||
            a.rows_per_wg >= 65536)  // (a record's count field is 16 bits)
            return hipErrorInvalidValue;
    }
    hipError_t e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    if (launch == 2) {  // KSCHED_PLAIN_LAUNCH (profiled runs): the caller checked the occupancy
        hipLaunchKernelGGL(fn, dim3(L.base[L.R]), dim3(kPipeThreads), lds, s, L);
        return hipGetLastError();
    }
    void *args[] = {&L};
    return hipLaunchCooperativeKernel((const void *)fn, dim3(L.base[L.R]), dim3(kPipeThreads), args, (unsigned)lds, s);
}

template <int PRIO, int DOM, bool LAB, bool F53>
hipError_t pipe_kk(int KC, int K, const PipeLaunch &a, int launch, PipeInfo *info, hipStream_t s) {
    if (KC == 4 && K == 4) return pipe_one<4, 4, PRIO, DOM, LAB, F53>(a, launch, info, s);
    if (KC == 4 && K == 8) return pipe_one<4, 8, PRIO, DOM, LAB, F53>(a, launch, info, s);
    if (KC == 4 && K == 16) return pipe_one<4, 16, PRIO, DOM, LAB, F53>(a, launch, info, s);
    if (KC == 8 && K == 8) return pipe_one<8, 8, PRIO, DOM, LAB, F53>(a, launch, info, s);
    if (KC == 8 && K == 16) return pipe_one<8, 16, PRIO, DOM, LAB, F53>(a, launch, info, s);
    return hipErrorNotSupported;
}

template <int PRIO, int DOM>
hipError_t pipe_lf(int KC, int K, bool lab, bool f53, const PipeLaunch &a, int launch, PipeInfo *info, hipStream_t s) {
    if (PRIO == kPrioPrice) f53 = false;  // best-price never divides
    if (lab) return f53 ? pipe_kk<PRIO, DOM, true, true>(KC, K, a, launch, info, s)
                        : pipe_kk<PRIO, DOM, true, false>(KC, K, a, launch, info, s);
    return f53 ? pipe_kk<PRIO, DOM, false, true>(KC, K, a, launch, info, s)
               : pipe_kk<PRIO, DOM, false, false>(KC, K, a, launch, info, s);
}

}  // namespace

#if KSCHED_PIPE_PART == 0
hipError_t pipe_part_price(int KC, int K, bool lab, bool f53, const PipeLaunch &a, int launch, PipeInfo *info,
                           hipStream_t s) {
    return pipe_lf<kPrioPrice, kDomFeasible>(KC, K, lab, f53, a, launch, info, s);
}

// All ranks meet on the device and agree on the minimum of `mine` (tag: this call's epoch0; the
// batches of the call use epoch0 + 1, ...).  One wave; lane r < R writes rank r's barrier granule.
__global__ __launch_bounds__(64) void k_xchg_min(PersistArgs P, int32_t mine, int32_t *out) {
    const int lane = threadIdx.x;
    const size_t off = (size_t)4 * P.R * P.B * (size_t)P.xchg_stride;
    const uint32_t tag = P.epoch0;
    if (lane < P.R) st_sys(reinterpret_cast<uint64_t *>(P.rx_peer[lane] + off) + P.rank, gran_enc((uint32_t)mine, gran_tag(tag)));
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
#elif KSCHED_PIPE_PART == 1
hipError_t pipe_part_res_all(int KC, int K, bool lab, bool f53, const PipeLaunch &a, int launch, PipeInfo *info,
                             hipStream_t s) {
    return pipe_lf<kPrioResource, kDomAll>(KC, K, lab, f53, a, launch, info, s);
}
#else
hipError_t pipe_part_res_feas(int KC, int K, bool lab, bool f53, const PipeLaunch &a, int launch, PipeInfo *info,
                              hipStream_t s) {
    return pipe_lf<kPrioResource, kDomFeasible>(KC, K, lab, f53, a, launch, info, s);
}
#endif

}  // namespace ksched
