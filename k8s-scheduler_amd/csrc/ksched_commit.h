// ksched_commit.h -- the ordered commit of one speculative batch (speculation + parallel check), shared by
// the stream pipeline's k_commit_spc (ksched_commit_spc.hip) and the commit workgroup of the persistent
// pipeline (ksched_pipe.hip).
//
// Same result as the sequential replay (k_commit): pods of the batch
// in order, each seeing every placement before it (anchor/schedule.go:185-197).  Instead of deciding
// one pod at a time, a round
//   1. (wave 0, integer work only) GUESSES every remaining pod's placement: its first list entry that
//      is neither touched nor guessed by an earlier pod of the round ("first touch"), or none when the
//      pod has no feasible node or its list is exhausted;
//   2. (all waves: 8 in k_commit_spc, 12 in the persistent commit) evaluates the guesses in parallel: for every guessed node, its state after the
//      guessing pod's commit, and every pod's exact key and predicate delta against that state;
//   3. (wave 0, lane = pod) checks each pod's exact sequential decision under the guesses of the pods
//      before it: fc = predicate count, t* = best touched node (confirmed + guessed before it), u* =
//      its guess.  The guesses up to the first pod whose decision differs are the sequential outcome
//      (induction from the round's start); that pod is resolved exactly and the next round starts
//      after it.
// Placements are first touches almost always (99.4 % on BASELINE c4), so a batch usually takes one or
// two rounds.  The guess window adapts (halves around failures) to bound the cost of adversarial
// batches.  The lists, cut rule, touched-set inheritance, export, plan and truncation are those of
// k_commit.
#pragma once

#include <hip/hip_runtime.h>

#ifndef KSCHED_XCHG_DEBUG
#define KSCHED_XCHG_DEBUG 0  // the exchange diagnostics of tests/diag/xchg_ring_experiment.py (a separate build)
#endif

#include "ksched_kernels.h"

namespace ksched {

namespace {

constexpr int kSpcHashBits = 11;  // touched + guessed node set (stale guesses stay until re-tagged)
constexpr int kSpcHash = 1 << kSpcHashBits;
// touched-node slots: the inherited commits of the previous batch (lag 2: the stream pipeline) or of the
// two previous batches (lag 3: the persistent pipeline), <= 64 each, + this batch's (<= 64)
template <bool LAG3>
constexpr int spc_slots() { return LAG3 ? 192 : 128; }
// commit_rescue publishes the touched set, at most every slot: RescueReq::ti holds them
static_assert(spc_slots<true>() + 1 <= kRescueMaxT, "RescueReq::ti must hold the persistent commit's touched slots");
constexpr int kSpcInvalid = kSpcHash - 1;  // table position reserved for "no entry" (always taken)
constexpr int kGS = 14;                     // words per guessed entry in SpcSmem::GS

// The touched-node screen (persistent commit, resource priority).  A pod's key for a touched
// node matters only where it can beat an untouched entry of the pod's list -- each of which keys at or above the
// list's last entry -- or where no untouched entry is left: a complete (not cut) list then takes the best touched
// node, a cut one compares it with its last entry (below it: rescue or truncation).  So a pair whose f32 screen
// (screen_pair: |screen - key| < 1.3e-5, or NaN) lies below thr = RN_f32(last key - 5e-5) of a CUT list keys
// below every entry of the list, and its exact key is skipped: S holds kSkipKey (a NaN, which no comparison ranks)
// instead.  Only the rescue of an exhausted cut list compares touched nodes below the last entry; it re-keys the
// pod's skipped slots first (rekey_row).  On c4 about 0.1 % of these pairs could matter.
constexpr uint64_t kSkipKeyBits = 0x7ff8000000000badull;
__device__ __forceinline__ double skip_key() { return __longlong_as_double((long long)kSkipKeyBits); }
// the f32 reciprocal the screen takes, from the refined f64 one (screen_recip's domain: NaN unless 0 < a < 2^52)
__device__ __forceinline__ float screen_y(int64_t a, double y) {
    return (a > 0 && a < (1ll << 52)) ? (float)y : __builtin_nanf("");
}

struct alignas(8) SpcSlot {
    int32_t idx;
    int32_t mine;     // committed by this batch (exported)
    int64_t sb[3];    // state when this batch's commit started
    int64_t cur[3];   // current state
    uint64_t labels;
    float price;
    int32_t pad;
};
static_assert(sizeof(SpcSlot) == 72, "SpcSlot");

struct SpcSmem {
    int32_t *hk;      // open-addressed table: node index per position (-1 = empty)
    int64_t *s0;      // prologue only (aliases D): [inherited slot][3] state at this batch's score snapshot
    double *iy;       // prologue only (aliases GS): [inherited slot][6] current state as doubles, reciprocals
    int32_t *HP;      // [K][64] table position of list entry (q, pod); kSpcInvalid for no entry
    uint32_t *tkc;    // [64] words: bit = position taken by a CONFIRMED touch (T)
    int32_t *ti;      // node index per slot
    SpcSlot *T;
    double *S;        // [64 pods][slots + 1] key of (pod, slot), -inf = not eligible
    double *LK;       // [K][64] list keys (lane-contiguous)
    int32_t *LI;      // [K][64] list node indices
    int8_t *D;        // [64 guessing pods][64 pods] predicate delta of the guessed commit
    int32_t *fcg;     // per pod: sum of D over this round's guesses before it
    int32_t *dfacc;   // per pod: predicate delta of the inherited slots
    int32_t *gn;      // per pod: guessed node (>= 0), -1 list exhausted, -2 predicted no fit
    int32_t *gq;      // per pod: list position of the guess
    int32_t *gs;      // per pod: slot of the guess
    double *pbk;      // [waves][64 pods] partial best key over the wave's guessed columns
    int64_t *pbx;     // [waves][64 pods] (slot << 32) | node of that best
    int32_t *ctl;     // [0] round start c, [1] window end, [2] stop
    int32_t *own;     // [kSpcHash] lowest pod proposing each position in a guess iteration (64 = none);
                      // step 1 only (aliases pbk/pbx, which steps 2-3 use)
    uint64_t *GS;     // [64 pods][kGS] each pod's guessed entry: state a[3], labels, price, and the state after
                      // the pod's commit n[3] with its (double) and refined reciprocals (computed once, lane = pod)
    float *thr;       // [64] per pod: a touched node's key screens below this -> it cannot matter (kSkipKey)
    // persistent commit: the slots of the older export (batch b - 2) are keyed by the merger workgroups
    int16_t *x2s;     // [64] slot of that export's entry e (-1: the node is also in export(b - 1): no slot)
};

__device__ __forceinline__ uint32_t spc_hash(int32_t idx) {
    return ((uint32_t)idx * 2654435761u) >> (32 - kSpcHashBits);
}

// Node -> position in an open-addressed table of every node the batch can touch (list entries and
// inherited slots).  The position is a compact node id: "taken" is one bit per position.
__device__ __forceinline__ int spc_pos_insert(int32_t *hk, int32_t idx, bool *existed = nullptr) {
    uint32_t h = spc_hash(idx);
    for (;;) {
        if (h != kSpcInvalid) {
            const int32_t prev = atomicCAS(&hk[h], -1, idx);
            if (prev == -1 || prev == idx) {
                if (existed) *existed = prev == idx;
                return (int)h;
            }
        }
        h = (h + 1) & (kSpcHash - 1);
    }
}

__device__ __forceinline__ int64_t rl64(int64_t v, int src) {
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)((uint64_t)v >> 32), src);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, src);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// plan_after_commit for the persistent commit (batch b plans batch b + kPipeLag): the plans come from
// (and go to) its LDS copy too
__device__ __forceinline__ void persist_plan(const CommitArgs &A, bool truncated, int64_t cursor) {
    PersistLocal *L = A.loc;
    const int64_t n1 = L->plan[(A.batch + kPipeLag - 1) % kPlanRing];
    int64_t nx = truncated ? cursor : (n1 < 0 ? -1 : n1 + A.B);
    if (nx >= A.pods.p) nx = -1;
    L->plan[(A.batch + kPipeLag) % kPlanRing] = nx;
    st_coh(A.plan2, (uint64_t)nx);
}

// a node state as the key needs it: the three doubles and their reciprocals (0 for a zero allocatable)
__device__ __forceinline__ void stage_state(double *o, const int64_t *a) {
    for (int r = 0; r < 3; ++r) {
        const double f = (double)a[r];
        o[r] = f;
        o[3 + r] = recip_or_zero(a[r], f);
    }
}

__device__ __forceinline__ void lds_order() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// pod (this lane)'s exact key against a node state; -inf when not eligible
template <int PRIO, int DOM, bool LAB, bool F53>
__device__ __forceinline__ double lane_key(bool f, int64_t rc, int64_t rm, int64_t rp, double rcf, double rmf,
                                           double rpf, int64_t n0, int64_t n1, int64_t n2, double y3, float pr) {
    const double nf0 = (double)n0, nf1 = (double)n1, nf2 = (double)n2;
    const double ny0 = recip_or_zero(n0, nf0), ny1 = recip_or_zero(n1, nf1), ny2 = recip_or_zero(n2, nf2);
    double k;
    const bool el = pair_key_fast<PRIO, DOM, F53>(f, rc, rm, rp, rcf, rmf, rpf, n0, n1, n2, nf0, nf1, nf2, ny0, ny1,
                                                  ny2, y3, pr, &k);
    return el ? k : -__builtin_inf();
}

// What a rescue found: the best node outside the touched set (idx = kNoIdx: none eligible) and its state.
struct RescueOut {
    double key;
    int32_t idx;
    int64_t a[3];
    uint64_t labels;
    float price;
};

// Node-sharded rescue (R > 1; wave 0 of the commit, o = this rank's best): every rank's commit made the same
// request q (the ranks replay one ordered commit), and each rank's merger slots scanned only its own shard.  The
// rank's best travels to every rank's ring -- rescue area slot (q % 2, this rank) as 14 tagged 8-byte granules
// (gran_enc, tag epoch0 + q; two parities: a rank can be one request ahead of a peer still reading the last one, never
// two) -- and the R bests fold the same way on every rank (lane = source rank, (key desc, idx asc)).  Restated by
// oracle/cpu_ref.c or_schedule_lagged_rescue2 (shards).  false: a peer's record never came (error 12).
__device__ __forceinline__ bool rescue_rank_fold(const PersistArgs &X, unsigned long long q, int64_t timeout_ticks,
                                                 int32_t *err, RescueOut *o) {
    const int lane = threadIdx.x & 63;
    const int R = X.R;
    const uint32_t t16 = gran_tag(X.epoch0 + (uint32_t)q);
    const size_t off = xchg_rescue_off(R, X.B, (size_t)X.xchg_stride) +
                       ((size_t)(q & 1) * R) * kXchgRescueRec;
    Rec mine{};
    mine.key = o->key; mine.idx = o->idx; mine.valid = o->idx != kNoIdx ? 1 : 0;
    mine.a[0] = o->a[0]; mine.a[1] = o->a[1]; mine.a[2] = o->a[2];
    mine.labels = o->labels; mine.price = o->price; mine.pad = 0;
    const uint32_t *mw = reinterpret_cast<const uint32_t *>(&mine);
    // lane r < R: this rank's record into rank r's ring (word by word: the words are wave-uniform)
    if (lane < R) {
        uint64_t *dst = reinterpret_cast<uint64_t *>(X.rx_peer[lane] + off + (size_t)X.rank * kXchgRescueRec);
#pragma unroll
        for (int i = 0; i < kXchgRescueWords; ++i)
            __hip_atomic_store(dst + i, gran_enc(mw[i], t16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // lane r < R: rank r's record from this rank's own ring
    uint32_t rw[kXchgRescueWords];
    bool ok = true;
    if (lane < R) {
        const uint64_t *src = reinterpret_cast<const uint64_t *>(X.rx_peer[X.rank] + off + (size_t)lane * kXchgRescueRec);
        const uint64_t t0 = wall_clock64();
#pragma unroll
        for (int i = 0; i < kXchgRescueWords; ++i) {
            uint32_t wv = 0;
            while (ok && !gran_dec(__hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM), t16, &wv)) {
                if ((int64_t)(wall_clock64() - t0) > timeout_ticks) { ok = false; break; }
                __builtin_amdgcn_s_sleep(1);
            }
            rw[i] = wv;
        }
    } else {
#pragma unroll
        for (int i = 0; i < kXchgRescueWords; ++i) rw[i] = 0;
    }
    if (__ballot(!ok)) {
        if (lane == 0) atomicCAS(err, 0, 12);
        return false;
    }
    Rec rr;
    uint32_t *rp = reinterpret_cast<uint32_t *>(&rr);
#pragma unroll
    for (int i = 0; i < kXchgRescueWords; ++i) rp[i] = rw[i];
    double k = (lane < R && rr.valid) ? rr.key : -__builtin_inf();
    int32_t ix = (lane < R && rr.valid) ? rr.idx : kNoIdx;
    int32_t src = lane;
    wave_argbest(k, ix, src);
    o->key = k;
    o->idx = ix;
    for (int r = 0; r < 3; ++r) o->a[r] = rl64(rr.a[r], src);
    o->labels = (uint64_t)rl64((int64_t)rr.labels, src);
    o->price = __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(rr.price), src));
    return true;
}

// The rescue of pod f's exhausted candidate list (wave 0 of the persistent commit; pod f's list is cut, every
// entry is touched and no touched node beats its last entry, so the best untouched node may lie outside it):
// publish the request -- pod f's request and the touched set T = ti[0, nT) -- as sc1 stores, drained, then the
// request number in Ctl::rescue_req; the B merger slots each scan a share of the node rows (serve_rescue,
// ksched_pipe.hip) and count their results in Ctl::rescue_done; lane = slot, the wave's arg-best is the answer.
// false: the wait timed out (error 12).  Restated by oracle/cpu_ref.c or_rescue.
__device__ __forceinline__ bool commit_rescue(const CommitArgs &A, int f, int64_t rc, int64_t rm, int64_t rp,
                                              uint64_t sel, const int32_t *ti, int nT, RescueOut *o) {
    const int lane = threadIdx.x & 63;
    RescueReq *rq = reinterpret_cast<RescueReq *>(A.rescue);
    for (int t = lane; t < nT; t += 64) st_coh(&rq->ti[t], (uint64_t)(int64_t)ti[t]);
    if (lane == 0) {
        st_coh(&rq->rc, (uint64_t)rc);
        st_coh(&rq->rm, (uint64_t)rm);
        st_coh(&rq->rp, (uint64_t)rp);
        st_coh(&rq->sel, sel);
        st_coh(&rq->nT, (uint64_t)nT);
    }
    drain_stores();  // every store of the request, before the request number
    const unsigned long long q = (unsigned long long)A.loc->rseq + 1ull;
    lds_order();
    int ok = 1;
    if (lane == 0) {
        A.loc->rseq = (int64_t)q;
        __hip_atomic_store(&A.ctl->rescue_req.v, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned long long seen = 0;
        const uint64_t t0 = A.trace_row ? wall_clock64() : 0;
        ok = poll_ge(&A.ctl->rescue_done.v, q * (unsigned long long)A.rescue_n, A.timeout_ticks, &A.ctl->polls_rmw,
                     &seen) ? 1 : 0;
        if (A.trace_row) A.trace_row[17] += wall_clock64() - t0;  // time the rescues kept the commit waiting
        if (!ok) atomicCAS(A.err, 0, 12);
    }
    ok = __builtin_amdgcn_readfirstlane(ok);
    if (!ok) return false;
    const Rec *res = reinterpret_cast<const Rec *>(A.rescue + kRescueResOff);
    double k = -__builtin_inf();
    int32_t ix = kNoIdx, src = lane;
    uint64_t w[7] = {0, 0, 0, 0, 0, 0, 0};
    if (lane < A.rescue_n) {
        const uint64_t *rw = reinterpret_cast<const uint64_t *>(res + lane);
#pragma unroll
        for (int i = 0; i < 7; ++i) w[i] = ld_coh(rw + i);
        if ((uint32_t)(w[1] >> 32) != 0) { k = __longlong_as_double((long long)w[0]); ix = (int32_t)(uint32_t)w[1]; }
    }
    wave_argbest(k, ix, src);
    o->key = k;
    o->idx = ix;
    for (int r = 0; r < 3; ++r) o->a[r] = rl64((int64_t)w[2 + r], src);
    o->labels = (uint64_t)rl64((int64_t)w[5], src);
    o->price = __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)w[6], src));
    if (A.xp && A.xp->R > 1) return rescue_rank_fold(*A.xp, q, A.timeout_ticks, A.err, o);
    return true;
}

}  // namespace

// One batch's ordered commit by the whole workgroup (kSpcThreads).  COH: the lists arrive from other
// workgroups of a running persistent kernel (sc1 loads), and what the score workgroups read back --
// the XBuf export, the next plans, the cursor -- leaves as sc1 stores (ksched_persist.hip).
// a batch's pod requests, lane = pod (loaded early by the persistent commit, before its wait)
struct LanePods {
    int64_t rc, rm, rp;
    uint64_t sel;
};

template <bool LAB>
__device__ __forceinline__ LanePods load_lane_pods(const PodArgs &pods, int64_t p0, int nb) {
    const int lane = threadIdx.x & 63;
    const bool pj = lane < nb;
    LanePods q;
    q.rc = pj ? pods.rc[p0 + lane] : 0;
    q.rm = pj ? pods.rm[p0 + lane] : 0;
    q.rp = pj ? pods.rp[p0 + lane] : 0;
    q.sel = (LAB && pj) ? pods.sel[p0 + lane] : 0;
    return q;
}

struct NoWait {
    __device__ bool operator()() const { return true; }
};
// The persistent pipeline's hand-off from commit(b - 1) (the other commit workgroup) to commit(b): called by every
// thread; waits until commit(b - 1) has published, then returns what it left (0), the end of the call (1) or a
// timeout (-1), and to lane e < n1 of wave 0 entry e of export(b - 1).  The stream pipeline's single commit kernel
// needs none.
struct HandoffRes {
    int64_t cursor;     // first unresolved pod after commit(b - 1)
    int64_t plan_next;  // the plan of batch b + kPipeLag - 1, set by commit(b - 1)
    int64_t rseq;       // rescue requests issued so far in the call
    int32_t n1;         // entries of export(b - 1)
    int32_t pad;
};
struct NoHandoff {
    __device__ int operator()(HandoffRes *, XRec *) const { return 0; }
};
// commit(b)'s hand-off record for commit(b + 1) (one lane), behind a drain of every store of commit(b): both granules
// and every chunk of the export it announces carry the tag, and commit(b + 1) polls them all in one round of loads
__device__ __forceinline__ void put_handoff(Ctl *ctl, int64_t batch, int n1, int64_t cursor, int64_t rseq, int64_t plan_next) {
    const __amdgpu_buffer_rsrc_t r = coh_rsrc(&ctl->hrec);
    const uint32_t tag = (uint32_t)(batch + 1);
    st_coh16(r, 0, u32x4{tag, (uint32_t)n1, (uint32_t)(uint64_t)cursor, (uint32_t)((uint64_t)cursor >> 32)});
    st_coh16(r, 16, u32x4{tag, (uint32_t)rseq, (uint32_t)(uint64_t)plan_next, (uint32_t)((uint64_t)plan_next >> 32)});
}

// wait(): called by every thread once the work that needs no candidate list is done (the persistent
// commit waits there for the batch's merges); false = give up (the caller reports the timeout).
// Returns 1 done, 0 error (a wait timed out), 2 the call ended elsewhere (persistent pipeline: stop quietly).
template <int K, int PRIO, int DOM, bool LAB, bool F53, bool COH, int NT = kSpcThreads, typename Wait = NoWait,
          typename Handoff = NoHandoff>
__device__ __forceinline__ int commit_spc_batch(const CommitArgs &A, char *smem, const LanePods *pre = nullptr,
                                                Wait wait = Wait{}, Handoff handoff = Handoff{}) {
    constexpr int kSpcWaves = NT / 64;
    constexpr int kSpcThreads = NT;
    constexpr bool LAG3 = COH;  // the persistent pipeline runs at lag kPipeLag = 3
    constexpr bool SCR = COH && PRIO != kPrioPrice;  // the touched-node screen (above; KSCHED_NO_TOUCH_SCREEN=1 at run time)
    static_assert(!COH || kPipeLag == 3, "commit_spc_batch: the persistent pipeline's inheritance is lag 3");
    constexpr int kSpcRow = spc_slots<LAG3>() + 1;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    PersistLocal *const L = A.loc;
    const int64_t p0 = COH ? L->plan[A.batch % kPlanRing] : load_i64<COH>(A.plan);
    if constexpr (COH) {
        if (p0 < 0 || p0 >= A.pods.p) {
            // nothing planned: after commit(b - 1), plan batch b + kPipeLag and publish.  An empty export is never
            // written: the ring slot keeps an older batch's tag, which score(b + 3) and the commits read as empty.
            // (An idle commit waits for no merge, so a store here could land under a score workgroup still
            // reading the slot's previous export: ADVICE r3.)
            if (!wait()) return 0;
            HandoffRes ho;
            XRec hx;
            const int hr = handoff(&ho, &hx);
            if (hr != 0) return hr < 0 ? 0 : 2;
            if (wave == 0) {
                if (lane == 0) {
                    L->cursor = ho.cursor;
                    L->plan[(A.batch + kPipeLag - 1) % kPlanRing] = ho.plan_next;
                    L->rseq = ho.rseq;
                    persist_plan(A, false, ho.cursor);
                    st_coh(A.cursor_at, (uint64_t)ho.cursor);
                    drain_stores();  // every store of this commit lands before its hand-off record (below)
                    put_handoff(A.ctl, A.batch, 0, ho.cursor, ho.rseq, L->plan[(A.batch + kPipeLag) % kPlanRing]);
                }
                publish_committed<COH>(A);
            }
            return 1;
        }
    } else {
        const int64_t cursor = load_i64<COH>(&A.ctl->cursor);
        if (p0 < 0 || p0 >= A.pods.p || p0 != cursor) {
            if (!wait()) return 0;
            // nothing to do, or a speculative batch invalidated by an earlier truncation: skip it
            if (wave == 0) {
                if (lane == 0) {
                    A.xout->count = 0;
                    if (p0 >= 0 && p0 < A.pods.p) add_i64<COH>(&A.ctl->stats[3], 1);
                    plan_after_commit<COH>(A, false, cursor);
                }
                publish_committed<COH>(A);
            }
            return 1;
        }
    }
    const bool dbg = A.dbg != nullptr;  // diagnostics build of the phase timing (KSCHED_COMMIT_STAMPS)
    uint64_t t_start = dbg ? __builtin_amdgcn_s_memtime() : 0;
    uint64_t t_pre = 0;
    uint64_t t_s1 = 0, t_s2 = 0, t_s3 = 0, t_mark = 0;
    SpcSmem m;
    {
        // every array but S below 64 KB: an LDS instruction's immediate offset (16 bits) then reaches it from one
        // per-lane (or per-index) address register -- with S first, each of the arrays above it needed an address
        // register of its own, which the compiler hoisted out of the batch loop and spilled
        char *p = smem;
        m.pbk = reinterpret_cast<double *>(p); p += (size_t)kSpcWaves * 64 * sizeof(double);
        m.pbx = reinterpret_cast<int64_t *>(p); p += (size_t)kSpcWaves * 64 * sizeof(int64_t);
        m.LK = reinterpret_cast<double *>(p); p += (size_t)K * 64 * sizeof(double);
        m.GS = reinterpret_cast<uint64_t *>(p); p += 64 * kGS * sizeof(uint64_t);
        m.D = reinterpret_cast<int8_t *>(p); p += 64 * 64;
        m.T = reinterpret_cast<SpcSlot *>(p); p += (size_t)spc_slots<LAG3>() * sizeof(SpcSlot);
        m.LI = reinterpret_cast<int32_t *>(p); p += (size_t)K * 64 * sizeof(int32_t);
        m.HP = reinterpret_cast<int32_t *>(p); p += (size_t)K * 64 * sizeof(int32_t);
        m.hk = reinterpret_cast<int32_t *>(p); p += kSpcHash * sizeof(int32_t);
        m.tkc = reinterpret_cast<uint32_t *>(p); p += 64 * sizeof(uint32_t);
        m.ti = reinterpret_cast<int32_t *>(p); p += spc_slots<LAG3>() * sizeof(int32_t);
        m.fcg = reinterpret_cast<int32_t *>(p); p += 64 * sizeof(int32_t);
        m.dfacc = reinterpret_cast<int32_t *>(p); p += 64 * sizeof(int32_t);
        m.gn = reinterpret_cast<int32_t *>(p); p += 64 * sizeof(int32_t);
        m.gq = reinterpret_cast<int32_t *>(p); p += 64 * sizeof(int32_t);
        m.gs = reinterpret_cast<int32_t *>(p); p += 64 * sizeof(int32_t);
        m.ctl = reinterpret_cast<int32_t *>(p); p += 4 * sizeof(int32_t);
        m.thr = reinterpret_cast<float *>(p); p += 64 * sizeof(float);
        m.x2s = reinterpret_cast<int16_t *>(p); p += 64 * sizeof(int16_t);
        m.S = reinterpret_cast<double *>(p);
        m.own = reinterpret_cast<int32_t *>(m.pbk);
        m.s0 = reinterpret_cast<int64_t *>(m.D);
        m.iy = reinterpret_cast<double *>(m.GS);
    }
    const int nb = (int)((A.pods.p - p0 < A.B) ? A.pods.p - p0 : A.B);  // <= 64 (host-checked)
    // every wave: lane = pod j of the batch (lanes >= nb carry a zero request and are never read).
    // Issued before the prologue so these global loads overlap the list loads instead of following
    // them behind a barrier.
    const bool pj = lane < nb;
    const LanePods lp = pre ? *pre : load_lane_pods<LAB>(A.pods, p0, nb);
    const int64_t rc = lp.rc, rm = lp.rm, rp = lp.rp;
    const uint64_t sel = lp.sel;
    // the batch's candidate lists: fc0 and cut flag per pod, and every thread's list entries -- only
    // their (key, idx | valid) words, all loads in flight at once.  Lists that are ready at entry (the
    // stream pipeline) are loaded before the table initialisation so their latency overlaps it; the
    // persistent commit loads them after wait(), when the merges have published them.
    constexpr int kHeadPer = (64 * K + kSpcThreads - 1) / kSpcThreads;
    uint64_t w0[kHeadPer], w1[kHeadPer];
    int64_t fc0v = 0;
    int cut0 = 0;
    int32_t thr0 = 0;  // SCR: the list's screen threshold as f32 bits (entry 1's pad)
    auto load_lists = [&]() {
        fc0v = (wave == 0 && pj) ? load_i64<COH>(A.fc0 + lane) : 0;
        cut0 = (wave == 0 && pj) ? (int32_t)(uint32_t)(load_i64<COH>(
                                       reinterpret_cast<const int64_t *>(A.lists + (size_t)lane * K) + 6) >> 32) : 0;
        if (SCR)
            thr0 = (wave == 0 && pj) ? (int32_t)(uint32_t)(load_i64<COH>(
                                           reinterpret_cast<const int64_t *>(A.lists + (size_t)lane * K + 1) + 6) >> 32) : 0;
#pragma unroll
        for (int u = 0; u < kHeadPer; ++u) {
            const int e = tid + u * kSpcThreads;
            w0[u] = 0; w1[u] = 0;  // valid = 0
            if (e < 64 * K && e / K < nb) {
                const uint64_t *w = reinterpret_cast<const uint64_t *>(A.lists + e);
                if (COH) { w0[u] = ld_coh(w); w1[u] = ld_coh(w + 1); }
                else { w0[u] = w[0]; w1[u] = w[1]; }
            }
        }
    };
    if constexpr (!COH) load_lists();

    // ---- prologue ----
    int n1 = 0, n2 = 0, nin = 0;
    uint64_t dbg_x1 = 0;  // diagnostics (KSCHED_XCHG_DUMP, a KSCHED_XCHG_DEBUG build)
    (void)dbg_x1;
    const double rcf = (double)rc, rmf = (double)rm, rpf = (double)rp;
    const double y3 = recip(3.0);
    double *Srow = m.S + (size_t)lane * kSpcRow;
    uint64_t smv[3] = {0, 0, 0};  // COH: the merger's summary of this pod against the older export (wave 0)
    // keys of the newer inherited export's entries at their current state, predicate deltas against the entry's
    // start state s0, per-wave partial row bests; entry e -> slot sl(e)
    auto key_inherited = [&](int ne, auto sl) {
        int dfl = 0;
        double pk = -__builtin_inf();
        int32_t pi = kNoIdx, ps = -1;
        const float thrf = SCR ? m.thr[lane] : 0.0f;
        const float qc = screen_req(rc), qm = screen_req(rm), qp = screen_req(rp);
        int64_t nex = 0;
        for (int e = wave; e < ne; e += kSpcWaves) {
            const int t = sl(e);
            const SpcSlot &x = m.T[t];
            const int64_t *x0 = m.s0 + e * 3;
            const bool f0 = fits(rc, rm, rp, sel, x0[0], x0[1], x0[2], x.labels, LAB);
            const bool f1 = fits(rc, rm, rp, sel, x.cur[0], x.cur[1], x.cur[2], x.labels, LAB);
            dfl += (int)f1 - (int)f0;
            const double *yy = m.iy + e * 6;  // the entry's state as doubles and its reciprocals, staged once
            bool need = true;
            if constexpr (SCR) {
                bool lo;
                const float v = screen_pair(qc, qm, qp, screen_y(x.cur[0], yy[3]), screen_y(x.cur[1], yy[4]),
                                            screen_y(x.cur[2], yy[5]), x.cur[0] >= rc, x.cur[1] >= rm, x.cur[2] >= rp, &lo);
                need = pj && !(v < thrf);
            }
            double k;
            if (!SCR || __ballot(need) != 0) {
                ++nex;
                const bool el = pair_key_fast<PRIO, DOM, F53>(f1, rc, rm, rp, rcf, rmf, rpf, x.cur[0], x.cur[1], x.cur[2],
                                                              yy[0], yy[1], yy[2], yy[3], yy[4], yy[5], y3, x.price, &k);
                k = el ? k : -__builtin_inf();
            } else {
                k = skip_key();
            }
            Srow[t] = k;
            const bool up = k != -__builtin_inf() && better(k, x.idx, pk, pi);
            pk = up ? k : pk; pi = up ? x.idx : pi; ps = up ? t : ps;
        }
        m.pbk[wave * 64 + lane] = pk;
        m.pbx[wave * 64 + lane] = ((int64_t)ps << 32) | (uint32_t)pi;
        if (dfl != 0) atomicAdd(&m.dfacc[lane], dfl);
        if (SCR && A.dbg && lane == 0 && wave < ne) {  // diagnostics: entries keyed, exactly
            atomicAdd(reinterpret_cast<unsigned long long *>(&A.dbg[16]), (unsigned long long)((ne - 1 - wave) / kSpcWaves + 1));
            atomicAdd(reinterpret_cast<unsigned long long *>(&A.dbg[17]), (unsigned long long)nex);
        }
    };
    // the batch's candidate lists -> LK / LI and their table positions HP
    auto hash_lists = [&]() {
#pragma unroll
        for (int u = 0; u < kHeadPer; ++u) {
            const int e = tid + u * kSpcThreads;
            if (e < 64 * K) {
                const int j = e / K, q = e % K;
                const bool v = (uint32_t)(w1[u] >> 32) != 0;
                const double key = v ? __longlong_as_double((long long)w0[u]) : -__builtin_inf();
                const int32_t idx = v ? (int32_t)(uint32_t)w1[u] : kNoIdx;
                m.LK[q * 64 + j] = key;
                m.LI[q * 64 + j] = idx;
                m.HP[q * 64 + j] = idx == kNoIdx ? kSpcInvalid : spc_pos_insert(m.hk, idx);
            }
        }
    };
    if constexpr (!COH) {
        // ---- the stream pipeline (lag 2): slots [0, n1) = the previous batch's commits, s0 = their start state
        // (= this batch's snapshot) ----
        n1 = A.xin->count;  // <= 64
        XRec xi{};
        if (wave == 0 && lane < n1) xi = load_xrec<COH>(A.xin->e, lane);
        for (int w = tid; w < kSpcHash; w += kSpcThreads) m.hk[w] = -1;
        if (tid < 64) { m.dfacc[tid] = 0; m.fcg[tid] = 0; m.tkc[tid] = tid == (kSpcInvalid >> 5) ? (1u << (kSpcInvalid & 31)) : 0u; }
        __syncthreads();
        if (wave == 0 && lane < n1) {
            SpcSlot &x = m.T[lane];
            x.idx = xi.idx; x.mine = 0;
            for (int r = 0; r < 3; ++r) { m.s0[lane * 3 + r] = xi.sb[r]; x.sb[r] = xi.cur[r]; x.cur[r] = xi.cur[r]; }
            x.labels = xi.labels; x.price = xi.price; x.pad = 0;
            m.ti[lane] = xi.idx;
            stage_state(m.iy + lane * 6, xi.cur);
            const int h = spc_pos_insert(m.hk, xi.idx);
            atomicOr(&m.tkc[h >> 5], 1u << (h & 31));
        }
        nin = n1;
        __syncthreads();
        key_inherited(n1, [](int e) { return e; });
        if (!wait()) return 0;
        hash_lists();
        __syncthreads();
    } else {
        // ---- the persistent pipeline (lag 3; two commit workgroups alternate batches).  P1, while the other
        // workgroup commits batch b - 1: the tables, the slots of export(b - 2) -- this workgroup's own previous
        // batch --, the batch's lists and the mergers' keys of export(b - 2).  Then the hand-off from commit(b - 1)
        // and P2: export(b - 1)'s slots and keys ----
        {
            const uint64_t hdr = A.batch >= 2 ? ld_coh(&A.xin2->count) : 0ull;
            n2 = (A.batch >= 2 && (uint32_t)(hdr >> 32) == (uint32_t)(A.batch - 2)) ? (int)(uint32_t)hdr : 0;
        }
        XRec xi{};
        if (wave == 1 && lane < n2) xi = load_xrec<COH>(A.xin2->e, lane);
        for (int w = tid; w < kSpcHash; w += kSpcThreads) m.hk[w] = -1;
        if (tid < 64) { m.dfacc[tid] = 0; m.fcg[tid] = 0; m.tkc[tid] = tid == (kSpcInvalid >> 5) ? (1u << (kSpcInvalid & 31)) : 0u; }
        __syncthreads();
        // slots [0, n2) = export(b - 2) in entry order (a node export(b - 1) also holds is superseded in P2); own[]
        // (free until the guess step) maps their table positions to their slots
        if (wave == 1) {
            m.x2s[lane] = lane < n2 ? (int16_t)lane : (int16_t)-1;
            if (lane < n2) {
                SpcSlot &x = m.T[lane];
                x.idx = xi.idx; x.mine = 0;
                for (int r = 0; r < 3; ++r) { x.sb[r] = xi.cur[r]; x.cur[r] = xi.cur[r]; }
                x.labels = xi.labels; x.price = xi.price; x.pad = 0;
                m.ti[lane] = xi.idx;
                const int h = spc_pos_insert(m.hk, xi.idx);
                m.own[h] = lane;
                atomicOr(&m.tkc[h >> 5], 1u << (h & 31));
            }
        }
        if (dbg) {
            t_pre = __builtin_amdgcn_s_memtime() - t_start;
            if (lane == 0 && wave != 0) atomicAdd(reinterpret_cast<unsigned long long *>(&A.dbg[9]), (unsigned long long)t_pre);
        }
        if (!wait()) return 0;  // the batch's merges (a workgroup barrier)
        if (dbg) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            if (tid == 0) A.dbg[7] += t - t_start;  // entry -> past the merges' wait (wave 0)
            t_start = t;
        }
        load_lists();
        if (wave == 0 && A.batch >= 2 && n2 > 0 && pj) {
            const uint64_t *sm = reinterpret_cast<const uint64_t *>(A.inh + ((size_t)(A.batch % 4) * A.B + lane) * 32);
            smv[0] = ld_coh(sm); smv[1] = ld_coh(sm + 1); smv[2] = ld_coh(sm + 2);
        }
        // the mergers' key columns of export(b - 2): element (pod j, entry e) of inh keys[batch % 4] -> S[j][e]
        constexpr int kX2Per = 64 * 64 / kSpcThreads + (64 * 64 % kSpcThreads != 0);
        double x2v[kX2Per];
        const double *x2col = reinterpret_cast<const double *>(A.inh + (size_t)4 * A.B * 32) + (size_t)(A.batch % 4) * A.B * 64;
#pragma unroll
        for (int u = 0; u < kX2Per; ++u) {
            const int i = tid + u * kSpcThreads;
            x2v[u] = (i < 64 * 64 && (i & 63) < n2 && (i >> 6) < nb) ? ld_coh_f64(x2col + i) : 0.0;
        }
#if KSCHED_XCHG_DEBUG
        if (A.xp && A.xp->xdbg && A.dbg_act >= 0 && A.dbg_act < A.xp->xdbg_cap) {  // diagnostics: the lists as loaded
            uint64_t *sums = A.xp->xdbg + xdbg_sums_off(A.xp->xdbg_cap, A.xp->B, A.xp->R, K);
#pragma unroll
            for (int u = 0; u < kHeadPer; ++u) {
                const int e = tid + u * kSpcThreads;
                if (e < 64 * K && e / K < nb)
                    atomicAdd(reinterpret_cast<unsigned long long *>(sums + ((size_t)A.dbg_act * A.xp->B + e / K) * 2 + 1),
                              (unsigned long long)dbg_mix(w0[u], w1[u], e % K));
            }
        }
#endif
        hash_lists();
#pragma unroll
        for (int u = 0; u < kX2Per; ++u) {
            const int i = tid + u * kSpcThreads;
            if (i < 64 * 64 && (i & 63) < n2 && (i >> 6) < nb) m.S[(size_t)(i >> 6) * kSpcRow + (i & 63)] = x2v[u];
        }
        // the touched-node screen's thresholds: the mergers' (list_thr_bits, entry 1's pad); the hand-off's barrier
        // publishes them
        if (SCR && wave == 0) m.thr[lane] = (pj && A.touch_screen) ? __uint_as_float((uint32_t)thr0) : -__builtin_inff();
        // ---- the hand-off: commit(b - 1) published (a workgroup barrier) ----
        // (wave 0 lane e < n1 receives entry e of export(b - 1) with the record: the same round of loads)
        if (A.xp) jitter_at(A.xp->jitter, A.batch, 103);  // P1 done late
        HandoffRes ho;
        const int hr = handoff(&ho, &xi);
        if (hr != 0) return hr < 0 ? 0 : 2;  // timed out / the end of the call (or another workgroup's error)
        if (tid == 0) {
            L->cursor = ho.cursor;
            L->plan[(A.batch + kPipeLag - 1) % kPlanRing] = ho.plan_next;  // set by commit(b - 1)
            L->rseq = ho.rseq;
        }
        if (p0 != ho.cursor) {  // speculative batch invalidated by a truncation in commit(b - 1): skip it
            if (wave == 0) {
                if (lane == 0) {
                    __hip_atomic_fetch_add(reinterpret_cast<unsigned long long *>(&A.ctl->stats[3]), 1ull,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    persist_plan(A, false, ho.cursor);
                    st_coh(A.cursor_at, (uint64_t)ho.cursor);
                    drain_stores();  // every store of this commit lands before its hand-off record (below)
                    put_handoff(A.ctl, A.batch, 0, ho.cursor, ho.rseq, L->plan[(A.batch + kPipeLag) % kPlanRing]);
                }
                publish_committed<COH>(A);
            }
            return 1;
        }
        n1 = ho.n1;
#if KSCHED_XCHG_DEBUG
        if (A.xp && A.xp->xdbg && wave == 0) {  // diagnostics: export(b - 1) as received
            int64_t x = lane < n1 ? (int64_t)dbg_mix((uint64_t)xi.idx ^ ((uint64_t)xi.cur[0] << 20), (uint64_t)xi.cur[1] ^
                                                     (uint64_t)xi.cur[2] ^ (uint64_t)xi.sb[0], lane) : 0;
            x = wave_sum_i64(x);
            dbg_x1 = (uint64_t)x;
        }
#endif
        // P2: export(b - 1).  A node export(b - 2) holds too keeps that slot (its state and key superseded: x2s = -1);
        // the others take slots [n2, nin)
        if (wave == 0) {
            int h = 0;
            bool dup = false;
            if (lane < n1) {
                h = spc_pos_insert(m.hk, xi.idx);
                dup = (m.tkc[h >> 5] >> (h & 31)) & 1u;  // only export(b - 2)'s slots are taken yet
            }
            const uint64_t nm = __ballot(lane < n1 && !dup);
            const int slot = dup ? m.own[h] : n2 + __popcll(nm & ((1ull << lane) - 1ull));
            if (lane < n1) {
                SpcSlot &x = m.T[slot];
                x.idx = xi.idx; x.mine = 0;
                for (int r = 0; r < 3; ++r) { m.s0[lane * 3 + r] = xi.sb[r]; x.sb[r] = xi.cur[r]; x.cur[r] = xi.cur[r]; }
                x.labels = xi.labels; x.price = xi.price; x.pad = 0;
                m.ti[slot] = xi.idx;
                m.gs[lane] = slot;  // (gs is the guess step's; free until then)
                stage_state(m.iy + lane * 6, xi.cur);
                if (dup) m.x2s[slot] = -1;
                else atomicOr(&m.tkc[h >> 5], 1u << (h & 31));
            }
            if (lane == 0) m.ctl[3] = n2 + __popcll(nm);
        }
        __syncthreads();
        if (tid == 0 && A.trace_row) A.trace_row[23] = wall_clock64();  // export(b - 1) in its slots
        nin = m.ctl[3];
        key_inherited(n1, [&](int e) { return (int)m.gs[e]; });
        __syncthreads();
        if (tid == 0 && A.trace_row) A.trace_row[24] = wall_clock64();  // its keys
    }

    // ---- wave 0 state: lane j = pod j ----
    int32_t fcc = 0;          // predicate count with the confirmed commits
    double rbk = -__builtin_inf();  // best confirmed touched slot (key, node, slot)
    int32_t rbi = kNoIdx, rbs = -1;
    int cv = 0, cut = 0;      // list length, cut flag
    int32_t my_idx = 0, my_feas = 0;
    int32_t my_src = 0;  // diagnostics: the path that set my_idx (reported with device error 14)
    double my_score = 0.0;
    int32_t my_g = -2, my_q = -1, my_s = -1, my_h = kSpcInvalid;
    int nT = nin, done = nb, W = 64;
    int nresc = 0;  // wave 0: rescues of this batch
    // wave 0: quarter rescues this batch may spend -- the persistent commit's bucket refills by rescue_rate per
    // batch of this workgroup up to 4 * rescue_max, so exhausted lists are rescued where they are rare and
    // truncate early where they cluster (the rescues of a batch that truncates anyway are wasted)
    // and a batch may spend rescue_max of them while the bucket is at least half full, rescue_low below that
    int rcredit = 0, rmax = 0;
    if constexpr (COH) {
        const int c = A.loc->rescue_credit + A.rescue_rate;
        rcredit = c < 4 * A.rescue_cap ? c : 4 * A.rescue_cap;
        rmax = rcredit >= 2 * A.rescue_cap ? A.rescue_max : A.rescue_low;
    }
    int64_t placed = 0, nrounds = 0, nfail = 0, niters = 0, nseq = 0;
    if (wave == 0) {
        int64_t ds2 = 0;
        double xk = -__builtin_inf();
        int32_t xix = kNoIdx, xe = -1;
        if (LAG3 && A.batch >= 2 && n2 > 0 && pj) {  // the merger's summary: {sum of deltas, best key, idx | entry}
            ds2 = (int64_t)smv[0];
            xk = __longlong_as_double((long long)smv[1]);
            xix = (int32_t)(uint32_t)smv[2];
            xe = (int32_t)(smv[2] >> 32);
        }
        fcc = pj ? (int32_t)(fc0v + m.dfacc[lane] + ds2) : 0;
        cut = cut0;
#pragma unroll
        for (int q = 0; q < K; ++q) cv += m.LI[q * 64 + lane] != kNoIdx;  // valid entries form a prefix
        for (int w = 0; w < kSpcWaves; ++w) {
            const double k = m.pbk[w * 64 + lane];
            const int64_t x = m.pbx[w * 64 + lane];
            const int32_t xi = (int32_t)(uint32_t)x;
            if (k != -__builtin_inf() && better(k, xi, rbk, rbi)) { rbk = k; rbi = xi; rbs = (int32_t)(x >> 32); }
        }
        if (LAG3 && xix != kNoIdx) {
            if (m.x2s[xe] >= 0) {  // the best entry has a slot of its own
                if (better(xk, xix, rbk, rbi)) { rbk = xk; rbi = xix; rbs = m.x2s[xe]; }
            } else {
                // its node is also in the newer export, whose current state superseded this key: the best of the
                // entries that keep a slot of their own, from the mergers' key column
                for (int e = 0; e < n2; ++e) {
                    if (m.x2s[e] < 0) continue;
                    const double k = Srow[m.x2s[e]];
                    const int32_t xi = m.ti[m.x2s[e]];
                    if (k != -__builtin_inf() && better(k, xi, rbk, rbi)) { rbk = k; rbi = xi; rbs = m.x2s[e]; }
                }
            }
        }
        if (lane == 0) { m.ctl[0] = 0; m.ctl[2] = 0; }
    }

    // wave 0: pod f's exact best touched slot, its screened-out slots re-keyed (the rescue compares below the last
    // list entry); (wk, wi, s) holds the best of the slots it keyed exactly
    auto rekey_row = [&](int f, double &wk, int32_t &wi, int &s) {
        const int64_t fc = rl64(rc, f), fm = rl64(rm, f), fp = rl64(rp, f);
        const uint64_t fs = (uint64_t)rl64((int64_t)sel, f);
        const double fcf = (double)fc, fmf = (double)fm, fpf = (double)fp;
        double *row = m.S + (size_t)f * kSpcRow;
        int64_t nrk = 0;
        for (int t0 = 0; t0 < nT; t0 += 64) {
            const int t = t0 + lane;
            double k = -__builtin_inf();
            int32_t x = kNoIdx, ts_ = t;
            if (t < nT && row[t] != row[t]) {  // skipped
                const SpcSlot &y = m.T[t];
                const bool fy = fits(fc, fm, fp, fs, y.cur[0], y.cur[1], y.cur[2], y.labels, LAB);
                k = lane_key<PRIO, DOM, LAB, F53>(fy, fc, fm, fp, fcf, fmf, fpf, y.cur[0], y.cur[1], y.cur[2], y3, y.price);
                row[t] = k;
                x = k != -__builtin_inf() ? y.idx : kNoIdx;
                ++nrk;
            }
            wave_argbest_fast(k, x, ts_);
            if (x != kNoIdx && better(k, x, wk, wi)) { wk = k; wi = x; s = ts_; }
        }
        if (A.dbg && lane == 0) atomicAdd(reinterpret_cast<unsigned long long *>(&A.dbg[22]), 1ull);
        (void)nrk;
    };
    int c = 0;
    if (COH && tid == 0 && A.trace_row) A.trace_row[25] = wall_clock64();  // the rounds start
    uint64_t *const tr1 = (COH && tid == 0) ? A.trace_row : nullptr;  // the first round's stamps (cols 49-51)
    bool first = true;
    const uint64_t t_pro = dbg ? __builtin_amdgcn_s_memtime() - t_start : 0;
    for (;;) {
        // ---- step 1 (wave 0): guesses for pods [c, cend) ----
        if (dbg) t_mark = __builtin_amdgcn_s_memtime();
        if (wave == 0) {
            const int cend = (c + W < nb) ? c + W : nb;
            // Guesses by fixpoint iteration, lane = pod: g_i = the first list entry of pod i that is neither
            // confirmed-taken nor proposed by a pod < i (own[pos] < i) in the previous iteration.  Pod i's
            // proposal is final once those of all pods < i are, so the fixpoint is reached after at most
            // (cend - c) + 1 iterations and equals the sequential greedy guess order; with first touches
            // the rule (99 %), it is reached after two.  The entries' table positions and the mask of those
            // not confirmed-taken are loaded once per round; an iteration probes own[] only.
            // own[] aliases pbk / pbx, which the wave-0 state (or the last check) just read as doubles: an LDS order
            // on both sides of its initialisation, so no load or store moves across it (the accesses differ in type)
            lds_order();
            for (int w = lane * 4; w < kSpcHash; w += 256) *reinterpret_cast<int4 *>(m.own + w) = make_int4(64, 64, 64, 64);
            lds_order();
            const uint64_t fitm = __ballot(fcc != 0);  // pods with a feasible node before this round
            const bool act = lane >= c && lane < cend && ((fitm >> lane) & 1);
            int32_t hp[K];
            uint32_t am = 0;
#pragma unroll
            for (int qq = 0; qq < K; ++qq) hp[qq] = m.HP[qq * 64 + lane];
#pragma unroll
            for (int qq = 0; qq < K; ++qq) {  // kSpcInvalid's table bit is always set: ends the list
                const int pos = hp[qq];
                am |= ((m.tkc[pos >> 5] >> (pos & 31)) & 1u) ? 0u : (1u << qq);
            }
            if (!act) am = 0;
            int32_t pq = -1, ph = kSpcInvalid;  // current proposal (list position, table position)
            for (int it = 0;; ++it) {
                ++niters;
                // the first entry not confirmed-taken and not proposed by an earlier pod: every probe of own[] in
                // flight at once (highest entry first, so the lowest match is the one kept), no branch per entry
                int32_t nq = -1, nh = kSpcInvalid;
                if (am) {
#pragma unroll
                    for (int qq = K - 1; qq >= 0; --qq) {
                        const bool ok = (((am >> qq) & 1u) != 0u) & (m.own[hp[qq]] >= lane);
                        nq = ok ? qq : nq;
                        nh = ok ? hp[qq] : nh;
                    }
                }
                const bool changed = __ballot(act && nq != pq) != 0;
                if (act && pq >= 0) m.own[ph] = 64;
                lds_order();
                pq = nq; ph = nh;
                if (!changed && it > 0) break;
                if (act && pq >= 0) atomicMin(&m.own[ph], lane);
                lds_order();
            }
            const uint64_t gm = __ballot(act && pq >= 0);
            if (lane >= c && lane < cend) {
                my_g = act ? (pq >= 0 ? 0 : -1) : -2;
                my_q = pq;
                my_h = act && pq >= 0 ? ph : kSpcInvalid;
                my_s = act && pq >= 0 ? nT + __popcll(gm & ((1ull << lane) - 1ull)) : -1;
            }
            const bool in = lane >= c && lane < cend;
            if (in && my_g == 0) my_g = m.LI[my_q * 64 + lane];  // the guessed node
            m.gn[lane] = in ? my_g : -2;
            m.gq[lane] = my_q;
            m.gs[lane] = my_s;
            m.fcg[lane] = 0;
            if (lane == 0) { m.ctl[0] = c; m.ctl[1] = cend; }
        }
        __syncthreads();
        if (first && tr1) tr1[49] = wall_clock64();  // the first guess step done
        if (dbg) { const uint64_t t = __builtin_amdgcn_s_memtime(); t_s1 += t - t_mark; t_mark = t; }
        const int rc0 = m.ctl[0], rce = m.ctl[1];
        // ---- step 2 (all waves): evaluate the guessed commits in parallel ----
        {
            double pk = -__builtin_inf();
            int32_t pi = kNoIdx, ps = -1;
            // the guessed entries' snapshot state and the state after the guessing pod's commit, with its
            // doubles and reciprocals, staged in LDS once per guess by the guessing pod's own lane (wave 0)
            if (wave == 0 && lane >= rc0 && lane < rce && m.gn[lane] >= 0) {
                const uint64_t *src = reinterpret_cast<const uint64_t *>(A.lists + (size_t)lane * K + m.gq[lane]) + 2;
                uint64_t v[5];
#pragma unroll
                for (int w = 0; w < 5; ++w) v[w] = COH ? ld_coh(src + w) : src[w];
                // commit of pod `lane`: used += request, ONE pod (anchor/predicate.go:99-102)
                const int64_t n0 = wsub((int64_t)v[0], rc), n1 = wsub((int64_t)v[1], rm), n2 = wsub((int64_t)v[2], 1);
                const double nf0 = (double)n0, nf1 = (double)n1, nf2 = (double)n2;
                uint64_t *o = m.GS + (size_t)lane * kGS;
#pragma unroll
                for (int w = 0; w < 5; ++w) o[w] = v[w];
                o[5] = (uint64_t)n0; o[6] = (uint64_t)n1; o[7] = (uint64_t)n2;
                o[8] = (uint64_t)__double_as_longlong(nf0); o[9] = (uint64_t)__double_as_longlong(nf1);
                o[10] = (uint64_t)__double_as_longlong(nf2);
                o[11] = (uint64_t)__double_as_longlong(recip_or_zero(n0, nf0));
                o[12] = (uint64_t)__double_as_longlong(recip_or_zero(n1, nf1));
                o[13] = (uint64_t)__double_as_longlong(recip_or_zero(n2, nf2));
            }
            __syncthreads();
            const float thrf = SCR ? m.thr[lane] : 0.0f;
            const float qc = screen_req(rc), qm = screen_req(rm), qp = screen_req(rp);
            int64_t nev = 0, nex = 0;
            for (int k = rc0 + wave; k < rce; k += kSpcWaves) {
                const int32_t g = __builtin_amdgcn_readfirstlane(m.gn[k]);
                if (g < 0) continue;  // wave-uniform
                const int s = __builtin_amdgcn_readfirstlane(m.gs[k]);
                const uint64_t *gsk = m.GS + (size_t)k * kGS;
                const int64_t a0 = (int64_t)gsk[0], a1 = (int64_t)gsk[1], a2 = (int64_t)gsk[2];
                const uint64_t lab = gsk[3];
                const float pr = __uint_as_float((uint32_t)gsk[4]);
                const int64_t n0 = (int64_t)gsk[5], n1 = (int64_t)gsk[6], n2 = (int64_t)gsk[7];
                const bool fo = fits(rc, rm, rp, sel, a0, a1, a2, lab, LAB);
                const bool fn = fits(rc, rm, rp, sel, n0, n1, n2, lab, LAB);
                const int d = (int)fn - (int)fo;
                const double ny0 = __longlong_as_double((long long)gsk[11]), ny1 = __longlong_as_double((long long)gsk[12]),
                             ny2 = __longlong_as_double((long long)gsk[13]);
                bool need = true;
                if constexpr (SCR) {  // only the pods after the guessing one use its column
                    bool lo;
                    const float v = screen_pair(qc, qm, qp, screen_y(n0, ny0), screen_y(n1, ny1), screen_y(n2, ny2),
                                                n0 >= rc, n1 >= rm, n2 >= rp, &lo);
                    need = lane > k && pj && !(v < thrf);
                }
                double kv;
                ++nev;
                if (!SCR || __ballot(need) != 0) {
                    ++nex;
                    const bool el = pair_key_fast<PRIO, DOM, F53>(
                        fn, rc, rm, rp, rcf, rmf, rpf, n0, n1, n2, __longlong_as_double((long long)gsk[8]),
                        __longlong_as_double((long long)gsk[9]), __longlong_as_double((long long)gsk[10]), ny0, ny1, ny2,
                        y3, pr, &kv);
                    kv = el ? kv : -__builtin_inf();
                } else {
                    kv = skip_key();
                }
                Srow[s] = kv;
                m.D[k * 64 + lane] = (int8_t)d;
                if (lane > k) {
                    if (d != 0) atomicAdd(&m.fcg[lane], d);
                    const bool up = kv != -__builtin_inf() && better(kv, g, pk, pi);
                    pk = up ? kv : pk; pi = up ? g : pi; ps = up ? s : ps;
                }
                if (lane == 0) {
                    SpcSlot &x = m.T[s];
                    x.idx = g; x.mine = 1;
                    x.sb[0] = a0; x.sb[1] = a1; x.sb[2] = a2;  // untouched before this batch
                    x.cur[0] = n0; x.cur[1] = n1; x.cur[2] = n2;
                    x.labels = lab; x.price = pr; x.pad = 0;
                    m.ti[s] = g;
                }
            }
            m.pbk[wave * 64 + lane] = pk;
            m.pbx[wave * 64 + lane] = ((int64_t)ps << 32) | (uint32_t)pi;
            if (SCR && A.dbg && lane == 0 && nev) {  // diagnostics: guessed columns keyed, exactly
                atomicAdd(reinterpret_cast<unsigned long long *>(&A.dbg[18]), (unsigned long long)nev);
                atomicAdd(reinterpret_cast<unsigned long long *>(&A.dbg[19]), (unsigned long long)nex);
            }
        }
        __syncthreads();
        if (first && tr1) tr1[50] = wall_clock64();  // its evaluation done
        if (dbg) { const uint64_t t = __builtin_amdgcn_s_memtime(); t_s2 += t - t_mark; t_mark = t; }
        // ---- step 3 (wave 0): check, confirm the valid prefix, resolve the first failure ----
        if (wave == 0) {
            ++nrounds;
            const int cend = rce;
            // t* = best of the confirmed slots and of the guessed commits before this pod
            double tk = rbk;
            int32_t ti = rbi, ts = rbs;
            for (int w = 0; w < kSpcWaves; ++w) {
                const double k = m.pbk[w * 64 + lane];
                const int64_t x = m.pbx[w * 64 + lane];
                const int32_t xi = (int32_t)(uint32_t)x;
                const bool up = k != -__builtin_inf() && better(k, xi, tk, ti);
                tk = up ? k : tk; ti = up ? xi : ti; ts = up ? (int32_t)(x >> 32) : ts;
            }
            const bool has_t = ti != kNoIdx;
            const int32_t fcj = fcc + m.fcg[lane];
            // kind: 0 no placement, 1 the guess (first touch), 2 t*, 3 overflow, 4 guess unknown (re-probe)
            int kind;
            double uk = -__builtin_inf();
            if (fcj == 0) {
                kind = 0;
            } else if (my_g >= 0) {
                uk = m.LK[my_q * 64 + lane];
                kind = (has_t && better(tk, ti, uk, my_g)) ? 2 : 1;
            } else if (my_g == -2) {
                kind = 4;  // predicted no fit, but a node fits: u* was never looked up
            } else if (!cut) {
                kind = has_t ? 2 : 0;
            } else if (cv > 0) {
                const double lk = m.LK[(cv - 1) * 64 + lane];
                const int32_t lx = m.LI[(cv - 1) * 64 + lane];
                kind = (has_t && better(tk, ti, lk, lx)) ? 2 : 3;
            } else {
                kind = 3;  // unreachable: a cut list keeps at least its cutoff entry
            }
            const bool guessed_commit = my_g >= 0;
            const bool valid = (kind == 0 && !guessed_commit) || (kind == 1);
            const bool inw = lane >= c && lane < cend;
            const uint64_t bad = __ballot(inw && !valid);
            int f = bad ? (int)__builtin_ctzll(bad) : cend;
            // confirm [c, f)
            const bool conf = lane >= c && lane < f;
            if (conf) {
                my_idx = kind == 1 ? my_g : (fcj == 0 ? -1 : -2);
                my_src = 1 + kind + 8 * my_q;
                my_score = kind == 1 ? (PRIO == kPrioPrice ? 0.0 - uk : uk) : 0.0;
                my_feas = fcj;
                if (guessed_commit) atomicOr(&m.tkc[my_h >> 5], 1u << (my_h & 31));
            }
            placed += __popcll(__ballot(conf && kind == 1));
            const int ncg = __popcll(__ballot(conf && guessed_commit));
            nT += ncg;
            if (f < nb) {
                // bring the confirmed state of the pods still to come up to date with [c, f)
                for (int k = c; k < f; ++k) {
                    const int32_t g = __builtin_amdgcn_readlane(my_g, k);
                    if (g < 0) continue;
                    const int s = __builtin_amdgcn_readlane(my_s, k);
                    const double v = Srow[s];
                    fcc += m.D[k * 64 + lane];
                    const bool up = v != -__builtin_inf() && better(v, g, rbk, rbi);
                    rbk = up ? v : rbk; rbi = up ? g : rbi; rbs = up ? s : rbs;
                }
            }
            if (f < cend) {
                ++nfail;
                // resolve pod f exactly (its inputs are exact: every pod before it is confirmed)
                int kf = __builtin_amdgcn_readlane(kind, f);
                int32_t fcf = __builtin_amdgcn_readlane(fcj, f);
                double wk = readlane_f64(tk, f);
                int32_t wi = __builtin_amdgcn_readlane(ti, f);
                int s = __builtin_amdgcn_readlane(ts, f);
                const int fr = f;  // the round's first failure
                // A pod whose answer is a node the batch already touched (kind 2) made the guesses after it
                // void; where that happens pods tend to follow the same node, so the pods after it are resolved
                // one by one here (the same exact step, the probe of kind 4) for as long as their answers keep
                // being touched nodes, instead of a guess round (all waves, ~15 us) per pod.  A first touch or
                // an overflow hands back to the guess rounds.
                for (;;) {
                int qf = -1;
                if (kf == 4) {
                    // first list entry of pod f not in T (guesses before f are confirmed, later ones void)
                    const int cvf = __builtin_amdgcn_readlane(cv, f);
                    bool free_ = false;
                    int32_t e = kNoIdx;
                    if (lane < cvf) {
                        e = m.LI[lane * 64 + f];
                        const int pos = m.HP[lane * 64 + f];
                        free_ = !((m.tkc[pos >> 5] >> (pos & 31)) & 1u);
                    }
                    const uint64_t fm = __ballot(free_);
                    const bool ht = wi != kNoIdx;
                    if (fm) {
                        qf = __builtin_ctzll(fm);
                        const int32_t ue = __builtin_amdgcn_readlane(e, qf);
                        const double ukf = m.LK[qf * 64 + f];
                        if (ht && better(wk, wi, ukf, ue)) kf = 2;
                        else { kf = 1; wk = ukf; wi = ue; }
                    } else if (!__builtin_amdgcn_readlane(cut, f)) {
                        kf = ht ? 2 : 0;
                    } else if (cvf > 0) {
                        const double lk = m.LK[(cvf - 1) * 64 + f];
                        const int32_t lx = m.LI[(cvf - 1) * 64 + f];
                        kf = (ht && better(wk, wi, lk, lx)) ? 2 : 3;
                    } else {
                        kf = 3;
                    }
                }
                kf = __builtin_amdgcn_readfirstlane(kf);
                bool rescued = false;
                RescueOut ro{};
                if constexpr (COH) {
                    // the persistent commit (one rank) rescues an exhausted list instead of truncating the batch
                    bool afford = kf == 3 && A.rescue && nresc < rmax && 4 * (nresc + 1) <= rcredit;
                    if (afford && A.rescue_look) {
                        // look ahead: the later pods of the batch whose cut list is exhausted already (every entry a
                        // touched node).  When they would overrun the credit the batch truncates anyway -- a rescue
                        // before that truncation is wasted -- so it truncates here
                        bool risk = false;
                        if (lane > f && lane < nb && cut) {
                            risk = true;
#pragma unroll
                            for (int q = 0; q < K; ++q) {
                                if (q < cv) {
                                    const int pos = m.HP[q * 64 + lane];
                                    risk = risk && ((m.tkc[pos >> 5] >> (pos & 31)) & 1u);
                                }
                            }
                        }
                        const int n = nresc + 1 + __popcll(__ballot(risk));
                        afford = n <= rmax && 4 * n <= rcredit;
                    }
                    if (afford &&
                        commit_rescue(A, f, rl64(rc, f), rl64(rm, f), rl64(rp, f), (uint64_t)rl64((int64_t)sel, f),
                                      m.ti, nT, &ro)) {
                        ++nresc;
                        if (lane == 0) ++L->stats[4];
#if KSCHED_XCHG_DEBUG
                        if (A.xp && A.xp->xdbg && lane == 0 && nresc <= 4 && A.dbg_act >= 0 && A.dbg_act < A.xp->xdbg_cap) {
                            uint64_t *d = A.xp->xdbg + xdbg_commit_off(A.xp->xdbg_cap, A.xp->B, A.xp->R, K) +
                                          (size_t)A.xp->xdbg_cap * 8 + (size_t)A.dbg_act * 8 + 2 * (nresc - 1);
                            d[0] = (uint64_t)(uint32_t)f | (uint64_t)(uint32_t)ro.idx << 32;  // diagnostics: the rescue
                            d[1] = (uint64_t)__double_as_longlong(ro.key);
                        }
#endif
                        if constexpr (SCR) rekey_row(f, wk, wi, s);  // t* below the last entry: every slot counts
                        const bool ht = wi != kNoIdx;
                        if (ro.idx != kNoIdx && !(ht && better(wk, wi, ro.key, ro.idx))) {
                            kf = 1;  // a first touch of a node no candidate list held
                            rescued = true;
                            wk = ro.key;
                            wi = ro.idx;
                        } else {
                            kf = ht ? 2 : 0;
                        }
                    }
                }
                if (kf == 3) {
                    done = f;  // overflow: the batch stops before pod f
                } else {
                    if (lane == f) {
                        my_idx = kf == 0 ? (fcf == 0 ? -1 : -2) : wi;
                        my_src = 1000 + kf + (rescued ? 10 : 0) + 100 * (qf + 1) + 10000 * (int)(nseq & 63);
                        my_score = kf == 0 ? 0.0 : (PRIO == kPrioPrice ? 0.0 - wk : wk);
                        my_feas = fcf;
                    }
                    if (kf != 0) {
                        ++placed;
                        int64_t b0, b1, b2;
                        uint64_t lab;
                        float pr;
                        if (kf == 1 && rescued) {  // first touch of the rescued node
                            b0 = ro.a[0]; b1 = ro.a[1]; b2 = ro.a[2]; lab = ro.labels; pr = ro.price;
                            s = nT++;
                        } else if (kf == 1) {  // first touch of list entry qf
                            int64_t ra[3];
                            load_rec_state<COH>(A.lists + (size_t)f * K + qf, ra, &lab, &pr);
                            b0 = ra[0]; b1 = ra[1]; b2 = ra[2];
                            s = nT++;
                        } else {
                            const SpcSlot &x = m.T[s];
                            b0 = x.cur[0]; b1 = x.cur[1]; b2 = x.cur[2]; lab = x.labels; pr = x.price;
                        }
                        const int64_t n0 = wsub(b0, rl64(rc, f)), n1 = wsub(b1, rl64(rm, f)), n2 = wsub(b2, 1);
                        const bool fo = fits(rc, rm, rp, sel, b0, b1, b2, lab, LAB);
                        const bool fn = fits(rc, rm, rp, sel, n0, n1, n2, lab, LAB);
                        fcc += (int32_t)fn - (int32_t)fo;
                        double kv;
                        if constexpr (SCR) {  // the pods after f use this column
                            const double nf0 = (double)n0, nf1 = (double)n1, nf2 = (double)n2;
                            const double ny0 = recip_or_zero(n0, nf0), ny1 = recip_or_zero(n1, nf1),
                                         ny2 = recip_or_zero(n2, nf2);
                            bool lo;
                            const float v = screen_pair(screen_req(rc), screen_req(rm), screen_req(rp), screen_y(n0, ny0),
                                                        screen_y(n1, ny1), screen_y(n2, ny2), n0 >= rc, n1 >= rm, n2 >= rp,
                                                        &lo);
                            const bool need = lane > f && pj && !(v < m.thr[lane]);
                            const bool any = __ballot(need) != 0;
                            if (any) {
                                const bool el = pair_key_fast<PRIO, DOM, F53>(fn, rc, rm, rp, rcf, rmf, rpf, n0, n1, n2, nf0,
                                                                              nf1, nf2, ny0, ny1, ny2, y3, pr, &kv);
                                kv = el ? kv : -__builtin_inf();
                            } else {
                                kv = skip_key();
                            }
                            if (A.dbg && lane == 0) {  // diagnostics: sequential columns keyed, exactly
                                atomicAdd(reinterpret_cast<unsigned long long *>(&A.dbg[20]), 1ull);
                                if (any) atomicAdd(reinterpret_cast<unsigned long long *>(&A.dbg[21]), 1ull);
                            }
                        } else {
                            kv = lane_key<PRIO, DOM, LAB, F53>(fn, rc, rm, rp, rcf, rmf, rpf, n0, n1, n2, y3, pr);
                        }
                        Srow[s] = kv;
                        if (lane == 0) {
                            SpcSlot &x = m.T[s];
                            if (kf == 1) {
                                x.idx = wi;
                                x.sb[0] = b0; x.sb[1] = b1; x.sb[2] = b2;
                                x.labels = lab; x.price = pr; x.pad = 0;
                                m.ti[s] = wi;
                                const int pos = rescued ? spc_pos_insert(m.hk, wi) : m.HP[qf * 64 + f];
                                m.tkc[pos >> 5] |= 1u << (pos & 31);
                            }
                            x.mine = 1;
                            x.cur[0] = n0; x.cur[1] = n1; x.cur[2] = n2;
                        }
                        lds_order();
                        // running best: a better value takes over; a holder that got worse forces a rescan
                        const bool up = kv != -__builtin_inf() && better(kv, wi, rbk, rbi);
                        const bool rescan = !up && rbs == s;
                        rbk = up ? kv : rbk; rbi = up ? wi : rbi; rbs = up ? s : rbs;
                        if (__ballot(rescan)) {
                            if (rescan) {
                                // four slots' loads in flight, two running maxima (better() is a total order on
                                // distinct nodes, so the fold order does not change the result)
                                double k0 = -__builtin_inf(), k1 = -__builtin_inf();
                                int32_t i0 = kNoIdx, i1 = kNoIdx;
                                int s0 = -1, s1 = -1;
                                int t = 0;
                                for (; t + 4 <= nT; t += 4) {
                                    double v[4];
                                    int32_t x[4];
#pragma unroll
                                    for (int u = 0; u < 4; ++u) { v[u] = Srow[t + u]; x[u] = m.ti[t + u]; }
#pragma unroll
                                    for (int u = 0; u < 4; u += 2) {
                                        if (v[u] != -__builtin_inf() && better(v[u], x[u], k0, i0)) { k0 = v[u]; i0 = x[u]; s0 = t + u; }
                                        if (v[u + 1] != -__builtin_inf() && better(v[u + 1], x[u + 1], k1, i1)) {
                                            k1 = v[u + 1]; i1 = x[u + 1]; s1 = t + u + 1;
                                        }
                                    }
                                }
                                for (; t < nT; ++t) {
                                    const double v = Srow[t];
                                    const int32_t x = m.ti[t];
                                    if (v != -__builtin_inf() && better(v, x, k0, i0)) { k0 = v; i0 = x; s0 = t; }
                                }
                                if (k1 != -__builtin_inf() && better(k1, i1, k0, i0)) { k0 = k1; i0 = i1; s0 = s1; }
                                rbk = k0; rbi = i0; rbs = s0;
                            }
                        }
                    }
                }
                if (kf != 2 || f + 1 >= nb) break;
                // the next pod, exactly: every pod before it is resolved, rbk/fcc are current
                ++f;
                ++nseq;
                fcf = __builtin_amdgcn_readlane(fcc, f);
                kf = fcf == 0 ? 0 : 4;
                wk = readlane_f64(rbk, f);
                wi = __builtin_amdgcn_readlane(rbi, f);
                s = __builtin_amdgcn_readlane(rbs, f);
                }
                W = 2 * (fr - c + 1);
                W = W < 4 ? 4 : (W > 64 ? 64 : W);
                c = f + 1;
            } else {
                W = 2 * W > 64 ? 64 : 2 * W;
                c = cend;
            }
            if (lane == 0) { m.ctl[0] = c; m.ctl[2] = (done < nb || c >= nb) ? 1 : 0; }
        }
        __syncthreads();
        if (first && tr1) tr1[51] = wall_clock64();  // its check done
        first = false;
        if (dbg) { const uint64_t t = __builtin_amdgcn_s_memtime(); t_s3 += t - t_mark; t_mark = t; }
        if (m.ctl[2]) break;
        c = m.ctl[0];
    }
    if (wave != 0) return true;
    if (tr1) tr1[52] = wall_clock64();  // the rounds done

    auto store_out = [&]() {
        // an index no path of the commit can produce (a node index is < 2^30) is a device error, never an output
        const bool bad_out = COH && lane < done && (my_idx < -2 || my_idx >= (1 << 30));
        const uint64_t bm = __ballot(bad_out);
        if (bm) {
            const int l = (int)__builtin_ctzll(bm);
            const int src = __builtin_amdgcn_readlane(my_src, l);
            const int val = __builtin_amdgcn_readlane(my_idx, l);
            if (lane == 0 && atomicCAS(A.err, 0, 14) == 0 && A.xp && A.xp->prog) {  // the words the host reports
                A.xp->prog[kProgWords * (A.xp->G + A.xp->B) + 3] =
                    (uint64_t)A.batch << 40 | (uint64_t)l << 32 | (uint64_t)(uint32_t)src;
                A.xp->prog[kProgWords * (A.xp->G + A.xp->B) + 4] = (uint64_t)(uint32_t)val;
            }
        }
        if (lane < done) {
            A.out.idx[p0 + lane] = my_idx;
            A.out.score[p0 + lane] = my_score;
            A.out.feas[p0 + lane] = my_feas;
        }
    };
    if (!COH) store_out();
    // export this batch's commits (wave-ordered compaction)
    int base = 0;
    for (int t0 = 0; t0 < nT; t0 += 64) {
        const int t = t0 + lane;
        const bool mine = t < nT && m.T[t].mine;
        const uint64_t mask = __ballot(mine);
        if (mine) {
            const SpcSlot &x = m.T[t];
            XRec o;
            o.idx = x.idx; o.pad = 0;
            o.sb[0] = x.sb[0]; o.sb[1] = x.sb[1]; o.sb[2] = x.sb[2];
            o.cur[0] = x.cur[0]; o.cur[1] = x.cur[1]; o.cur[2] = x.cur[2];
            o.labels = x.labels; o.price = x.price; o.pad2 = 0;
            const int slot = base + __popcll(mask & ((1ull << lane) - 1));
            store_xrec<COH>(A.xout->e, slot, o, (uint32_t)(A.batch + 1));
        }
        base += __popcll(mask);
    }
#if KSCHED_XCHG_DEBUG
    if (COH && A.xp && A.xp->xdbg && A.dbg_act >= 0 && A.dbg_act < A.xp->xdbg_cap) {  // diagnostics: the outputs
        int64_t x = lane < done ? (int64_t)dbg_mix((uint64_t)(uint32_t)my_idx, (uint64_t)__double_as_longlong(my_score), lane) : 0;
        x = wave_sum_i64(x);
        if (lane == 0) A.xp->xdbg[xdbg_commit_off(A.xp->xdbg_cap, A.xp->B, A.xp->R, K) + (size_t)A.dbg_act * 8 + 3] = (uint64_t)x;
    }
#endif
    if (lane == 0) {
        if (COH) {
            st_coh(&A.xout->count, (uint64_t)(uint32_t)base | (uint64_t)(uint32_t)A.batch << 32);  // {count, tag}
            L->cursor = p0 + done;
            persist_plan(A, done < nb, p0 + done);
            st_coh(A.cursor_at, (uint64_t)L->cursor);  // (publish_committed<true> relies on this store and the drain)
            // every store of this commit -- the export, its {count, tag} header, the plan -- lands before the hand-off
            // record: commit(b + 1) may publish Ctl::committed = b + 2 before this workgroup publishes b + 1, and a
            // reader that sees b + 2 reads export(b) (round 5: without this drain a score workgroup could read the
            // header before it landed and skip a whole export)
            drain_stores();
            if (A.xp) jitter_at(A.xp->jitter, A.batch, 101);
            put_handoff(A.ctl, A.batch, base, L->cursor, L->rseq, L->plan[(A.batch + kPipeLag) % kPlanRing]);
            if (A.trace_row) A.trace_row[53] = wall_clock64();  // the hand-off record issued
        } else {
            A.xout->count = base;
            store_i64<COH>(&A.ctl->cursor, p0 + done);
            add_i64<COH>(&A.ctl->stats[0], 1);
            add_i64<COH>(&A.ctl->stats[1], (done < nb) ? 1 : 0);
            add_i64<COH>(&A.ctl->stats[2], placed);
            plan_after_commit<COH>(A, done < nb, p0 + done);
        }
#if KSCHED_XCHG_DEBUG
        if (COH && A.xp && A.xp->xdbg && A.dbg_act >= 0 && A.dbg_act < A.xp->xdbg_cap) {  // diagnostics
            uint64_t *d = A.xp->xdbg + xdbg_commit_off(A.xp->xdbg_cap, A.xp->B, A.xp->R, K) + (size_t)A.dbg_act * 8;
            d[0] = (uint64_t)p0;
            d[1] = (uint64_t)done | (uint64_t)nresc << 16 | (uint64_t)nrounds << 32 | (uint64_t)nfail << 48;
            d[2] = (uint64_t)n1 | (uint64_t)n2 << 16 | (uint64_t)nin << 32 | (uint64_t)base << 48;
            d[4] = dbg_x1;
            d[7] = (uint64_t)A.batch;
        }
#endif
        if (A.trace_row)  // rounds | rescues << 16 | resolved pods << 24 | failed guesses << 32 | pods resolved one by one << 48
            A.trace_row[16] = (uint64_t)nrounds | (uint64_t)nresc << 16 | (uint64_t)done << 24 | (uint64_t)nfail << 32 |
                              (uint64_t)nseq << 48;
        if (A.dbg) {
            A.dbg[12] += nrounds; A.dbg[13] += nfail; A.dbg[14] += 1; A.dbg[5] += niters;
            A.dbg[0] += t_pro; A.dbg[1] += t_s1; A.dbg[2] += t_s2; A.dbg[3] += t_s3;
            if (A.trace_row) { A.trace_row[18] = t_pro; A.trace_row[19] = t_s1; A.trace_row[20] = t_s2; A.trace_row[21] = t_s3; }
            A.dbg[4] += __builtin_amdgcn_s_memtime() - t_start;
            A.dbg[6] += t_pre;
        }
    }
    if (COH && A.xp) jitter_at(A.xp->jitter, A.batch, 102);
    publish_committed<COH>(A);  // wave 0 made every global store of this batch
    if (COH) {
        // persistent pipeline: the outputs, the cursor and the counters are read by the host after the kernel
        // (and by the next call's commit), by no workgroup of this one -- off the hand-off's critical path
        // (two commit workgroups: the counters are added, the cursor only grows)
        store_out();
        if (lane == 0) {
            unsigned long long *st = reinterpret_cast<unsigned long long *>(A.ctl->stats);
            __hip_atomic_fetch_max(reinterpret_cast<unsigned long long *>(&A.ctl->cursor), (unsigned long long)L->cursor,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(st + 0, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (done < nb) __hip_atomic_fetch_add(st + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(st + 2, (unsigned long long)placed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (nresc) __hip_atomic_fetch_add(st + 4, (unsigned long long)nresc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (threadIdx.x == 0) A.loc->rescue_credit = rcredit - 4 * nresc;
    }
    return 1;
}

// the arrays in front of S (SpcSmem's layout in commit_spc_batch)
template <int K, int NT = kSpcThreads, bool LAG3 = false>
constexpr size_t spc_small_bytes() {
    return (size_t)(NT / 64) * 64 * 16 + (size_t)K * 64 * 8 + 64 * kGS * 8 + 64 * 64 + spc_slots<LAG3>() * sizeof(SpcSlot) +
           (size_t)K * 64 * 8 + (size_t)kSpcHash * 4 + 64 * 4 + spc_slots<LAG3>() * 4 + 5 * 64 * 4 + 16 + 64 * 4 + 64 * 2;
}
template <int K, int NT = kSpcThreads, bool LAG3 = false>
constexpr size_t spc_lds_bytes() {
    return (size_t)64 * (spc_slots<LAG3>() + 1) * 8 + (size_t)(NT / 64) * 64 * 16 + (size_t)K * 64 * 12 +
           spc_slots<LAG3>() * sizeof(SpcSlot) + (size_t)kSpcHash * 4 + (size_t)K * 64 * 4 + 64 * 4 +
           spc_slots<LAG3>() * 4 + 5 * 64 * 4 + 16 + 64 * kGS * 8 + 64 * 4 + 64 * 2 + 64 * 64;
}
static_assert(spc_lds_bytes<16>() <= 160 * 1024, "k_commit_spc LDS");
static_assert(spc_lds_bytes<16, kPipeThreads, true>() == spc_small_bytes<16, kPipeThreads, true>() + 64 * 193 * 8,
              "SpcSmem: S last");
// the prologue's aliases: the inherited snapshot states in D, their staged doubles in GS
static_assert(64 * 64 >= 128 * 3 * 8 && 64 * kGS * 8 >= 128 * 6 * 8, "SpcSmem prologue aliases");
static_assert((size_t)(kSpcThreads / 64) * 64 * 16 >= kSpcHash * 4 && (kPipeThreads / 64) * 64 * 16 >= kSpcHash * 4,
              "SpcSmem::own aliases pbk/pbx");

}  // namespace ksched
