// ksched_kernels.h -- HIP kernels of the scheduling core (gfx950 / CDNA4).
//
// Exact mode  : k_exact        persistent, node-per-lane, node state in registers, one grid-wide
//                              arg-best per pod through tagged 8-byte granules (no host round trip).
// Batched mode: k_score_topk   pod-per-lane fused predicate + score + per-lane top-K over a node
//                              chunk (node rows are wave-uniform -> scalar loads);
//               k_merge        sorted-list merge, one wave per (pod, <=64 lists), DPP/shuffle arg-best;
//               k_commit       one wave replays the batch in pod order: re-scores the nodes already
//                              committed in the batch, takes the first untouched candidate, commits,
//                              stops at the first candidate-list overflow.
// Every resource score divides by hoisted refined reciprocals (recip/qdiv, ksched_device.h), which
// are bit-identical to hipcc's f64 division for this path's operands.
// See DESIGN.md for the correctness argument of the batched commit.
#pragma once

#include "ksched_device.h"

namespace ksched {

struct alignas(8) Touched {
    int32_t idx;
    int32_t mine;     // committed to by a pod of THIS batch (exported to the next batch)
    int64_t s0[3];    // state at this batch's score snapshot
    int64_t sb[3];    // state when this batch's commit started
    int64_t cur[3];   // current state
    double curf[3];   // (double)cur
    double cury[3];   // recip((double)cur)
    uint64_t labels;
    float price;
    int32_t pad2;
};
static_assert(sizeof(Touched) == 144, "Touched layout");

// Nodes committed by one batch, handed to the next batch's commit (which scored against a snapshot
// one batch older) and to the apply kernel that writes them into the node rows (the stream pipeline's layout;
// the persistent pipeline stores them as tagged 16-byte chunks, below).
struct alignas(16) XRec {
    int32_t idx;
    int32_t pad;
    int64_t cur[3];   // state after the batch
    int64_t sb[3];    // state before the batch (= the next batch's snapshot state)
    uint64_t labels;
    float price;
    int32_t pad2;
    int64_t pad3;
};
static_assert(sizeof(XRec) == 80, "XRec layout");

// The persistent pipeline's export records: 96 B, six 16-byte chunks, each led by the exporting batch's tag (batch
// + 1; the ring is zeroed before every launch, so 0 is never live): {tag, idx, cur0} {tag, cur1, cur2.lo} {tag,
// cur2.hi, sb0} {tag, sb1, sb2.lo} {tag, sb2.hi, labels} {tag, price, -, -}.  A consumer that polls the records
// themselves knows every chunk it holds is the batch's (MI355X_MICROARCH R2: a 16-byte sc1 access is untorn) with
// no drained flag in front of them -- the commit(b - 1) -> commit(b) hand-off reads export(b - 1) in the same
// round of loads as the hand-off record.  The score workgroups' export apply reads the first three (idx, cur).
constexpr uint32_t kXRecPipe = 96;
constexpr size_t xbuf_bytes_pipe(int B) { return 16 + (size_t)2 * B * kXRecPipe; }
__device__ __forceinline__ int64_t w64(uint32_t lo, uint32_t hi) { return (int64_t)(((uint64_t)hi << 32) | lo); }

// entry i of the array at (wave-uniform) e: one buffer resource for the wave, the lane's record by offset (a
// per-lane base would make the resource divergent, which the compiler serialises lane by lane).  Persistent
// layout; true when every chunk carries `tag` (callers that validated a header pass any tag and ignore it).
__device__ __forceinline__ bool load_xrec_pipe(const XRec *e, int i, uint32_t tag, XRec *o) {
    const __amdgpu_buffer_rsrc_t r = coh_rsrc(e);
    const uint32_t off = (uint32_t)i * kXRecPipe;
    u32x4 c[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) c[k] = ld_coh16(r, off + 16u * k);
    o->idx = (int32_t)c[0].y; o->pad = 0;
    o->cur[0] = w64(c[0].z, c[0].w); o->cur[1] = w64(c[1].y, c[1].z); o->cur[2] = w64(c[1].w, c[2].y);
    o->sb[0] = w64(c[2].z, c[2].w); o->sb[1] = w64(c[3].y, c[3].z); o->sb[2] = w64(c[3].w, c[4].y);
    o->labels = (uint64_t)w64(c[4].z, c[4].w);
    o->price = __uint_as_float(c[5].y); o->pad2 = 0; o->pad3 = 0;
    return (c[0].x == tag) & (c[1].x == tag) & (c[2].x == tag) & (c[3].x == tag) & (c[4].x == tag) & (c[5].x == tag);
}

template <bool COH>
__device__ __forceinline__ XRec load_xrec(const XRec *e, int i) {
    if constexpr (!COH) {
        return e[i];
    } else {
        XRec o;
        (void)load_xrec_pipe(e, i, 0u, &o);
        return o;
    }
}

// tag: the persistent layout's chunk tag (the exporting batch + 1); unused by the stream pipeline's plain records
template <bool COH>
__device__ __forceinline__ void store_xrec(XRec *e, int i, const XRec &o, uint32_t tag) {
    if constexpr (!COH) {
        e[i] = o;
    } else {
        const __amdgpu_buffer_rsrc_t r = coh_rsrc(e);
        const uint32_t b = (uint32_t)i * kXRecPipe;
        auto lo = [](int64_t v) { return (uint32_t)(uint64_t)v; };
        auto hi = [](int64_t v) { return (uint32_t)((uint64_t)v >> 32); };
        st_coh16(r, b, u32x4{tag, (uint32_t)o.idx, lo(o.cur[0]), hi(o.cur[0])});
        st_coh16(r, b + 16, u32x4{tag, lo(o.cur[1]), hi(o.cur[1]), lo(o.cur[2])});
        st_coh16(r, b + 32, u32x4{tag, hi(o.cur[2]), lo(o.sb[0]), hi(o.sb[0])});
        st_coh16(r, b + 48, u32x4{tag, lo(o.sb[1]), hi(o.sb[1]), lo(o.sb[2])});
        st_coh16(r, b + 64, u32x4{tag, hi(o.sb[2]), lo((int64_t)o.labels), hi((int64_t)o.labels)});
        st_coh16(r, b + 80, u32x4{tag, __float_as_uint(o.price), 0u, 0u});
    }
}

template <bool COH>
__device__ __forceinline__ void add_i64(int64_t *p, int64_t v) {
    if (COH) st_coh(p, (uint64_t)((int64_t)ld_coh(p) + v)); else *p += v;
}

struct alignas(16) XBuf {
    int32_t count;
    int32_t pad;      // the persistent pipeline's batch tag
    int64_t pad2;
    XRec e[1];        // [2 * B] follow
};

// Device-side pipeline control (one per context).  plan[] holds each in-flight batch's first pod
// (ring of kPlanRing; -1 = nothing to do).  cursor/resync are written by k_commit, spec_next by k_plan.
constexpr int kPlanRing = 8;
// The persistent pipeline's lag: batch b is scored against the node state after commit(b - kPipeLag),
// and commit(b) inherits the nodes the kPipeLag - 1 batches before it committed.
// The stream pipeline runs at lag 2.
constexpr int kPipeLag = 3;
// The persistent pipeline's commit workgroups: they alternate batches (ksched_pipe.hip commit_role)
constexpr int kCommitWGs = 2;
constexpr int kCtlReplicas = 8;
struct alignas(128) CtlLine {
    unsigned long long v;
    unsigned long long pad[15];
};
struct alignas(128) Ctl {
    int64_t cursor;     // first unresolved pod
    int64_t spec_next;  // next speculative batch start
    int64_t resync;     // 1: a batch truncated; the next plan restarts at cursor
    int64_t stats[5];   // batches committed, truncated, placed, skipped, pairs scored
    int64_t plan[kPlanRing];
    unsigned long long scored;     // score workgroups finished this call (device hand-off to the merge)
    unsigned long long committed;  // batches committed this call: commit(b) publishes b + 1 (release)
    int64_t cursor_at[kPlanRing];  // cursor right after commit(b), slot b % kPlanRing
    int64_t nact;                  // persistent pipeline: active batches of the call (merger 0)
    unsigned long long polls_rmw;  // persistent waits that only the periodic atomic read satisfied
    // persistent pipeline (ksched_persist.hip).  Every polled or atomically counted word has a 128-byte line
    // of its own: one line shared by the commit's flag, 248 pollers and two families of atomic counters
    // starved single workgroups of their poll loads for seconds on MI355X.
    // per active batch a (counted identically by every workgroup), slot a % 4 -- a workgroup can run one
    // batch ahead of the slowest, so one shared counter would mix batches; four slots cannot (batch
    // a + 4 waits for commit(a + 2), which waited for every merge of a + 2)
    CtlLine arrive[4];             // score workgroups done with active batch a: G per use of the slot
    CtlLine merged[4];             // merger workgroups done with active batch a: B per use of the slot
    CtlLine committed_x[kCtlReplicas];  // Ctl::committed, one replica per XCD: workgroup w polls w % 8
    // the rescue of an exhausted candidate list (persistent pipeline, one rank): the commit publishes request
    // number q in rescue_req, each of the B merger slots scans its share of the nodes and counts its result in
    // rescue_done (B per request)
    CtlLine rescue_req;
    CtlLine rescue_done;
    // the persistent pipeline's hand-off between its two commit workgroups: commit(b) leaves two 16-byte sc1
    // granules, each tagged b + 1: {tag, export count, cursor} and {tag, rescue requests, plan of b + 3}; commit(b + 1)
    // polls them instead of Ctl::committed and a second round of loads
    CtlLine hrec;
};
// The rescue request the commit writes (PersistArgs::rescue; sc1 stores, then Ctl::rescue_req) and the merger
// slots' results after it: {rc, rm, rp, sel, nT} and the touched set's node indices, then Rec res[B].
constexpr int kRescueMaxT = 256;  // >= the persistent commit's touched slots (spc_slots<true>() + 1)
struct alignas(16) RescueReq {
    int64_t rc, rm, rp;
    uint64_t sel;
    int64_t nT;
    int64_t pad;
    int64_t ti[kRescueMaxT];
};
constexpr size_t kRescueResOff = (sizeof(RescueReq) + 127) / 128 * 128;
constexpr size_t rescue_bytes(int B) { return kRescueResOff + (size_t)B * sizeof(Rec); }

struct PodArgs {
    const int64_t *rc, *rm, *rp;
    const uint64_t *sel;
    int64_t p;
};

struct OutArgs {
    int32_t *idx;
    double *score;
    int32_t *feas;
};

struct ExactArgs {
    NodeRec *nodes;
    int64_t n;
    int32_t G;        // workgroups (all co-resident)
    int32_t per_wg;   // nodes per workgroup
    PodArgs pods;
    OutArgs out;
    uint64_t *slots;  // [2][G][4] granules {epoch:32 | value:32}; zeroed before every launch
    int32_t *err;     // device error word (1 = exchange timeout)
    int64_t timeout_ticks;
    const int32_t *perm;  // k_exact1: slot -> node (best-price: nodes by price asc, index asc); null: slot = node
};

struct ScoreArgs {
    NodeRec *nodes;    // read; the rows of `patch` are written back by their chunk's wave
    int64_t n_local;
    int64_t node_offset;
    int32_t S;         // unused
    int32_t n_chunks;  // NSC sub-chunks = workgroups x kScoreWaves
    PodArgs pods;
    const int64_t *cursor;  // this batch's plan slot (first pod, or -1)
    int32_t B;
    Cand *part;        // [B][workgroups][KC]
    int64_t *part_cnt; // [B][workgroups]
    const XBuf *patch; // batch b-2's commits: overlaid on the rows as they are read, then written back
    // device-side wait for commit(b-2): poll *wait_committed >= wait_target (null: the stream waits)
    const unsigned long long *wait_committed;
    unsigned long long wait_target;
    int32_t *err;                    // device error word (4 = the wait timed out)
};

struct MergeArgs {
    const void *in;         // Cand [B][C_in][K]  or, INPUT_REC, C_in rank blocks of rank_stride bytes,
                            // each {Rec [B][K]; int64 fc[B]} (the RCCL all-gather layout)
    const int64_t *in_cnt;  // [B][C_in] (Cand input only)
    int64_t rank_stride;    // bytes per rank block (INPUT_REC)
    int32_t C_in;
    int32_t C_out;          // ceil(C_in / 64)
    int32_t chunk_input;    // 1: inputs are score-kernel chunk lists (cut when full)
    int64_t *dbg;           // diagnostics only (KSCHED_MERGE_STAMPS): per-phase cycle sums, else null
    Cand *out;              // [B][C_out][K] (non-final)
    int64_t *out_cnt;       // [B][C_out]
    Rec *out_rec;           // [B][K]  (final)
    int64_t *out_fc;        // [B]
    const NodeRec *nodes;   // final + !INPUT_REC: gather node snapshot state
    int64_t node_offset;
    const int64_t *cursor;
    int64_t P;
    int32_t B;
    int32_t p0_known;   // 1: p0v is this batch's first pod (the persistent score grid read it already)
    int64_t p0v;
    int32_t *err;                        // device error word
    uint32_t *lds_msg;                   // non-null: the final list goes to LDS as a PodMsg (kMsgWords)
    uint32_t tag;                        // persistent pipeline: the batch's 16-bit record tag (score_role)
};

// One pod's merged candidate list as 32-bit words, the unit the ranks exchange in the persistent
// multi-rank pipeline: K Rec rows (14 words each, the Rec layout) then the feasible count (2 words).
constexpr int kRecWords = (int)(sizeof(Rec) / 4);
constexpr int msg_words(int K) { return K * kRecWords + 2; }

// The persistent commit workgroup's private control state (LDS): it is the only writer of the plans,
// the cursor, the stats and the export once its kernel runs, so it reads its own copies instead of
// loading them back from HBM -- every global load of the commit's serial chain costs ~1-2 us.
struct PersistLocal {
    int64_t plan[kPlanRing];
    int64_t cursor;
    int64_t stats[5];  // as Ctl::stats; [4] = rescues
    int32_t xcount;   // entries of the previous batch's export
    int32_t xcount2;  // entries of the export of the batch before it (both are inherited: lag kPipeLag)
    int64_t rseq;     // rescue requests issued this call
    int32_t rescue_credit;  // the rescue bucket, in quarter rescues (CommitArgs::rescue_rate)
};

struct PersistArgs;
struct CommitArgs {
    const Rec *lists;       // [B][K]
    const int64_t *fc0;     // [B]
    PodArgs pods;
    const int64_t *plan;    // this batch's plan slot
    const int64_t *plan1;   // the next batch's plan slot (already set)
    int64_t *plan2;         // the slot of the batch after next: written by this commit
    Ctl *ctl;
    int32_t B;
    const XBuf *xin;        // nodes committed by the previous batch (relative to this batch's snapshot)
    const XBuf *xin2;       // persistent pipeline (lag 3): nodes committed two batches earlier; else null
    XBuf *xout;             // nodes committed by this batch
    OutArgs out;
    int64_t *dbg;           // diagnostics only (KSCHED_COMMIT_STAMPS): per-phase cycle sums, else null
    int64_t batch;          // this batch's index in the call (published to Ctl::committed when done)
    int64_t *cursor_at;     // persistent pipeline: &Ctl::cursor_at[batch % kPlanRing] (else null)
    PersistLocal *loc;      // persistent pipeline (COH): the commit workgroup's LDS control state
    int32_t release;        // COH: also write back the XCD's L2 (agent release) before Ctl::committed
    char *rescue;           // persistent pipeline: the rescue request / results (else null: truncate)
    int32_t rescue_n;       // merger slots serving a rescue (= B)
    int32_t rescue_max;     // rescues per batch; the next exhausted list truncates the batch
    int32_t rescue_cap;     // persistent: the rescue bucket's capacity, in rescues
    int32_t rescue_low;     // persistent: rescues per batch while the bucket is below half full
    int32_t rescue_look;    // persistent: skip a rescue when the batch's exhausted lists already overrun the credit
    int32_t rescue_rate;    // persistent: the bucket's refill per batch of this workgroup, in quarter rescues (a batch
                            // spends at most min(rescue_max, credit) rescues; rate >= 4 * rescue_max: a fixed budget)
    int32_t touch_screen;   // persistent commit: the touched-node screen on (KSCHED_NO_TOUCH_SCREEN=1 turns it off)
    const char *inh;        // persistent commit: the mergers' keys of the older export (inherit_x2_keys), else null
    int64_t timeout_ticks;  // bound of the rescue wait
    int32_t *err;           // device error word (12 = the rescue wait timed out)
    uint64_t *trace_row;    // KSCHED_PERSIST_TRACE: this batch's trace row (else null)
    const PersistArgs *xp;  // persistent pipeline: its arguments (R > 1: the rescue's rank fold through the rings)
    int64_t dbg_act;        // diagnostics (KSCHED_XCHG_DUMP): this batch's active-batch index
};
// KSCHED_XCHG_DUMP's list sums: (key, idx | valid) words of a pod's merged list as written / as the commit loaded
// them, [cap][B][2] u64 after the hashes and the messages
__device__ __forceinline__ uint64_t dbg_mix(uint64_t w0, uint64_t w1, int q) {
    return (w0 * 0x9e3779b97f4a7c15ull + w1) * (uint64_t)(2 * q + 1);
}
__host__ __device__ inline size_t xdbg_sums_off(int64_t cap, int B, int R, int K) {
    return (size_t)cap * B * (R + 1) + ((size_t)16 * B * (K * 14 + 2) + 1) / 2;
}
// ... then per active batch the commit's summary [cap][8] u64 (ksched_commit.h)
__host__ __device__ inline size_t xdbg_commit_off(int64_t cap, int B, int R, int K) {
    return xdbg_sums_off(cap, B, R, K) + (size_t)cap * B * 2;
}

// Commit(b) -> score(b + lag) hand-off on the device (lag 2 on the stream pipeline, kPipeLag in k_pipe): the
// committing wave drains its stores, writes back the XCD L2 (agent release) and publishes
// Ctl::committed = b + 1; the later score polls it instead of waiting
// on a cross-queue stream event (~12 us per hand-off).  Call from ONE wave that
// made every global store of the commit (the others made none).
// COH (persistent pipeline): every handed-off store was an sc1 store, so no L2 write-back is needed.
// COH (persistent pipeline): the caller stored Ctl::cursor_at (store_cursor_at) before the drain in front of its
// hand-off record, so every store a reader of Ctl::committed needs has landed: no store and no drain here (the
// hand-off record itself is read only by the next commit, which polls it).
template <bool COH = false>
__device__ __forceinline__ void publish_committed(const CommitArgs &A) {
    if (!COH) {
        if ((threadIdx.x & 63) == 0 && A.cursor_at) st_coh(A.cursor_at, ld_coh(&A.ctl->cursor));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if ((threadIdx.x & 63) == 0) {
        if (!COH || A.release) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (COH)  // two commit workgroups: a maximum, so the count never steps back
            __hip_atomic_fetch_max(&A.ctl->committed, (unsigned long long)A.batch + 1ull, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        else
            __hip_atomic_store(&A.ctl->committed, (unsigned long long)A.batch + 1ull, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    // persistent pipeline: the per-XCD replicas (lanes 0..7 of the publishing wave, one each)
    if (COH && (threadIdx.x & 63) < kCtlReplicas)
        __hip_atomic_fetch_max(&A.ctl->committed_x[threadIdx.x & 63].v, (unsigned long long)A.batch + 1ull,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// every replica of Ctl::committed (the persistent pipeline's end and error paths; lanes 0..7)
__device__ __forceinline__ void publish_committed_all(Ctl *ctl, unsigned long long v) {
    const int l = threadIdx.x & 63;
    if (l == 0) __hip_atomic_store(&ctl->committed, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (l < kCtlReplicas) __hip_atomic_store(&ctl->committed_x[l].v, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct alignas(8) PodStage {
    int64_t rc, rm, rp;
    uint64_t sel;
    int64_t fc0;
    int32_t cut;  // the pod's merged list is cut (entry 0's pad; see k_merge)
    int32_t pad;
};
constexpr size_t kPodStageBytes = sizeof(PodStage);

// A candidate as staged in the commit kernel's LDS (idx = kNoIdx for an empty slot).
struct alignas(8) CandStage {
    double key;
    int32_t idx;
    float price;
    int64_t a[3];
    uint64_t labels;
};
static_assert(sizeof(CandStage) == 48, "CandStage layout");

constexpr int kTouchHashBits = 9;  // touched-node set: 512 slots >= 2 x max batch (256)
constexpr int kTouchHash = 1 << kTouchHashBits;

constexpr int kTouchFilterBits = 16;  // 64K-bit filter in front of the hash (bit = idx & 0xffff)
constexpr int kTouchFilterWords = (1 << kTouchFilterBits) / 32;

// LDS bytes of k_commit for a batch of B pods with K candidates each (touched table: the previous
// batch's nodes + this batch's, <= 2B).
constexpr size_t commit_lds_bytes(int B, int K) {
    return kTouchHash * sizeof(int32_t) + kTouchFilterWords * sizeof(uint32_t) +
           (size_t)B * (2 * sizeof(Touched) + sizeof(PodStage) + (size_t)K * sizeof(CandStage));
}
// Speculative planning, done by the commit of batch k for batch k+2 (stream order makes plan(k+2)
// visible to score(k+2), which waits for commit(k)): after a truncation restart at the committed
// frontier, otherwise continue one batch after plan(k+1).  -1 = past the last pod.
template <bool COH = false>
__device__ __forceinline__ void plan_after_commit(const CommitArgs &A, bool truncated, int64_t cursor) {
    const int64_t n1 = load_i64<COH>(A.plan1);
    int64_t nx = truncated ? cursor : (n1 < 0 ? -1 : n1 + A.B);
    if (nx >= A.pods.p) nx = -1;
    store_i64<COH>(A.plan2, nx);
}

constexpr size_t xbuf_bytes(int B) { return 16 + (size_t)2 * B * sizeof(XRec); }

// FailedScheduling diagnostics of a whole schedule call (ksched_explain.hip).
struct ExplainArgs {
    const int32_t *idx;           // the call's results (global node index | NO_FIT | NO_POSITIVE_SCORE)
    int64_t p;
    const int64_t *rc, *rm, *rp;  // the call's pods
    const uint64_t *sel;
    const NodeRec *nodes;         // this rank's node rows after the call
    int64_t n_local, node_lo;
    bool use_labels;
    int32_t *fpod_out;            // explain_batch: the NO_FIT pods, in pod order (device, >= p entries)
    int64_t *n_nofit;             // explain_batch: their number (host)
    int64_t q_rc, q_rm, q_rp;     // explain_pod_at: that pod's request
    uint64_t q_sel;
};
// counts[f][kNumReasons] (zeroed by the caller) for the f-th NO_FIT pod; ws is a growable workspace.
hipError_t explain_batch(const ExplainArgs &a, void **ws, size_t *ws_bytes, unsigned long long *counts, hipStream_t s);
// per-node reasons + counts of ONE pod against the state it saw at its turn (state: 3 * n_local int64)
hipError_t explain_pod_at(const ExplainArgs &a, int64_t pod, int64_t *state, uint8_t *reason,
                          unsigned long long *counts, hipStream_t s);

// host-side launchers (ksched_kernels.hip).  fast53: every allocatable and request magnitude stays
// below 2^52 for the whole call (host-checked), enabling (double)(a-r) == (double)a - (double)r.
hipError_t launch_prep_nodes(NodeRec *nodes, int64_t n, hipStream_t s);
hipError_t launch_exact(int npt, int prio, int dom, bool lab, bool fast53, const ExactArgs &a, int block,
                        bool cooperative, hipStream_t s);
hipError_t launch_score_topk(int KC, int prio, int dom, bool lab, bool fast53, const ScoreArgs &a, int pod_groups,
                             hipStream_t s);
// one workgroup per pod: the score kernel's workgroup lists -> the pod's K-entry Rec list (C_in <= 256)
hipError_t launch_merge_pod(int KC, int K, const MergeArgs &a, hipStream_t s);
hipError_t launch_merge(int KIN, int K, bool input_rec, bool final_stage, const MergeArgs &a, hipStream_t s);
hipError_t launch_commit(int K, int prio, int dom, bool lab, bool fast53, const CommitArgs &a, size_t lds_bytes,
                         hipStream_t s);
constexpr int kSpcThreads = 512;  // speculative commit: wave 0 guesses and checks, 8 waves evaluate
hipError_t launch_commit_spc(int K, int prio, int dom, bool lab, bool fast53, const CommitArgs &a, hipStream_t s);
hipError_t commit_spc_attributes(int K, int prio, int dom, bool lab, bool fast53, hipFuncAttributes *at, size_t *lds);
// Can the batch's commit workgroup dispatch onto a CU that holds a score workgroup (VGPRs, LDS, wave
// slots)?  Only then may score(b) be resident and poll for commit(b-2): otherwise the score grid
// could occupy every CU while the commit it waits for never gets in.
bool commit_fits_beside_score(int KC, int K, int B, bool spc, int prio, int dom, bool lab, bool fast53);
constexpr int kNumReasons = 5;  // fit, Insufficient CPU, Insufficient Memory, Insufficient Pod, labels
hipError_t launch_explain(const NodeRec *nodes, int64_t n, int64_t rc, int64_t rm, int64_t rp, uint64_t sel,
                          bool use_labels, uint8_t *reason, unsigned long long *counts, hipStream_t s);
hipError_t launch_apply_delta(NodeRec *nodes, int64_t n, int64_t k, const int32_t *idx, const int64_t *d,
                              hipStream_t s);
hipError_t launch_ctl_init(Ctl *ctl, int B, int64_t P, int lag, hipStream_t s);
// zero `bytes` (a multiple of 8) at p with system-scope 8-byte stores: the path the exchange's granules take
// (a hipMemset of an uncached ring was not what a later kernel's system-scope loads read: DESIGN.md section 6.1)
hipError_t launch_zero_sys(void *p, size_t bytes, hipStream_t s);

// ---- persistent single-rank pipeline (ksched_persist.hip) -------------------------------------
// One score grid of G workgroups (one per CU, the WG's node rows resident in LDS for the whole call)
// and one resident commit workgroup, joined by device counters in Ctl instead of launches and stream
// events: score(b) waits for commit(b-2) (Ctl::committed), the last B score workgroups to finish batch
// b merge one pod each (Ctl::arrive), commit(b) waits for the B merges (Ctl::merged).
struct PersistArgs {
    NodeRec *nodes;
    int64_t n_local;
    PodArgs pods;
    Ctl *ctl;
    int32_t B, G, rows_per_wg;
    int32_t M;              // merger workgroups (after the G score workgroups): kPipeMergeSlots pod slots each
    Cand *part;             // [kPipeLag][B][G][KC], entry 0's pad = the list's predicate count
    char *lring;            // 4 x {Rec [B][K]; int64 fc[B]}
    int64_t lists_bytes;
    char *xring;            // 4 XBufs + the permanently empty one (slot 4)
    int64_t xbuf_bytes;
    OutArgs out;
    int32_t *err;           // device error word (5..9 = a persistent wait timed out)
    int64_t timeout_ticks;
    int32_t no_screen;      // diagnostics (KSCHED_NO_SCREEN): the exact scan in every batch
    int32_t no_pairs;       // diagnostics (KSCHED_NO_PAIRS): the screened scan's exact phase by rows, never by pairs
    int32_t screen_ok;      // the screened scan's reciprocals fit in a score workgroup's LDS
    int32_t screen_h;       // ... and so do pass 1's per-pair records
    // optional (KSCHED_PERSIST_TRACE): wall-clock stamps per batch, [trace_cap][kTraceCols]
    uint64_t *trace;
    int64_t trace_cap;
    // optional (KSCHED_TRACE_WG=<path>): per batch and score workgroup {scan start, arrival} as the low and
    // high 32 bits of the 100 MHz wall clock, [trace_cap][G]
    uint64_t *trace_wg;
    // optional (KSCHED_XCHG_DUMP=<path>, R > 1): per active batch a and pod m, [R + 1] hashes of the messages the
    // merger received from each rank, then of the one it sent: [(a * B + m) * (R + 1) + r]
    uint64_t *xdbg;
    int64_t xdbg_cap;       // active batches it holds
    int64_t *cdbg;  // KSCHED_COMMIT_STAMPS: commit phase cycle sums (CommitArgs::dbg), else null
    int64_t *mdbg;  // KSCHED_MERGE_STAMPS: merge phase cycle sums (MergeArgs::dbg), else null
    // node-sharded (R > 1, one process per GPU): this rank owns global nodes [node_offset, +n_local);
    // merger m of every rank writes pod m's list into EVERY rank's receive ring (rx_peer[r], slot
    // (active batch % 4, source rank, pod) of xchg_stride bytes) as tagged 8-byte granules (gran_enc),
    // then gathers the R lists of pod m from its own ring and rank-merges them (ksched_persist.hip)
    int64_t node_offset;
    int32_t R, rank;
    uint32_t epoch0;        // granule tag of this call's active batch a is epoch0 + a (a >= 1)
    int64_t xchg_stride;    // bytes per pod message in a ring
    char *rx_peer[8];       // every rank's receive ring, mapped into this process (rx_peer[rank] = own)
    // progress words, kProgWords per workgroup ([G] score, [B] merger, [1] commit): {batch << 8 | phase, hw id
    // << 32 | low word of the last value a wait saw, busy-time sums}; read by the host when a wait timed out
    // (and by the phase trace)
    uint64_t *prog;
    char *rescue;           // this rank's RescueReq + Rec res[B] (null: exhausted lists truncate their batch)
    int32_t poison_lds;     // diagnostics (KSCHED_POISON): bytes of dynamic LDS every workgroup fills with 0xff first
    uint32_t lds_fill;      // diagnostics (KSCHED_LDS_FILL): the fill pattern (KSCHED_POISON: 0xffffffff)
    int32_t lds_fill_role;  // roles filled: 1 commit, 2 score, 4 merge (KSCHED_LDS_ROLE, default all)
    int32_t lds_fill_lo, lds_fill_hi;  // byte range filled (KSCHED_LDS_LO / KSCHED_LDS_HI)
    uint32_t jitter;        // diagnostics (KSCHED_JITTER): seed of the random delays at the protocol points, 0 = off
    int32_t rescue_max;     // rescues per batch before an exhausted list truncates it (KSCHED_RESCUE_MAX)
    int32_t rescue_cap;     // the rescue bucket's capacity in rescues (KSCHED_RESCUE_CAP, default rescue_max)
    int32_t rescue_low;     // rescues per batch while the bucket is below half full (KSCHED_RESCUE_LOW)
    int32_t rescue_look;    // KSCHED_RESCUE_LOOK (default 0): the commit's look-ahead over the batch's exhausted lists
    int32_t rescue_rate;    // the commit workgroup's rescue bucket refill per batch, quarter rescues (KSCHED_RESCUE_RATE)
    int32_t touch_screen;   // the commit's touched-node screen (KSCHED_NO_TOUCH_SCREEN=1: every key exact)
    // the merger slots' keys of their pod against the entries of export(b - 2), which commit(b) inherits:
    // [4 batches][B] summaries {sum of predicate deltas, best key, best idx | entry << 32, -} then [4][B][64] keys
    char *inh;
};
constexpr size_t inh_bytes(int B) { return (size_t)4 * B * 32 + (size_t)4 * B * 64 * 8; }
// progress phases (PersistArgs::prog); kProgWords 8-byte words per workgroup
constexpr int kProgWords = 6;  // 0 phase, 1 where/seen, 2 heartbeat, 3 busy, 4 rows scored exactly, 5 rows scanned
enum : int { kProgWaitCommit = 1, kProgScan = 2, kProgArrived = 3, kProgWaitArrive = 4, kProgMerged = 5,
             kProgWaitMerged = 6, kProgCommitted = 7, kProgIdle = 8, kProgRescue = 9, kProgWaitRescue = 10,
             kProgTimedOut = 0x80 };
__device__ __forceinline__ uint32_t hw_where() {
    uint32_t xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    // xcc[3:0] | se[15:13] | cu[11:8] of HW_ID
    return (xcc & 0xf) << 8 | ((hw >> 13) & 7) << 4 | ((hw >> 8) & 0xf);
}
__device__ __forceinline__ void prog_at(const PersistArgs &P, int slot, int64_t b, int phase, uint64_t seen) {
    if (!P.prog) return;
    __hip_atomic_store(P.prog + kProgWords * slot, (uint64_t)b << 8 | (uint64_t)phase, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(P.prog + kProgWords * slot + 1, (uint64_t)hw_where() << 32 | (seen & 0xffffffffull),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// busy-time sums of a workgroup (KSCHED_PERSIST_TRACE calls only: P.trace set): word 2 += scan ticks, word 3
// += ticks from its wait's end to its arrival (word 2 is the heartbeat of a long wait otherwise)
__device__ __forceinline__ void prog_add(const PersistArgs &P, int slot, uint64_t scan, uint64_t busy) {
    if (!P.prog || !P.trace) return;
    P.prog[kProgWords * slot + 2] += scan;
    P.prog[kProgWords * slot + 3] += busy;
}
// Atomic read of a control word at the coherence point: an RMW that adds a zero the compiler cannot see
// (an idempotent RMW it would turn back into a plain atomic load, which may be served by a cached line).
__device__ __forceinline__ uint64_t ld_rmw(const void *p) {
    uint64_t zero = 0;
    asm volatile("" : "+v"(zero));
    return __hip_atomic_fetch_add(reinterpret_cast<uint64_t *>(const_cast<void *>(p)), zero, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
}
// Bounded wait for *p >= v (one lane).  Polls are relaxed agent-scope (sc1) loads with s_sleep; every 1024th
// poll reads the counter with an atomic RMW instead (performed at the coherence point, never served from a
// cached line), so a poll can not stay behind the counter for longer than ~1024 sleeps; each such read
// also stores the poll count to *heartbeat (a stuck wait shows whether it still runs).  A wait that only the
// RMW read satisfied is counted in *rmw_hits.  false: timed out (*seen = the last value read).
__device__ __forceinline__ bool poll_ge(const unsigned long long *p, unsigned long long v, int64_t limit,
                                        unsigned long long *rmw_hits, unsigned long long *seen,
                                        uint64_t *heartbeat = nullptr) {
    unsigned long long x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (x >= v) { *seen = x; return true; }
    const uint64_t t0 = wall_clock64();
    for (int it = 1;; ++it) {
        __builtin_amdgcn_s_sleep(1);
        if ((it & 1023) == 0) {
            if (heartbeat) __hip_atomic_store(heartbeat, (uint64_t)it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            x = (unsigned long long)ld_rmw(p);
            if (x >= v) {
                if (rmw_hits) __hip_atomic_fetch_add(rmw_hits, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                *seen = x;
                return true;
            }
            if ((int64_t)(wall_clock64() - t0) > limit) { *seen = x; return false; }
        } else {
            x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (x >= v) { *seen = x; return true; }
        }
    }
}
// The exchange's 8-byte granules carry one 32-bit word and the writer's tag in EACH 32-bit half: {tag16 | word
// bits 0..15} low, {tag16 | word bits 16..31} high, tag16 = (tag & 0x7fff) | 0x8000 (never 0: a zeroed ring holds no
// live granule).  A reader accepts the granule only when both halves carry the tag, so a granule read half old and
// half new (an 8-byte access split into two 4-byte ones -- seen on uncached rings) is never
// taken for the new one.  Tags 32768 apart would alias: every call zeroes the message and rescue areas before its
// rank barrier (ksched_engine.hip rx_zero_regions), within a call a region is rewritten every 4 active batches, and
// consecutive calls' barrier tags never differ by a multiple of 2^15.
__device__ __forceinline__ uint32_t gran_tag(uint32_t tag) { return (tag & 0x7fffu) | 0x8000u; }
__device__ __forceinline__ uint64_t gran_enc(uint32_t word, uint32_t t16) {
    return ((uint64_t)((t16 << 16) | (word >> 16)) << 32) | (uint64_t)((t16 << 16) | (word & 0xffffu));
}
__device__ __forceinline__ bool gran_dec(uint64_t v, uint32_t t16, uint32_t *word) {
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    *word = (lo & 0xffffu) | (hi << 16);
    return ((lo >> 16) == t16) & ((hi >> 16) == t16);
}

constexpr int kMaxXchgRanks = 8;
// receive ring: [4 active-batch slots][R source ranks][B pods] messages, then R barrier granules, then the
// rescue area: [2 request parities][R source ranks] one Rec as 14 tagged granules (128 bytes each)
constexpr size_t xchg_stride_bytes(int K) { return ((size_t)msg_words(K) * 8 + 63) / 64 * 64; }
constexpr int kXchgRescueWords = (int)(sizeof(Rec) / 4);  // 14
constexpr size_t kXchgRescueRec = 128;
__host__ __device__ constexpr size_t xchg_rescue_off(int R, int B, size_t stride) { return (size_t)4 * R * B * stride + 64 * (size_t)R; }
constexpr size_t xchg_ring_bytes(int R, int B, int K) {
    return xchg_rescue_off(R, B, xchg_stride_bytes(K)) + 2 * (size_t)R * kXchgRescueRec;
}
// all ranks meet on the device and agree on the minimum of a small value (tag: this call's epoch0)
hipError_t launch_xchg_min(const PersistArgs &a, int32_t mine, int32_t *out, hipStream_t s);
// trace columns: score start (WG 0 past its wait), last arrival, last merge done, commit start, commit end
// trace row: 0-15 stamps (col 13: exact rows), 16 the commit's counters, 17 its rescue waits; with
// KSCHED_COMMIT_STAMPS 18-21 its prologue / guess / evaluate / check cycles, 22-23 prologue marks (lists hashed, all
// waves past), 24 before the wait, 25 entry -> past the wait, 26-30 the check step's split (update, probe, commit,
// rescan, state load), 31-32 the guess step's (set-up, fixpoint), 33-36 the wave-0 state's (26-36: builds with
// KSCHED_COMMIT_SPLIT only)
constexpr int kTraceCols = 54;  // + 37-48: score WG 0's waves' pass-1 ends; 49-53: the commit's rounds
// KSCHED_JITTER (race hunting): at one in four (workgroup, batch, site) triples, sleep the wave for up to ~50 us,
// chosen by a hash of the seed -- a protocol that depends on timing then fails often instead of rarely
__device__ __forceinline__ void jitter_at(uint32_t seed, int64_t b, int site) {
    if (!seed) return;
    uint32_t h = seed ^ (uint32_t)((uint64_t)b * 0x9E3779B1u) ^ ((uint32_t)site * 0x85EBCA77u) ^ (blockIdx.x * 0xC2B2AE3Du);
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
    if ((h & 3) != 0) return;
    const int n = (int)((h >> 8) & 255);
    for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(8);
}
__device__ __forceinline__ void trace_at(const PersistArgs &P, int64_t b, int col) {
    if (P.trace && b < P.trace_cap) P.trace[b * kTraceCols + col] = wall_clock64();
}
// The persistent pipeline (ksched_pipe.hip): ONE kernel of 1 + G workgroups x kPipeThreads, workgroup 0
// the commit, workgroups 1 .. G score, workgroups G + 1 .. G + M merge (kPipeMergeSlots pods each).
constexpr int kPipeThreads = 768;
constexpr int kPipeWaves = kPipeThreads / 64;
constexpr int kPipeScoreWaves = kPipeWaves;  // a score workgroup scores with all its waves
constexpr int kPipeMergeThreads = 256;       // one pod merge: one thread per score workgroup's list
constexpr int kPipeMergeSlots = kPipeThreads / kPipeMergeThreads;  // pods a merger workgroup merges at once
struct PipeInfo {
    size_t lds;         // dynamic LDS per workgroup (max of the commit's and a score workgroup's layout)
    size_t static_lds;
    int vgprs;
    size_t spill;       // private (scratch) bytes per thread
    int occ;            // workgroups per CU the occupancy query admits at that LDS (1: one per CU)
};
// One launch of k_pipe: the grids of R ranks (R = 1: a single rank) back to back, rank r's workgroups
// [base[r], base[r + 1]).  R > 1 only for ranks of ONE process sharing ONE device (ksched_xchg_join_local):
// their persistent kernels must be resident at once, which one cooperative launch guarantees and separate
// launches do not.
constexpr int kMaxLocalRanks = 8;  // PipeLaunch: 8 x 344-byte PersistArgs = 2.8 KB of kernel arguments
struct PipeLaunch {
    PersistArgs P[kMaxLocalRanks];
    int32_t R;
    int32_t base[kMaxLocalRanks + 1];
};
// launch: 0 = query PipeInfo only (L.P[0]), 1 = cooperative launch (the runtime checks the grid against the
// occupancy query, so every workgroup of every rank in L is resident at once).
// hipErrorNotSupported: no instantiation for (KC, K) -- the caller runs the stream pipeline.
hipError_t pipe_part_price(int KC, int K, bool lab, bool f53, const PipeLaunch &L, int launch, PipeInfo *info,
                           hipStream_t s);
hipError_t pipe_part_res_all(int KC, int K, bool lab, bool f53, const PipeLaunch &L, int launch, PipeInfo *info,
                             hipStream_t s);
hipError_t pipe_part_res_feas(int KC, int K, bool lab, bool f53, const PipeLaunch &L, int launch, PipeInfo *info,
                              hipStream_t s);
inline hipError_t launch_pipe(int KC, int K, int prio, int dom, bool lab, bool f53, const PipeLaunch &a, int launch,
                              PipeInfo *info, hipStream_t s) {
    if (prio == kPrioPrice) return pipe_part_price(KC, K, lab, false, a, launch, info, s);
    if (dom == kDomFeasible) return pipe_part_res_feas(KC, K, lab, f53, a, launch, info, s);
    return pipe_part_res_all(KC, K, lab, f53, a, launch, info, s);
}
hipError_t launch_apply_batch(const XBuf *x, NodeRec *nodes, int64_t node_lo, int64_t n_local, hipStream_t s);
// diagnostics: qdiv(a, b, recip(b)) against the native a / b, bit for bit
hipError_t launch_selftest_div(int64_t n, const double *a, const double *b, double *native, double *fast,
                               hipStream_t s);

constexpr int kExactBlock = 256;
constexpr int kExact1Block = 1024;  // k_exact1: the whole node set in one workgroup
// exact mode on one workgroup of bs threads, npt node slots each: bs 1024 with npt 1-4 (resource) or 1-6, 8, 12, 16
// (best-price); best-price also (512, 10) and (256, 20)
hipError_t launch_exact1(int npt, int bs, int prio, int dom, bool lab, bool f53, const ExactArgs &a, hipStream_t s);

// score kernel geometry: 4 waves per workgroup, 2 workgroups per CU at the default grid
constexpr int kScoreWaves = 8;
constexpr int kMergeThreads = 512;  // merge: one workgroup per pod, lane = one workgroup list (<= 512)
constexpr int kScoreThreads = kScoreWaves * 64;
constexpr size_t score_lds_bytes(int KC) { return (size_t)(kScoreWaves / 2) * KC * 64 * 12 + 64 * 4; }

// (priority, domain, labels, fast53) -> instantiation.  Best-price always ranges over feasible nodes
// and never divides (fast53 irrelevant).
#define KSCHED_DISPATCH(prio, dom, lab, f53, CALL)                                              \
    do {                                                                                        \
        if ((prio) == kPrioPrice) {                                                             \
            constexpr int P_ = kPrioPrice, D_ = kDomFeasible; constexpr bool F_ = false;        \
            if (lab) { constexpr bool L_ = true; return CALL; }                                 \
            else { constexpr bool L_ = false; return CALL; }                                    \
        }                                                                                       \
        constexpr int P_ = kPrioResource;                                                       \
        if ((dom) == kDomFeasible) {                                                            \
            constexpr int D_ = kDomFeasible;                                                    \
            if (lab) { constexpr bool L_ = true;                                                \
                if (f53) { constexpr bool F_ = true; return CALL; } else { constexpr bool F_ = false; return CALL; } } \
            else { constexpr bool L_ = false;                                                   \
                if (f53) { constexpr bool F_ = true; return CALL; } else { constexpr bool F_ = false; return CALL; } } \
        } else {                                                                                \
            constexpr int D_ = kDomAll;                                                         \
            if (lab) { constexpr bool L_ = true;                                                \
                if (f53) { constexpr bool F_ = true; return CALL; } else { constexpr bool F_ = false; return CALL; } } \
            else { constexpr bool L_ = false;                                                   \
                if (f53) { constexpr bool F_ = true; return CALL; } else { constexpr bool F_ = false; return CALL; } } \
        }                                                                                       \
    } while (0)

}  // namespace ksched
