// ksched_engine.hip -- libksched: the C-ABI (include/ksched.h) over the HIP kernels.
//
// Device residency: node state (64-B NodeRec rows), pending pods (SoA), outputs and all batch
// workspaces live in HBM for the life of the context; a schedule call moves only the pods in and the
// per-pod results out.  The batched loop keeps its cursor (first unresolved pod) on the device, so
// batches are enqueued back to back with no host round trip; the host only polls the cursor every
// few dozen batches to know when to stop.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <tuple>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ksched.h"
#include "ksched_kernels.h"

using namespace ksched;

// In-process rank group (include/ksched.h).  The all-gather is host-coordinated and synchronous:
// every rank waits for its own send block, the ranks meet, each copies every rank's block into its
// receive buffer (device-to-device on the shared device) and waits for the copies, and the ranks meet
// again before any send block can be rewritten.  No kernel ever waits on another rank's work, so the
// ranks' streams may share hardware queues (GPU_MAX_HW_QUEUES) without deadlock.  Slower than RCCL by
// a host round trip per batch: a test vehicle for the multi-rank code, not a bench path.
struct ksched_group {
    int nranks = 0, dev = 0;
    int64_t block_bytes = 0;
    std::vector<const char *> send;  // each rank's send block of the current exchange
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0, acc = 0, result = 0;
    uint64_t gen = 0;
};

// Ranks of ONE process sharing ONE device, joined by ksched_xchg_join_local: the device exchange of the
// node-sharded persistent pipeline without IPC, and their persistent kernels as ONE cooperative launch
// (k_pipe over a PipeLaunch of every rank's arguments), so every rank's grid is resident at once by
// construction.  Per call the ranks meet twice on the host: to agree on FAST53, and to launch -- the last
// rank to arrive issues the launch on its stream behind every rank's pre-launch work (events) and the others'
// streams wait for it.
struct ksched_lgroup {
    int R = 0, dev = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool broken = false;        // a rank never arrived: the group is unusable
    int acc = 0, result = 0;    // FAST53 agreement
    PipeLaunch L{};             // the staged launch (rank r's arguments in L.P[r])
    hipStream_t stream[kMaxLocalRanks] = {};
    hipEvent_t ready[kMaxLocalRanks] = {};
    hipEvent_t done = nullptr;
    int kc = 0, k = 0, prio = 0, dom = 0;
    bool lab = false, f53 = false;
    hipError_t launch_err = hipSuccess;
    ~ksched_lgroup() {
        hipSetDevice(dev);
        for (int r = 0; r < kMaxLocalRanks; ++r)
            if (ready[r]) hipEventDestroy(ready[r]);
        if (done) hipEventDestroy(done);
    }
};

namespace {
// The R ranks of a local group meet: `mine` runs under the lock on arrival, `last` on the last arrival
// (before anyone is released).  false: a peer never arrived within 60 s (the group is then broken).
template <class Mine, class Last>
bool lg_meet(ksched_lgroup *g, Mine mine, Last last) {
    std::unique_lock<std::mutex> lk(g->mu);
    if (g->broken) return false;
    const uint64_t gen = g->gen;
    mine();
    if (++g->arrived == g->R) {
        last();
        g->arrived = 0;
        ++g->gen;
        g->cv.notify_all();
        return true;
    }
    if (!g->cv.wait_for(lk, std::chrono::seconds(60), [&] { return g->gen != gen; })) {
        g->broken = true;
        return false;
    }
    return true;
}

// all R ranks meet; returns the minimum of their values (false: a rank never arrived)
bool group_min(ksched_group *g, int v, int *out) {
    std::unique_lock<std::mutex> lk(g->mu);
    const uint64_t gen = g->gen;
    g->acc = g->arrived == 0 ? v : std::min(g->acc, v);
    if (++g->arrived == g->nranks) {
        g->result = g->acc;
        g->arrived = 0;
        ++g->gen;
        g->cv.notify_all();
    } else if (!g->cv.wait_for(lk, std::chrono::seconds(30), [&] { return g->gen != gen; })) {
        return false;
    }
    *out = g->result;
    return true;
}
}  // namespace

struct ksched_ctx {
    ksched_opts o{};
    int dev = 0;
    int cus = 256;
    hipStream_t stream = nullptr;
    std::string err;
    // nodes
    int64_t n_local = -1;
    int64_t n_global = 0;
    bool has_labels = false, has_price = false;
    uint64_t max_abs_alloc = 0;  // saturating bound on |allocatable| (fast53 check)
    uint64_t sum_abs_req = 0;    // saturating sum of |request| over the staged pods
    uint64_t snap_max_abs_alloc = 0;  // max_abs_alloc of the save_state snapshot
    NodeRec *d_nodes = nullptr, *d_snap = nullptr;
    int64_t node_cap = 0;
    // pods
    int64_t p = 0, p_cap = 0;
    int64_t *d_rc = nullptr, *d_rm = nullptr, *d_rp = nullptr;
    uint64_t *d_sel = nullptr;
    int32_t *d_oidx = nullptr, *d_ofeas = nullptr;
    double *d_osc = nullptr;
    // batched workspace
    int K = 16, KC = 4, B = 128;
    int64_t ws_bytes = 0;
    void *d_ws = nullptr;
    int64_t *d_cursor = nullptr;  // [0] cursor, [1..3] stats
    int64_t *h_cursor = nullptr;  // pinned
    int64_t *d_dbg = nullptr;     // KSCHED_COMMIT_STAMPS diagnostics
    uint32_t jitter_calls = 0;    // KSCHED_JITTER: calls so far (the seed changes per call)
    int64_t *d_mdbg = nullptr;    // KSCHED_MERGE_STAMPS diagnostics
    hipStream_t stream2 = nullptr;  // merge + commit stream of the batched pipeline
    hipEvent_t ev_lists[4] = {}, ev_commit[4] = {}, ev_scored[4] = {}, ev_pipe[3] = {};
    void *d_xring = nullptr, *d_lring = nullptr;
    int64_t xring_bytes = 0, lring_bytes = 0;
    // exact workspace
    uint64_t *d_slots = nullptr;
    int32_t *d_perm = nullptr;     // exact mode on one workgroup, best-price: nodes by (price asc, index asc)
    int64_t perm_cap = 0;
    int32_t *d_err = nullptr;
    int64_t slots_cap = 0;
    // multi-GPU
    ncclComm_t comm = nullptr;
    ksched_group *group = nullptr;  // in-process rank group (instead of comm)
    // timing
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool running = false;
    bool fast53 = false;
    std::vector<hipEvent_t> ev_pool;  // sampled per-family event pairs (opts.timing)
    struct Timed { int fam; int e0, e1; int64_t pairs; };
    std::vector<Timed> timed;
    size_t ev_used = 0;
    ksched_stats st{};
    int64_t run_batches = 0;
    // batch FailedScheduling diagnostics (ksched_explain_batch / ksched_explain_pod)
    bool explain_valid = false;  // the last state change was the last schedule call's placements
    void *d_xws = nullptr;
    size_t xws_bytes = 0;
    void *d_xbuf = nullptr;      // counts + NO_FIT pod list, or one pod's state + counts
    size_t xbuf_bytes = 0;
    // persistent single-rank pipeline (ksched_persist.hip)
    void *d_pws = nullptr;       // per-workgroup part lists + counts
    uint64_t *d_prog = nullptr;   // persistent pipeline: per-workgroup progress words (in d_pws)
    int prog_G = 0, prog_B = 0, prog_rows = 0;
    uint64_t *d_trace = nullptr;  // KSCHED_PERSIST_TRACE: per-batch wall-clock stamps
    int64_t trace_cap = 0;
    uint64_t *d_xdbg = nullptr;      // KSCHED_XCHG_DUMP: the exchange's message hashes (PersistArgs::xdbg)
    int64_t xdbg_cap = 0, xdbg_calls = 0;
    uint64_t *d_trace_wg = nullptr;  // KSCHED_TRACE_WG: per batch and score workgroup {start, arrival}
    int64_t trace_wg_elems = 0;
    size_t pws_bytes = 0;
    bool persist_stats = false;  // stats come from the Ctl copy queued behind the run
    int64_t persist_B = 0;
    // device-side candidate exchange of the node-sharded persistent pipeline (ksched_xchg_*)
    void *d_rx = nullptr;          // this rank's receive ring (rx_prepare)
    size_t rx_bytes = 0;
    bool rx_uncached = false;      // d_rx is hipDeviceMallocUncached memory (xchg_export's kind)
    char *rx_peer[kMaxXchgRanks] = {};  // every rank's ring as mapped here (own = d_rx)
    bool rx_ipc[kMaxXchgRanks] = {};    // rx_peer[r] was opened by hipIpcOpenMemHandle (closed by rx_unmap_peers)
    bool xchg_ready = false;       // rings imported: batched runs take the persistent multi-rank path
    bool xchg_run = false;         // the current run uses the exchange
    uint32_t xchg_epoch = 1;       // granule tag base of the next call (identical on every rank)
    int32_t *d_xmin = nullptr;     // k_xchg_min result
    std::shared_ptr<ksched_lgroup> lg;  // ranks of this process on this device (ksched_xchg_join_local)
    // diagnostics, read from the environment once at ksched_create (never a tuning switch):
    //   KSCHED_PERSIST_TRACE=1   per-batch phase stamps of the persistent pipeline, summary to stderr at sync
    //   KSCHED_COMMIT_STAMPS=1   commit phase cycle sums;  KSCHED_MERGE_STAMPS=1  merge phase cycle sums
    //   KSCHED_PERSIST_TIMEOUT_MS (10000)  bound of every persistent-pipeline wait (tests force timeouts with 0)
    //   KSCHED_EXCHANGE_TIMEOUT_MS (2000)  bound of the exact kernel's cross-workgroup exchange
    //   KSCHED_DEBUG=1           launch decisions to stderr
    struct {
        bool trace = false, commit_stamps = false, merge_stamps = false, debug = false;
        bool no_screen = false;  // KSCHED_NO_SCREEN: the exact scan everywhere (A/B of the screened scan)
        bool no_pairs = false;   // KSCHED_NO_PAIRS: the screened scan's exact phase by rows (A/B of the pair lists)
        bool poison = false;     // KSCHED_POISON: workspace and LDS filled with 0xff before every persistent run
        int xchg_diag = 0;       // KSCHED_XCHG_DIAG (section 6.1's experiment): 1 ring zeroed by hipMemsetAsync, 2 local tags from 1
        int64_t epoch_base = 0;
        int exact1_bs = 1024;    // KSCHED_EXACT1_BS (A/B): the one-workgroup exact kernel's block (1024, 512, 256)  // KSCHED_XCHG_EPOCH_BASE (tests): a setup's granule tags start at least here (near 2^15: wrap)
        bool plain_launch = false;  // KSCHED_PLAIN_LAUNCH: the persistent kernels without the cooperative launch API
                                    // (same residency check; profiled runs: DESIGN.md section 6.1)
        uint32_t jitter = 0;     // KSCHED_JITTER=<seed>: random delays at the persistent pipeline's protocol points
        bool touch_screen = true;  // KSCHED_NO_TOUCH_SCREEN=1: the commit keys every touched node exactly
        // the rescue policy (the rescue table).  A rescue costs ~20 us of the commit's loop,
        // a truncation ~2 voided batches, so rescues pay where exhausted lists are rare and lose where they cluster
        // (the rescues of a batch that truncates anyway are wasted).  Each commit workgroup keeps a bucket of
        // credit: rescue_rate quarter rescues per batch of its own, at most rescue_cap rescues; a batch spends at
        // most rescue_max while the bucket is at least half full and rescue_low below that
        int rescue_max = 4;      // KSCHED_RESCUE_MAX (0: exhausted lists always truncate)
        int rescue_rate = 4;     // KSCHED_RESCUE_RATE, quarter rescues per batch of the workgroup
        int rescue_cap = 16;     // KSCHED_RESCUE_CAP
        int rescue_low = 2;      // KSCHED_RESCUE_LOW
        int rescue_look = 0;     // KSCHED_RESCUE_LOOK=1: also truncate when the batch's other exhausted lists would
                                 // overrun the allowance (helps a fixed budget, loses with the bucket)
        int64_t persist_timeout_ms = 10000, exchange_timeout_ms = 2000;
    } diag;
};

namespace {

int fail(ksched_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    return code;
}

#define HIPCHK(c, expr)                                                                        \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) {                                                                \
            (void)hipGetLastError(); /* reported here: not again by a later launch's check */   \
            return fail((c), KSCHED_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
        }                                                                                      \
    } while (0)

#define NCCLCHK(c, expr)                                                                       \
    do {                                                                                       \
        ncclResult_t r_ = (expr);                                                              \
        if (r_ != ncclSuccess)                                                                 \
            return fail((c), KSCHED_E_DEVICE, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

template <typename T>
hipError_t grow(T **ptr, int64_t *cap, int64_t need, size_t elem) {
    if (*ptr && *cap >= need) return hipSuccess;
    if (*ptr) { hipFree(*ptr); *ptr = nullptr; }
    *cap = 0;
    hipError_t e = hipMalloc((void **)ptr, (size_t)std::max<int64_t>(need, 1) * elem);
    if (e == hipSuccess) *cap = need;
    return e;
}

uint64_t sat_add(uint64_t a, uint64_t b) { return a + b < a ? UINT64_MAX : a + b; }
uint64_t uabs(int64_t v) { return v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v; }

int env_int(const char *name, int dflt) {
    const char *v = std::getenv(name);
    return v && *v ? std::atoi(v) : dflt;
}

// Sampled kernel timing: a (start, stop) event pair around one kernel family of one batch.
hipError_t ev_take(ksched_ctx *c, int *idx) {
    if (c->ev_used >= c->ev_pool.size()) {
        hipEvent_t e;
        hipError_t r = hipEventCreate(&e);
        if (r != hipSuccess) return r;
        c->ev_pool.push_back(e);
    }
    *idx = (int)c->ev_used++;
    return hipSuccess;
}

hipError_t ev_begin(ksched_ctx *c, bool on, int *e0, hipStream_t s) {
    if (!on) return hipSuccess;
    hipError_t r = ev_take(c, e0);
    if (r != hipSuccess) return r;
    return hipEventRecord(c->ev_pool[(size_t)*e0], s);
}

hipError_t ev_end(ksched_ctx *c, bool on, int fam, int e0, int64_t pairs, hipStream_t s) {
    if (!on) return hipSuccess;
    int e1;
    hipError_t r = ev_take(c, &e1);
    if (r != hipSuccess) return r;
    r = hipEventRecord(c->ev_pool[(size_t)e1], s);
    if (r == hipSuccess) c->timed.push_back({fam, e0, e1, pairs});
    return r;
}

// Batched-mode geometry for one schedule call.
struct BatchPlan {
    int K, KC, B, pod_groups;
    int S, n_chunks;       // score kernel: nodes per chunk, chunks
    int stages;            // merge stages (chunk lists -> final)
    int C[4];              // lists per pod entering each stage
    size_t off_part, off_pcnt, off_m1, off_m1cnt, off_lists, off_fc, off_send, off_recv, off_glists, off_gfc;
    size_t send_bytes, total;
};

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

BatchPlan plan_batch(const ksched_ctx *c) {
    BatchPlan pl{};
    pl.K = c->K;
    pl.KC = c->KC;
    pl.B = c->B;
    pl.pod_groups = (pl.B + 63) / 64;
    const int64_t n = std::max<int64_t>(c->n_local, 1);
    // NSC sub-chunks (one wave each) in workgroups of kScoreWaves: 8 waves per CU at full size,
    // >= 16 nodes per wave, <= kMergeThreads workgroups (one merge lane per list)
    const int target_waves = c->cus * 8;
    int64_t nsc = std::max<int64_t>(1, target_waves / pl.pod_groups);
    const int min_s = 16;
    nsc = std::min<int64_t>(nsc, (n + min_s - 1) / min_s);
    nsc = std::min<int64_t>(nsc, (int64_t)kMergeThreads * kScoreWaves);
    nsc = std::max<int64_t>(kScoreWaves, nsc / kScoreWaves * kScoreWaves);
    pl.n_chunks = (int)nsc;
    pl.S = (int)((n + nsc - 1) / nsc);
    const int G = (int)(nsc / kScoreWaves);
    pl.C[0] = G;
    pl.stages = 1;
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off = align_up(off + bytes, 256); return o; };
    pl.off_part = take((size_t)2 * pl.B * G * pl.KC * sizeof(Cand));  // ring of 2: score(b+1) || merge(b)
    pl.off_pcnt = take((size_t)2 * pl.B * G * sizeof(int64_t));
    pl.off_m1 = pl.off_m1cnt = 0;
    pl.send_bytes = (size_t)pl.B * pl.K * sizeof(Rec) + (size_t)pl.B * sizeof(int64_t);
    pl.off_send = take(pl.send_bytes);  // local lists + fc (also the single-GPU final lists)
    const int R = std::max(1, c->o.nranks);
    pl.off_recv = take(pl.send_bytes * R);
    pl.off_glists = take((size_t)2 * pl.B * pl.K * sizeof(Rec));  // ring of 2 (rank-merged lists)
    pl.off_gfc = take((size_t)2 * pl.B * sizeof(int64_t));
    pl.off_lists = pl.off_send;
    pl.off_fc = pl.off_send + (size_t)pl.B * pl.K * sizeof(Rec);
    pl.total = off;
    return pl;
}


// The exchange fields of PersistArgs (node-sharded persistent pipeline; R > 1).
void fill_xchg_args(const ksched_ctx *c, PersistArgs *a) {
    a->B = c->B;
    a->node_offset = c->o.node_offset;
    a->R = c->xchg_run ? c->o.nranks : 1;
    a->rank = c->xchg_run ? c->o.rank : 0;
    a->epoch0 = c->xchg_epoch;
    a->xchg_stride = (int64_t)xchg_stride_bytes(c->K);
    for (int r = 0; r < kMaxXchgRanks; ++r) a->rx_peer[r] = c->rx_peer[r];
}

// The receive ring of a node-sharded rank, for every way an exchange is set up (ksched_xchg_export,
// ksched_xchg_join_local_ex): (re)allocated when its size or memory kind changes, and ZEROED AT EVERY SETUP, in
// this context's stream order and finished, before any peer can learn where it is.  So a ring never holds a
// granule of an earlier setup, and every setup's epochs start at 1 (tag 0 is never live) -- the one epoch rule
// of both paths.  Uncached (hipDeviceMallocUncached): a peer GPU's xGMI stores and this GPU's polls meet in
// memory, never in a stale L2 line.
// Uncached rings are never given back to the allocator: a page the allocator hands out uncached and later cached
// again (or the reverse) was read stale by the cached side -- L2 lines of its earlier cached use survive the uncached
// stores, and a later buffer on those pages (a group's node rows) read them back: the round-4 exchange failure
// (DESIGN.md section 6.1).  A process-wide pool per device keeps every uncached page uncached for good.
struct UcPool {
    std::mutex mu;
    std::vector<std::tuple<int, void *, size_t>> free;  // (device, block, bytes)
};
UcPool &uc_pool() {
    static UcPool *p = new UcPool();  // never destroyed: its blocks outlive every context
    return *p;
}
hipError_t uc_alloc(int dev, size_t bytes, void **out, size_t *got) {
    UcPool &P = uc_pool();
    {
        std::lock_guard<std::mutex> lk(P.mu);
        size_t best = SIZE_MAX;
        int bi = -1;
        for (int i = 0; i < (int)P.free.size(); ++i) {
            const auto &[d, q, n] = P.free[(size_t)i];
            if (d == dev && n >= bytes && n < best) { best = n; bi = i; }
        }
        if (bi >= 0) {
            *out = std::get<1>(P.free[(size_t)bi]);
            *got = best;
            P.free.erase(P.free.begin() + bi);
            return hipSuccess;
        }
    }
    *got = bytes;
    return hipExtMallocWithFlags(out, bytes, hipDeviceMallocUncached);
}
void uc_release(int dev, void *p, size_t bytes) {
    UcPool &P = uc_pool();
    std::lock_guard<std::mutex> lk(P.mu);
    P.free.emplace_back(dev, p, bytes);
}
void rx_free(ksched_ctx *c) {
    if (c->d_rx) {
        if (c->rx_uncached) uc_release(c->dev, c->d_rx, c->rx_bytes);
        else hipFree(c->d_rx);
    }
    c->d_rx = nullptr;
    c->rx_bytes = 0;
}

int rx_prepare(ksched_ctx *c, size_t bytes, bool uncached) {
    if (c->d_rx && (c->rx_bytes < bytes || c->rx_uncached != uncached)) rx_free(c);
    if (!c->d_rx) {
        size_t got = bytes;
        if (uncached) HIPCHK(c, uc_alloc(c->dev, bytes, &c->d_rx, &got));
        else HIPCHK(c, hipMalloc(&c->d_rx, bytes));
        c->rx_bytes = got;
        c->rx_uncached = uncached;
    }
    // zeroed by system-scope stores, the granules' own path (a hipMemsetAsync of an uncached ring was not what the
    // persistent kernel's system-scope loads read afterwards: the round-4 failure)
    if (c->diag.xchg_diag & 1) HIPCHK(c, hipMemsetAsync(c->d_rx, 0, c->rx_bytes, c->stream));  // round 4's way
    else HIPCHK(c, launch_zero_sys(c->d_rx, c->rx_bytes, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return KSCHED_OK;
}

// The first granule tag no ring of this process has used yet.  Every setup starts its tags at (at least) this
// value on every rank, and every call moves it past the tags it used, so a tag never repeats in this process's
// memory: a granule left in memory that a new ring reuses can never carry a tag the new setup waits for, even
// where zeroing the ring did not reach what its loads read.
std::atomic<uint32_t> g_epoch_next{1};
void epoch_used_below(uint32_t e) {
    uint32_t cur = g_epoch_next.load();
    while (cur < e && !g_epoch_next.compare_exchange_weak(cur, e)) {}
}

// forget every peer ring this context mapped (IPC maps are closed; a local group's peers are plain pointers)
void rx_unmap_peers(ksched_ctx *c) {
    for (int r = 0; r < kMaxXchgRanks; ++r) {
        if (c->rx_ipc[r] && c->rx_peer[r]) hipIpcCloseMemHandle(c->rx_peer[r]);
        c->rx_peer[r] = nullptr;
        c->rx_ipc[r] = false;
    }
}

// rank r's ring as this context maps it from its IPC handle (ksched_xchg_import, and the local group's IPC mode)
int rx_map_peer(ksched_ctx *c, int r, const uint8_t *handle) {
    hipIpcMemHandle_t h;
    static_assert(sizeof(hipIpcMemHandle_t) + 8 <= KSCHED_XCHG_HANDLE_BYTES, "ipc handle + epoch hint");
    std::memcpy(&h, handle, sizeof(h));
    void *p = nullptr;
    HIPCHK(c, hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    c->rx_peer[r] = static_cast<char *>(p);
    c->rx_ipc[r] = true;
    return KSCHED_OK;
}

// Before every call's rank barrier each rank zeroes its own ring's message and rescue areas (not the barrier
// granules the barrier itself uses): granule tags keep 15 bits (gran_tag), so a region a call does not rewrite --
// the rescue area when no rescue happens, the message slots of a call with fewer than four active batches -- could
// otherwise hold, calls later, a granule whose tag matches a wait modulo 2^15.  A peer writes into this
// ring only after it has seen this rank at the barrier, which this rank reaches after the zeroing kernel finished
// (stream order), so no granule of the call is lost.  Within a call a region is rewritten every 4 active batches
// (messages) or every 2 rescues, and both are zeroed again by the next call.
int rx_zero_regions(ksched_ctx *c) {
    const int R = c->o.nranks;
    const size_t stride = xchg_stride_bytes(c->K);
    const size_t msg = (size_t)4 * R * c->B * stride;
    const size_t resc = xchg_rescue_off(R, c->B, stride);
    if (!c->d_rx || c->rx_bytes < xchg_ring_bytes(R, c->B, c->K)) return fail(c, KSCHED_E_STATE, "exchange ring missing");
    HIPCHK(c, launch_zero_sys(c->d_rx, msg, c->stream));
    HIPCHK(c, launch_zero_sys(static_cast<char *>(c->d_rx) + resc, 2 * (size_t)R * kXchgRescueRec, c->stream));
    return KSCHED_OK;
}

// fast53 for this call: every |alloc| + sum of |requests| < 2^52, on every rank.
int decide_fast53(ksched_ctx *c) {
    int flag = sat_add(c->max_abs_alloc, c->sum_abs_req) < (1ull << 52) ? 1 : 0;
    if (c->group) {
        int mn = flag;
        if (!group_min(c->group, flag, &mn)) return fail(c, KSCHED_E_DEVICE, "rank group: a peer never called run");
        flag = mn;
    } else if (c->xchg_run && c->lg) {
        ksched_lgroup *g = c->lg.get();
        int mn = flag;
        if (int rc = rx_zero_regions(c); rc != KSCHED_OK) return rc;
        HIPCHK(c, hipStreamSynchronize(c->stream));  // finished before any rank of the group can launch
        if (!lg_meet(g, [&] { g->acc = g->arrived == 0 ? flag : std::min(g->acc, flag); }, [&] { g->result = g->acc; }))
            return fail(c, KSCHED_E_DEVICE, "local rank group: a peer never called run");
        mn = g->result;
        flag = mn;
    } else if (c->xchg_run) {
        // the ranks meet on the device through their rings (no collective launch)
        PersistArgs a{};
        fill_xchg_args(c, &a);
        a.err = c->d_err;
        a.timeout_ticks = c->diag.persist_timeout_ms * 100000;
        int32_t mn = -1;
        if (int rc = rx_zero_regions(c); rc != KSCHED_OK) return rc;  // stream-ordered before the barrier
        HIPCHK(c, launch_xchg_min(a, flag, c->d_xmin, c->stream));
        HIPCHK(c, hipMemcpyAsync(&mn, c->d_xmin, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (mn < 0) {
            c->xchg_ready = false;
            (void)hipMemsetAsync(c->d_err, 0, sizeof(int32_t), c->stream);
            return fail(c, KSCHED_E_DEVICE, "node-sharded exchange: a peer rank never met this one (device barrier timed out)");
        }
        flag = mn;
    } else if (c->comm) {
        int32_t *d = c->d_err;  // scratch word (zeroed again before use by exact mode)
        HIPCHK(c, hipMemcpyAsync(d, &flag, sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
        NCCLCHK(c, ncclAllReduce(d, d, 1, ncclInt32, ncclMin, c->comm, c->stream));
        HIPCHK(c, hipMemcpyAsync(&flag, d, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipMemsetAsync(d, 0, sizeof(int32_t), c->stream));
    }
    c->fast53 = flag != 0;
    return KSCHED_OK;
}

// Batched mode, software-pipelined over two streams:
//   stream S: score(b)                     polls Ctl::committed >= b - 1 (commit(b-2) done) on the device,
//                                          then overlays / writes back b-2's commits as it scans
//   stream C: merge(b) [-> all-gather -> rank merge] -> commit(b)  (+ plan of batch b+2, publish)
// score(b) runs on every CU while commit(b-1) runs on one; commit(b) inherits the nodes committed by
// batch b-1 (its score snapshot is one batch older).  Each batch's start is planned speculatively
// (previous start + B) by the commit two batches back; a truncated batch invalidates the in-flight
// speculation, which commit skips, and plans its restart at the committed frontier.
// The commit(b-2) -> score(b) edge is a device-side flag (score(b) is already resident when it is
// released: ~2 us) instead of a cross-queue stream event (~13 us per batch measured on MI355X, even
// when the event has completed: profiles/r02_*) wherever the commit provably fits beside a resident
// score workgroup; score(b) -> merge(b) is a stream event.
int enqueue_batched(ksched_ctx *c) {
    const BatchPlan pl = plan_batch(c);
    if (c->ws_bytes < (int64_t)pl.total) {
        if (c->d_ws) hipFree(c->d_ws);
        c->d_ws = nullptr;
        c->ws_bytes = 0;
        HIPCHK(c, hipMalloc(&c->d_ws, pl.total));
        c->ws_bytes = (int64_t)pl.total;
    }
    const int64_t lds = (int64_t)commit_lds_bytes(pl.B, pl.K);
    if (lds > 160 * 1024 - 4096 || pl.B > 128)
        return fail(c, KSCHED_E_INVALID, "batched mode: batch <= 128 and B*(328+48K) <= ~150 KB of LDS");
    char *ws = static_cast<char *>(c->d_ws);
    const int prio = c->o.priority, dom = c->o.domain;
    const bool lab = c->o.use_labels != 0;
    const int R = std::max(1, c->o.nranks);
    PodArgs pods{c->d_rc, c->d_rm, c->d_rp, c->d_sel, c->p};
    const bool f53 = c->fast53;
    // commit implementation: speculative-parallel (B <= 64, default) or the single-wave sequencer (B <= 128)
    int impl = c->o.commit_impl ? c->o.commit_impl : KSCHED_COMMIT_SPECULATIVE;
    if (impl != KSCHED_COMMIT_SEQUENTIAL && pl.B > 64) impl = KSCHED_COMMIT_SEQUENTIAL;
    const bool spc_commit = impl != KSCHED_COMMIT_SEQUENTIAL;
    hipStream_t sS = c->stream, sC = c->stream2;
    // device-side score wait only where the commit provably fits beside a resident score workgroup
    const bool score_poll = commit_fits_beside_score(pl.KC, pl.K, pl.B, spc_commit, prio, dom, lab, f53);
    constexpr int kRing = 4;  // lists / X buffers / events in flight
    const size_t xb = xbuf_bytes(pl.B);
    if (c->xring_bytes < (int64_t)(xb * (kRing + 1))) {
        if (c->d_xring) hipFree(c->d_xring);
        c->d_xring = nullptr;
        HIPCHK(c, hipMalloc(&c->d_xring, xb * (kRing + 1)));
        c->xring_bytes = (int64_t)(xb * (kRing + 1));
    }
    if (c->lring_bytes < (int64_t)(pl.send_bytes * kRing)) {
        if (c->d_lring) hipFree(c->d_lring);
        c->d_lring = nullptr;
        HIPCHK(c, hipMalloc(&c->d_lring, pl.send_bytes * kRing));
        c->lring_bytes = (int64_t)(pl.send_bytes * kRing);
    }
    auto xbuf = [&](int64_t b) -> XBuf * {  // b = -1 -> the permanently empty buffer
        const int64_t slot = b < 0 ? kRing : (b % kRing);
        return reinterpret_cast<XBuf *>(static_cast<char *>(c->d_xring) + (size_t)slot * xb);
    };
    Ctl *ctl = reinterpret_cast<Ctl *>(c->d_cursor);
    HIPCHK(c, launch_ctl_init(ctl, pl.B, c->p, 2, sS));
    for (int r = 0; r <= kRing; ++r) HIPCHK(c, hipMemsetAsync(xbuf(r == kRing ? -1 : r), 0, 8, sS));
    if (c->diag.commit_stamps && !c->d_dbg) HIPCHK(c, hipMalloc(&c->d_dbg, 32 * sizeof(int64_t)));
    if (c->d_dbg) HIPCHK(c, hipMemsetAsync(c->d_dbg, 0, 32 * sizeof(int64_t), sS));
    if (c->diag.merge_stamps && !c->d_mdbg) HIPCHK(c, hipMalloc(&c->d_mdbg, 8 * sizeof(int64_t)));
    if (c->d_mdbg) HIPCHK(c, hipMemsetAsync(c->d_mdbg, 0, 8 * sizeof(int64_t), sS));
    HIPCHK(c, hipEventRecord(c->ev_pipe[0], sS));  // stream C starts after the initialisation above
    HIPCHK(c, hipStreamWaitEvent(sC, c->ev_pipe[0], 0));
    int64_t resolved = 0, b = 0;
    double avg_progress = std::max(1.0, pl.B * 0.75);
    while (resolved < c->p) {
        int64_t m = (int64_t)std::ceil((double)(c->p - resolved) / avg_progress) + 2;
        m = std::max<int64_t>(2, std::min<int64_t>(m, 256));
        const int64_t b_end = b + m;
        for (; b < b_end; ++b) {
            const bool tm = c->o.timing && (b % (c->o.timing_every > 0 ? c->o.timing_every : 16) == 0);
            int e0 = -1;
            const int slot = (int)(b % kPlanRing);
            const int64_t *plan = &ctl->plan[slot];
            char *lists_base = static_cast<char *>(c->d_lring) + (size_t)(b % kRing) * pl.send_bytes;
            // S: score b once commit(b-2) is done (its plan for b and its committed nodes, which score(b)
            // overlays on the rows it reads and writes back)
            ScoreArgs sa{};
            if (b >= 2) {
                if (score_poll) { sa.wait_committed = &ctl->committed; sa.wait_target = (unsigned long long)(b - 1); }
                else HIPCHK(c, hipStreamWaitEvent(sS, c->ev_commit[(b - 2) % kRing], 0));
            }
            sa.err = c->d_err;
            sa.nodes = c->d_nodes; sa.n_local = c->n_local; sa.node_offset = c->o.node_offset;
            sa.S = pl.S; sa.n_chunks = pl.n_chunks; sa.pods = pods; sa.cursor = plan; sa.B = pl.B;
            const size_t part_elems = (size_t)pl.B * pl.C[0];
            sa.part = reinterpret_cast<Cand *>(ws + pl.off_part) + (size_t)(b % 2) * part_elems * pl.KC;
            sa.part_cnt = reinterpret_cast<int64_t *>(ws + pl.off_pcnt) + (size_t)(b % 2) * part_elems;
            sa.patch = xbuf(b - 2);
            MergeArgs ma{};
            ma.in = sa.part; ma.in_cnt = sa.part_cnt; ma.C_in = pl.C[0]; ma.C_out = 1; ma.chunk_input = 1;
            ma.cursor = plan; ma.P = c->p; ma.B = pl.B;
            ma.nodes = c->d_nodes; ma.node_offset = c->o.node_offset;
            ma.dbg = c->d_mdbg;
            ma.err = c->d_err;
            ma.out_rec = reinterpret_cast<Rec *>(lists_base);
            ma.out_fc = reinterpret_cast<int64_t *>(lists_base + (size_t)pl.B * pl.K * sizeof(Rec));
            HIPCHK(c, ev_begin(c, tm, &e0, sS));
            HIPCHK(c, launch_score_topk(pl.KC, prio, dom, lab, f53, sa, pl.pod_groups, sS));
            HIPCHK(c, ev_end(c, tm, 0, e0, (int64_t)pl.B * c->n_local, sS));
            // C: merge b while stream S scores b+1 (the lists' part buffers alternate)
            HIPCHK(c, hipEventRecord(c->ev_scored[b % kRing], sS));
            HIPCHK(c, hipStreamWaitEvent(sC, c->ev_scored[b % kRing], 0));
            HIPCHK(c, ev_begin(c, tm, &e0, sC));
            HIPCHK(c, launch_merge_pod(pl.KC, pl.K, ma, sC));
            HIPCHK(c, ev_end(c, tm, 1, e0, 0, sC));
            const Rec *lists = reinterpret_cast<const Rec *>(lists_base);
            const int64_t *fc0 = reinterpret_cast<const int64_t *>(lists_base + (size_t)pl.B * pl.K * sizeof(Rec));
            if (c->comm || c->group) {  // node-sharded: exchange the local lists (a 1-rank communicator also takes this path)
                HIPCHK(c, ev_begin(c, tm, &e0, sC));
                if (c->comm) {
                    NCCLCHK(c, ncclAllGather(lists_base, ws + pl.off_recv, pl.send_bytes, ncclUint8, c->comm, sC));
                } else {
                    ksched_group *g = c->group;
                    int dummy;
                    HIPCHK(c, hipEventRecord(c->ev_pipe[0], sC));
                    HIPCHK(c, hipEventSynchronize(c->ev_pipe[0]));  // my block is final
                    g->send[(size_t)c->o.rank] = lists_base;
                    if (!group_min(g, 0, &dummy)) return fail(c, KSCHED_E_DEVICE, "rank group: a peer stopped exchanging");
                    for (int q = 0; q < R; ++q)
                        HIPCHK(c, hipMemcpyAsync(ws + pl.off_recv + (size_t)q * pl.send_bytes, g->send[(size_t)q],
                                                 pl.send_bytes, hipMemcpyDeviceToDevice, sC));
                    HIPCHK(c, hipStreamSynchronize(sC));
                    if (!group_min(g, 0, &dummy)) return fail(c, KSCHED_E_DEVICE, "rank group: a peer stopped exchanging");
                }
                MergeArgs mr{};
                mr.in = ws + pl.off_recv; mr.rank_stride = (int64_t)pl.send_bytes; mr.C_in = R; mr.C_out = 1;
                mr.cursor = plan; mr.P = c->p; mr.B = pl.B;
                mr.out_rec = reinterpret_cast<Rec *>(ws + pl.off_glists) + (size_t)(b % 2) * pl.B * pl.K;
                mr.out_fc = reinterpret_cast<int64_t *>(ws + pl.off_gfc) + (size_t)(b % 2) * pl.B;
                HIPCHK(c, launch_merge(pl.K, pl.K, true, true, mr, sC));
                lists = mr.out_rec;
                fc0 = mr.out_fc;
                HIPCHK(c, ev_end(c, tm, 3, e0, 0, sC));
            }
            // C: ordered commit of batch b
            CommitArgs ca{};
            ca.lists = lists; ca.fc0 = fc0; ca.pods = pods; ca.plan = plan; ca.ctl = ctl; ca.B = pl.B;
            ca.plan1 = &ctl->plan[(b + 1) % kPlanRing];
            ca.plan2 = &ctl->plan[(b + 2) % kPlanRing];
            ca.xin = xbuf(b - 1); ca.xout = xbuf(b);
            ca.out = OutArgs{c->d_oidx, c->d_osc, c->d_ofeas};
            ca.dbg = c->d_dbg;
            ca.batch = b;
            HIPCHK(c, ev_begin(c, tm, &e0, sC));
            if (spc_commit) HIPCHK(c, launch_commit_spc(pl.K, prio, dom, lab, f53, ca, sC));
            else HIPCHK(c, launch_commit(pl.K, prio, dom, lab, f53, ca, (size_t)lds, sC));
            HIPCHK(c, ev_end(c, tm, 2, e0, 0, sC));
            HIPCHK(c, hipEventRecord(c->ev_commit[b % kRing], sC));
        }
        HIPCHK(c, hipMemcpyAsync(c->h_cursor, ctl, sizeof(Ctl), hipMemcpyDeviceToHost, sC));
        HIPCHK(c, hipStreamSynchronize(sC));
        const Ctl *h = reinterpret_cast<const Ctl *>(c->h_cursor);
        if (h->cursor <= resolved) return fail(c, KSCHED_E_DEVICE, "batched mode made no progress");
        resolved = h->cursor;
        if (h->stats[0] > 0) avg_progress = std::max(1.0, (double)resolved / (double)(b));
    }
    // drain: write back the last two batches' commits (the others were applied in the pipeline)
    for (int64_t bb = std::max<int64_t>(0, b - 2); bb < b; ++bb) {
        HIPCHK(c, hipStreamWaitEvent(sS, c->ev_commit[bb % kRing], 0));
        HIPCHK(c, launch_apply_batch(xbuf(bb), c->d_nodes, c->o.node_offset, c->n_local, sS));
    }
    // the run's end event is recorded on stream S: make it cover stream C
    HIPCHK(c, hipEventRecord(c->ev_pipe[1], sC));
    HIPCHK(c, hipStreamWaitEvent(sS, c->ev_pipe[1], 0));
    if (c->d_mdbg) {
        int64_t hm[8];
        HIPCHK(c, hipStreamSynchronize(sS));
        HIPCHK(c, hipMemcpy(hm, c->d_mdbg, sizeof(hm), hipMemcpyDeviceToHost));
        const double nwg = hm[7] ? (double)hm[7] : 1.0;
        std::fprintf(stderr, "[ksched merge stamps] workgroups=%lld | cycles/wg: loads %.0f rank-heads %.0f barrier %.0f "
                     "global-heads %.0f rank-entries %.0f write %.0f\n", (long long)hm[7], hm[0] / nwg, hm[1] / nwg,
                     hm[2] / nwg, hm[3] / nwg, hm[4] / nwg, hm[5] / nwg);
    }
    const Ctl *h = reinterpret_cast<const Ctl *>(c->h_cursor);
    c->st.batches = h->stats[0];
    c->st.truncations = h->stats[1];
    c->st.placed = h->stats[2];
    c->st.pair_evals = (h->stats[0] + h->stats[3]) * (int64_t)pl.B * c->n_local;
    c->run_batches = b;
    if (c->d_dbg) {
        int64_t hd[16];
        HIPCHK(c, hipStreamSynchronize(sS));
        HIPCHK(c, hipMemcpy(hd, c->d_dbg, sizeof(hd), hipMemcpyDeviceToHost));
        if (spc_commit)
            std::fprintf(stderr, "[ksched commit_spc] kernels=%lld rounds=%lld failures=%lld (%.3f rounds/batch) | "
                         "cycles/kernel: prologue %.0f guess %.0f evaluate %.0f check %.0f total %.0f\n",
                         (long long)hd[14], (long long)hd[12], (long long)hd[13], (double)hd[12] / (hd[14] ? hd[14] : 1),
                         (double)hd[0] / hd[14], (double)hd[1] / hd[14], (double)hd[2] / hd[14], (double)hd[3] / hd[14],
                         (double)hd[4] / hd[14]);
        else
            std::fprintf(stderr, "[ksched commit stamps] pods=%lld kernels=%lld touched=%lld | cycles/pod: loads+rescore %.0f "
                         "reduce %.0f decide %.0f commit+store %.0f | loop cycles/pod %.0f | skipped %lld\n",
                         (long long)hd[5], (long long)hd[7], (long long)hd[6], (double)hd[0] / hd[5], (double)hd[1] / hd[5],
                         (double)hd[2] / hd[5], (double)hd[3] / hd[5], (double)hd[4] / hd[5], (long long)h->stats[3]);
    }
    return KSCHED_OK;
}

// KSCHED_PERSIST_TRACE=1: mean per-batch phase times of the last persistent run, to stderr (us)
void print_persist_trace(ksched_ctx *c) {
    std::vector<uint64_t> t((size_t)c->trace_cap * kTraceCols);
    if (hipMemcpy(t.data(), c->d_trace, t.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    // KSCHED_TRACE_DUMP=<path>: the raw stamps ([trace_cap][kTraceCols] u64, 100 MHz) for offline percentiles
    if (const char *dump = std::getenv("KSCHED_TRACE_DUMP")) {
        if (FILE *f = std::fopen(dump, "wb")) {
            std::fwrite(t.data(), 8, t.size(), f);
            std::fclose(f);
        }
    }
    auto at = [&](int64_t b, int col) { return t[(size_t)b * kTraceCols + col]; };
    double sum[16] = {};
    double scr[5] = {};  // WG 0 wave 0, screened batches: pass 1, bound merge, pass 2, exact phase (sums), exact rows
    int64_t nscr = 0, npair = 0;
    double pairs_sum = 0;  // WG 0: batches whose exact phase ran over the pair lists, and their pairs
    int64_t cnt = 0, first = -1, last = -1;
    constexpr int64_t L = kPipeLag;
    for (int64_t b = L; b < c->trace_cap; ++b) {
        if (!at(b, 0) || !at(b, 1) || !at(b, 2) || !at(b, 3) || !at(b, 4) || !at(b - L, 4)) continue;
        if (first < 0) first = b;
        last = b;
        ++cnt;
        sum[0] += (double)(int64_t)(at(b, 0) - at(b - L, 4));  // commit(b-L) end -> score(b) start
        sum[1] += (double)(int64_t)(at(b, 1) - at(b, 0));      // score (WG 0 start -> last arrival)
        sum[2] += (double)(int64_t)(at(b, 2) - at(b, 1));      // merge
        sum[3] += (double)(int64_t)(at(b, 3) - at(b, 2));      // last merge -> commit start
        sum[4] += (double)(int64_t)(at(b, 4) - at(b, 3));      // commit
        sum[5] += (double)(int64_t)(at(b, 3) - at(b - 1, 4));  // commit(b-1) end -> commit(b) start
        sum[6] += (double)(int64_t)(at(b, 6) - at(b - L, 4));  // WG 0: commit(b-L) end -> its poll returns
        sum[7] += (double)(int64_t)(at(b, 0) - at(b, 6));      // WG 0: plan loads + XBuf apply
        sum[8] += (double)(int64_t)(at(b, 5) - at(b, 0));      // WG 0: score + fold + list stores
        sum[9] += (double)(int64_t)(at(b, 7) - at(b, 1));      // last arrival -> merger past its poll
        sum[10] += (double)(int64_t)(at(b, 8) - at(b, 0));     // WG 0 wave 0: row loop (incl. pod loads)
        sum[11] += (double)(int64_t)(at(b, 9) - at(b, 8));     // WG 0: waiting for its slowest wave
        sum[12] += (double)(int64_t)(at(b, 10) - at(b, 9));    // WG 0: fold
        sum[13] += (double)(int64_t)(at(b, 5) - at(b, 10));    // WG 0: list stores + drain
        sum[14] += (double)(int64_t)(at(b, 15) - at(b - 1, 4));  // commit(b-1) end -> commit loop top of b
        sum[15] += (double)(int64_t)(at(b, 3) - at(b, 15));      // commit loop top -> past the merge wait
        if (at(b, 11) && at(b, 12)) {  // a screened batch (ksched_pipe.hip score_role)
            ++nscr;
            scr[0] += (double)(int64_t)(at(b, 11) - at(b, 0));
            scr[1] += (double)(int64_t)(at(b, 12) - at(b, 11));
            scr[2] += (double)(int64_t)(at(b, 14) - at(b, 12));
            scr[3] += (double)(int64_t)(at(b, 8) - at(b, 14));
            scr[4] += (double)(uint32_t)at(b, 13);
            const uint32_t pairs = (uint32_t)(at(b, 13) >> 32);
            if (pairs != 0xffffffffu) { ++npair; pairs_sum += pairs; }
        }
    }
    if (c->d_dbg) {
        int64_t hd[32];
        if (hipMemcpy(hd, c->d_dbg, sizeof(hd), hipMemcpyDeviceToHost) == hipSuccess && hd[14] && hd[16])
            fprintf(stderr, "persist commit screen: export(b-1) entries %lld keyed exactly %.4f | guessed columns %lld, "
                    "exactly %.4f | sequential columns %lld, exactly %.4f | rescue re-keys %lld\n", (long long)hd[16],
                    (double)hd[17] / std::max<int64_t>(1, hd[16]), (long long)hd[18], (double)hd[19] / std::max<int64_t>(1, hd[18]),
                    (long long)hd[20], (double)hd[21] / std::max<int64_t>(1, hd[20]), (long long)hd[22]);
        if (hd[14])
            fprintf(stderr, "persist commit: batches=%lld rounds/batch %.3f guess iterations/round %.2f failures %lld | "
                    "cycles/batch: before the wait %.0f (other waves %.0f) entry to past the wait %.0f (poll %.0f, poll + barrier %.0f, early read sufficed %.3f) | prologue %.0f guess %.0f evaluate %.0f check %.0f total %.0f\n",
                    (long long)hd[14], (double)hd[12] / hd[14], (double)hd[5] / std::max<int64_t>(1, hd[12]),
                    (long long)hd[13], (double)hd[6] / hd[14], (double)hd[9] / hd[14] / 11.0, (double)hd[7] / hd[14], (double)hd[10] / hd[14], (double)hd[11] / hd[14], (double)hd[15] / hd[14], (double)hd[0] / hd[14],
                    (double)hd[1] / hd[14], (double)hd[2] / hd[14], (double)hd[3] / hd[14], (double)hd[4] / hd[14]);
    }
    if (c->d_mdbg) {
        int64_t hm[8];
        if (hipMemcpy(hm, c->d_mdbg, sizeof(hm), hipMemcpyDeviceToHost) == hipSuccess && hm[7]) {
            const double nwg = (double)hm[7];
            fprintf(stderr, "persist merge: merges=%lld | cycles/merge: loads %.0f rank-heads %.0f barrier %.0f "
                    "global-heads %.0f rank-entries %.0f write %.0f\n", (long long)hm[7], hm[0] / nwg, hm[1] / nwg,
                    hm[2] / nwg, hm[3] / nwg, hm[4] / nwg, hm[5] / nwg);
        }
    }
    if (!cnt) return;
    const double us = 0.01 / (double)cnt;  // 100 MHz ticks -> us, mean
    fprintf(stderr,
            "persist trace: %lld batches, period %.2f us | to-score %.2f score %.2f merge %.2f to-commit %.2f "
            "commit %.2f commit-gap %.2f (to loop top %.2f, top to past the wait %.2f) | wg0: poll %.2f apply %.2f "
            "score %.2f (rows %.2f slowest-wave %.2f fold %.2f stores %.2f) | merger poll %.2f\n",
            (long long)cnt, 0.01 * (double)(int64_t)(at(last, 4) - at(first, 4)) / (double)std::max<int64_t>(1, last - first),
            sum[0] * us, sum[1] * us, sum[2] * us, sum[3] * us, sum[4] * us, sum[5] * us, sum[14] * us, sum[15] * us, sum[6] * us, sum[7] * us,
            sum[8] * us, sum[10] * us, sum[11] * us, sum[12] * us, sum[13] * us, sum[9] * us);
    if (nscr)
        fprintf(stderr, "persist screen (WG 0 wave 0): %lld of %lld batches screened | pass 1 %.2f us, bound %.2f us, "
                "pass 2 %.2f us, exact phase %.2f us (%.2f of the workgroup's %d rows needed; pair lists in %lld batches, "
                "%.1f pairs each)\n", (long long)nscr, (long long)cnt,
                0.01 * scr[0] / nscr, 0.01 * scr[1] / nscr, 0.01 * scr[2] / nscr, 0.01 * scr[3] / nscr, scr[4] / nscr,
                c->prog_rows, (long long)npair, npair ? pairs_sum / (double)npair : 0.0);
}

constexpr int kXcds = 8;  // MI355X: 8 XCDs x 32 CUs

// Batched mode as ONE persistent kernel (ksched_pipe.hip): no per-batch launches, no stream events,
// node rows in LDS.  Returns 1 (not taken) when the configuration does not fit it -- the stream pipeline
// was asked for, multi-rank without the device exchange, a sequential commit (batch > 64), chunk lists
// other than 4 / 8, more lists than merge threads, or rows that do not fit in LDS -- and the stream
// pipeline runs instead.
int enqueue_persistent(ksched_ctx *c) {
    if (c->o.pipeline == KSCHED_PIPELINE_STREAM) return 1;
    // single rank, or node-sharded with the device-side exchange (the RCCL / in-process group paths
    // run the stream pipeline)
    if (!c->xchg_run && (c->comm || c->group || c->o.nranks > 1 || c->o.node_offset != 0)) return 1;
    const int K = c->K, KC = c->KC, B = c->B;
    if (B > 64 || (KC != 4 && KC != 8) || (c->o.commit_impl == KSCHED_COMMIT_SEQUENTIAL)) return 1;
    const int64_t n = c->n_local;
    // node-sharded: every rank sizes its grid for the largest shard, so all ranks take the same path
    const int64_t n_geom = c->xchg_run ? std::max<int64_t>(n, (c->n_global + c->o.nranks - 1) / c->o.nranks) : n;
    // one workgroup per CU: the commit + G score workgroups.  At least ~96 rows per workgroup: a smaller
    // grid costs scan time but every list fewer shortens the merge (one rank's share of an 8-GPU c4,
    // 12.5k nodes: G = 128 -> 22.8 us per batch, 240 -> 23.8, 64 -> 24.6; round 2)
    // Ranks of a local group share the device in ONE cooperative launch: each takes an equal share of the
    // CUs (one workgroup per CU: k_pipe's LDS admits one, checked against the occupancy query below), whole
    // XCDs' worth (multiples of 8), one CU per XCD left over as a margin
    const ksched_lgroup *lgp = c->xchg_run ? c->lg.get() : nullptr;
    // (up to 4 ranks whole XCDs each; 5..8 ranks (31 CUs each on MI355X) are not rounded: whole XCDs would leave
    // 24 CUs per rank, too few for a batch of 32's merger workgroups beside the score workgroups)
    int share = c->cus;
    if (lgp) {
        share = (c->cus - kXcds) / lgp->R;
        if (lgp->R <= 4) share = share / kXcds * kXcds;
    }
    const int wgs = std::min(share, c->o.pipe_wgs > 0 ? c->o.pipe_wgs : c->cus);
    // merger workgroups: kPipeMergeSlots pods each, one slot per pod of a batch
    const int M = (B + kPipeMergeSlots - 1) / kPipeMergeSlots;
    const int G = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)wgs - kCommitWGs - M, (int64_t)kPipeMergeThreads,
                                                               (n_geom + 95) / 96}));
    if (wgs < kCommitWGs + 1 + M) return 1;
    const int R = (int)((n_geom + G - 1) / G);
    PipeLaunch L{};
    PersistArgs &a = L.P[0];
    a.rows_per_wg = R;
    a.G = G;
    a.M = M;
    a.B = B;
    L.R = 1;
    L.base[1] = kCommitWGs + G + M;
    PipeInfo info{};
    const bool f53 = c->fast53, lab = c->o.use_labels != 0;
    hipError_t e = launch_pipe(KC, K, c->o.priority, c->o.domain, lab, f53, L, 0, &info, c->stream);
    if (e == hipErrorNotSupported) return 1;
    HIPCHK(c, e);
    if (c->diag.debug)
        fprintf(stderr, "[ksched pipe] G=%d rows/wg=%d LDS %zu+%zu B, %d VGPRs, %zu B scratch, %d WG/CU\n", G, R,
                info.lds, info.static_lds, info.vgprs, info.spill, info.occ);
    if (info.lds + info.static_lds > 160 * 1024) return 1;  // the rows do not fit: the stream pipeline
    if (lgp && (info.occ < 1 || (int64_t)lgp->R * (kCommitWGs + G + M) > (int64_t)(c->cus - kXcds) * info.occ))
        return fail(c, KSCHED_E_INVALID, "local rank group: the ranks' grids do not fit the device together");
    // KSCHED_PLAIN_LAUNCH (profiled runs) has no runtime residency check: the same one made here
    if (!lgp && c->diag.plain_launch && (info.occ < 1 || (int64_t)(kCommitWGs + G + M) > (int64_t)c->cus * info.occ))
        return 1;
    // workspace: part lists [kPipeLag][B][G][KC] with the counts in entry 0's pad (score(b + kPipeLag) reuses
    // batch b's), list ring 4 x (B*K Rec + B fc), XBuf ring
    const size_t part_b = align_up((size_t)kPipeLag * B * G * KC * sizeof(Cand), 256);
    const size_t cnt_b = 0;
    const size_t lists_b = align_up((size_t)B * K * sizeof(Rec) + (size_t)B * sizeof(int64_t), 256);
    const size_t xb = align_up(xbuf_bytes_pipe(B), 256);
    const size_t prog_b = align_up((size_t)(G + B + kCommitWGs) * kProgWords * 8, 256);
    const size_t resc_b = align_up(rescue_bytes(B), 256);
    const size_t inh_b = align_up(inh_bytes(B), 256);
    const size_t need = part_b + cnt_b + 4 * lists_b + 5 * xb + prog_b + resc_b + inh_b;
    if (c->pws_bytes < need) {
        if (c->d_pws) hipFree(c->d_pws);
        c->d_pws = nullptr;
        c->d_prog = nullptr;
        c->pws_bytes = 0;
        HIPCHK(c, hipMalloc(&c->d_pws, need));
        c->pws_bytes = need;
    }
    char *w = static_cast<char *>(c->d_pws);
    a.nodes = c->d_nodes; a.n_local = n;
    a.pods = PodArgs{c->d_rc, c->d_rm, c->d_rp, c->d_sel, c->p};
    a.ctl = reinterpret_cast<Ctl *>(c->d_cursor);
    a.part = reinterpret_cast<Cand *>(w);
    a.lring = w + part_b + cnt_b;
    a.lists_bytes = (int64_t)lists_b;
    a.xring = a.lring + 4 * lists_b;
    a.xbuf_bytes = (int64_t)xb;
    a.prog = reinterpret_cast<uint64_t *>(a.xring + 5 * xb);
    // the rescue of exhausted lists: each rank's merger slots scan its own shard, node-sharded ranks fold their
    // results through the rings (ksched_commit.h rescue_rank_fold)
    a.rescue = c->diag.rescue_max <= 0 ? nullptr : reinterpret_cast<char *>(a.prog) + prog_b;
    a.rescue_max = c->diag.rescue_max;
    a.rescue_rate = c->diag.rescue_rate;
    a.rescue_look = c->diag.rescue_look;
    a.rescue_cap = c->diag.rescue_cap;
    a.rescue_low = c->diag.rescue_low;
    a.touch_screen = c->diag.touch_screen ? 1 : 0;
    if (c->diag.jitter) a.jitter = c->diag.jitter * 2654435761u + (uint32_t)(++c->jitter_calls) * 40503u + 1u;
    a.inh = reinterpret_cast<char *>(a.prog) + prog_b + resc_b;
    c->d_prog = a.prog;
    c->prog_G = G;
    c->prog_rows = R;
    c->prog_B = B;
    a.out = OutArgs{c->d_oidx, c->d_osc, c->d_ofeas};
    fill_xchg_args(c, &a);
    a.err = c->d_err;
    // every wait is bounded: 10 s of the 100 MHz wall clock by default (a profiler that suspends the
    // queues for a while must not turn into a spurious timeout)
    a.timeout_ticks = c->diag.persist_timeout_ms * 100000;
    a.no_screen = c->diag.no_screen ? 1 : 0;
    a.no_pairs = c->diag.no_pairs ? 1 : 0;
    if (c->diag.trace) {
        const int64_t cap = 4 * (c->p / B) + 64;
        if (c->trace_cap < cap) {
            if (c->d_trace) hipFree(c->d_trace);
            c->d_trace = nullptr;
            c->trace_cap = 0;
            HIPCHK(c, hipMalloc(&c->d_trace, (size_t)cap * kTraceCols * 8));
            c->trace_cap = cap;
        }
        HIPCHK(c, hipMemsetAsync(c->d_trace, 0, (size_t)c->trace_cap * kTraceCols * 8, c->stream));
        a.trace = c->d_trace;
        a.trace_cap = c->trace_cap;
    }
    if (const char *wgp = std::getenv("KSCHED_TRACE_WG"); wgp && *wgp) {
        const int64_t elems = (4 * (c->p / B) + 64) * (int64_t)G;
        if (c->trace_wg_elems < elems) {
            if (c->d_trace_wg) hipFree(c->d_trace_wg);
            c->d_trace_wg = nullptr;
            c->trace_wg_elems = 0;
            HIPCHK(c, hipMalloc(&c->d_trace_wg, (size_t)elems * 8));
            c->trace_wg_elems = elems;
        }
        HIPCHK(c, hipMemsetAsync(c->d_trace_wg, 0, (size_t)c->trace_wg_elems * 8, c->stream));
        a.trace_wg = c->d_trace_wg;
        a.trace_cap = c->trace_wg_elems / G;
    }
    if (const char *xd = std::getenv("KSCHED_XCHG_DUMP"); xd && *xd && c->xchg_run) {
        const int64_t cap = 4 * (c->p / B) + 64;
        const int64_t elems = (int64_t)xdbg_commit_off(cap, B, c->o.nranks, c->K) + cap * 16;
        if (c->xdbg_cap < cap) {
            if (c->d_xdbg) hipFree(c->d_xdbg);
            c->d_xdbg = nullptr;
            c->xdbg_cap = 0;
            HIPCHK(c, hipMalloc(&c->d_xdbg, (size_t)elems * 8));
            c->xdbg_cap = cap;
        }
        HIPCHK(c, hipMemsetAsync(c->d_xdbg, 0, (size_t)elems * 8, c->stream));
        a.xdbg = c->d_xdbg;
        a.xdbg_cap = cap;
    }
    if (c->diag.commit_stamps && !c->d_dbg) HIPCHK(c, hipMalloc(&c->d_dbg, 32 * sizeof(int64_t)));
    if (c->d_dbg) {
        HIPCHK(c, hipMemsetAsync(c->d_dbg, 0, 32 * sizeof(int64_t), c->stream));
        a.cdbg = c->d_dbg;
    }
    if (c->diag.merge_stamps && !c->d_mdbg) HIPCHK(c, hipMalloc(&c->d_mdbg, 8 * sizeof(int64_t)));
    if (c->d_mdbg) {
        HIPCHK(c, hipMemsetAsync(c->d_mdbg, 0, 8 * sizeof(int64_t), c->stream));
        a.mdbg = c->d_mdbg;
    }
    hipStream_t sS = c->stream;
    if (c->diag.poison) {  // read-before-write hunting: stale workspace and LDS become 0xff everywhere
        HIPCHK(c, hipMemsetAsync(c->d_pws, 0xff, need, sS));
        a.poison_lds = (int32_t)info.lds;
        a.lds_fill = ~0u; a.lds_fill_role = 7; a.lds_fill_lo = 0; a.lds_fill_hi = (int32_t)info.lds;
    } else if (const char *f = std::getenv("KSCHED_LDS_FILL"); f && *f) {  // LDS only, a chosen pattern and range
        a.poison_lds = (int32_t)info.lds;
        a.lds_fill = (uint32_t)std::strtoul(f, nullptr, 0);
        a.lds_fill_role = env_int("KSCHED_LDS_ROLE", 7);
        a.lds_fill_lo = env_int("KSCHED_LDS_LO", 0);
        a.lds_fill_hi = env_int("KSCHED_LDS_HI", (int)info.lds);
    }
    HIPCHK(c, launch_ctl_init(a.ctl, B, c->p, kPipeLag, sS));
    // the export ring whole: its records carry batch tags (store_xrec), which an earlier call's must never match
    HIPCHK(c, hipMemsetAsync(a.xring, 0, 5 * xb, sS));
    HIPCHK(c, hipMemsetAsync(a.prog, 0, (size_t)(G + B + kCommitWGs) * kProgWords * 8, sS));
    // score -> merge records carry 16-bit batch tags (1 + batch): no record of an earlier call may look current
    HIPCHK(c, hipMemsetAsync(a.part, 0, part_b, sS));
    // timing: the kernel (family 0) is bracketed by events on its stream -- one launch per call, so the
    // events cost nothing per batch and may stay on inside a timed region
    int e0 = -1;
    HIPCHK(c, ev_begin(c, c->o.timing != 0, &e0, sS));
    // cooperative launch: the runtime checks the grid against the occupancy query, so every workgroup is
    // resident at once.  A local group's ranks stage their arguments and the last to arrive launches all
    // of them as one grid on its stream, behind every rank's pre-launch work; the others' streams wait for it.
    if (lgp) {
        ksched_lgroup *g = c->lg.get();
        const int me = c->o.rank;
        HIPCHK(c, hipEventRecord(g->ready[me], sS));
        const bool met = lg_meet(
            g,
            [&] {
                g->L.P[me] = a;
                g->stream[me] = sS;
                if (g->arrived == 0) {
                    g->kc = KC; g->k = K; g->prio = c->o.priority; g->dom = c->o.domain; g->lab = lab; g->f53 = f53;
                    g->launch_err = hipSuccess;
                } else if (g->kc != KC || g->k != K || g->prio != c->o.priority || g->dom != c->o.domain ||
                           g->lab != lab || g->f53 != f53) {
                    g->launch_err = hipErrorInvalidValue;  // the ranks disagree on the kernel
                }
            },
            [&] {
                if (g->launch_err != hipSuccess) return;
                g->L.R = g->R;
                g->L.base[0] = 0;
                for (int r = 0; r < g->R; ++r) g->L.base[r + 1] = g->L.base[r] + kCommitWGs + g->L.P[r].G + g->L.P[r].M;
                hipError_t le = hipSuccess;
                for (int r = 0; r < g->R && le == hipSuccess; ++r)
                    if (r != me) le = hipStreamWaitEvent(sS, g->ready[r], 0);
                if (le == hipSuccess) le = launch_pipe(g->kc, g->k, g->prio, g->dom, g->lab, g->f53, g->L, c->diag.plain_launch ? 2 : 1,
                                                             nullptr, sS);
                if (le == hipSuccess) le = hipEventRecord(g->done, sS);
                g->launch_err = le;
            });
        if (!met) return fail(c, KSCHED_E_DEVICE, "local rank group: a peer never launched");
        if (g->launch_err != hipSuccess)
            return fail(c, KSCHED_E_DEVICE, std::string("local rank group launch: ") + hipGetErrorString(g->launch_err));
        HIPCHK(c, hipStreamWaitEvent(sS, g->done, 0));  // (a no-op on the launching rank's own stream)
        e = hipSuccess;
    } else {
        e = launch_pipe(KC, K, c->o.priority, c->o.domain, lab, f53, L, c->diag.plain_launch ? 2 : 1, nullptr, sS);
    }
    if (e == hipErrorCooperativeLaunchTooLarge && !c->xchg_run) {  // the stream pipeline runs instead
        if (c->diag.debug) fprintf(stderr, "[ksched pipe] cooperative launch too large: stream pipeline\n");
        (void)hipGetLastError();
        c->timed.clear();
        c->ev_used = 0;
        return 1;
    }
    if (e != hipSuccess) return fail(c, KSCHED_E_DEVICE, std::string("launch_pipe: ") + hipGetErrorString(e));
    HIPCHK(c, ev_end(c, c->o.timing != 0, 0, e0, c->p * n, sS));
    HIPCHK(c, hipMemcpyAsync(c->h_cursor, a.ctl, sizeof(Ctl), hipMemcpyDeviceToHost, sS));
    c->persist_stats = true;
    c->persist_B = B;
    c->run_batches = 0;
    return KSCHED_OK;
}

int enqueue_exact(ksched_ctx *c) {
    if (c->o.nranks > 1) return fail(c, KSCHED_E_INVALID, "exact mode is single-GPU; use batched mode across ranks");
    const int64_t n = c->n_local;
    // the whole node set in ONE workgroup's registers (k_exact1): no cross-workgroup exchange per pod
    const bool price = c->o.priority == KSCHED_PRIORITY_BEST_PRICE;
    const int max1 = price ? 16 : 4;
    if (c->o.exact_wgs <= 1 && n > 0 && n <= (int64_t)kExact1Block * max1 && (!price || c->d_perm)) {
        int bs = kExact1Block;
        if (price && c->diag.exact1_bs == 512 && n <= 5120) bs = 512;
        if (price && c->diag.exact1_bs == 256 && n <= 5120) bs = 256;
        int npt = bs == 512 ? 10 : bs == 256 ? 20 : 1;
        while ((int64_t)bs * npt < n) npt = npt < 4 ? npt + 1 : (npt < 6 && price ? npt + 1 : (npt < 8 ? 8 : (npt < 12 ? 12 : 16)));
        HIPCHK(c, hipMemsetAsync(c->d_err, 0, sizeof(int32_t), c->stream));
        ExactArgs a{};
        a.nodes = c->d_nodes; a.n = n; a.G = 1; a.per_wg = (int32_t)n;
        a.pods = PodArgs{c->d_rc, c->d_rm, c->d_rp, c->d_sel, c->p};
        a.out = OutArgs{c->d_oidx, c->d_osc, c->d_ofeas};
        a.err = c->d_err;
        a.perm = price ? c->d_perm : nullptr;
        int e0 = -1;
        HIPCHK(c, ev_begin(c, c->o.timing != 0, &e0, c->stream));
        HIPCHK(c, launch_exact1(npt, bs, c->o.priority, c->o.domain, c->o.use_labels != 0, c->fast53, a, c->stream));
        HIPCHK(c, ev_end(c, c->o.timing != 0, 0, e0, c->p * n, c->stream));
        c->st.pair_evals = c->p * n;
        c->st.batches = 0;
        c->st.truncations = 0;
        c->run_batches = 1;
        return KSCHED_OK;
    }
    int G = c->o.exact_wgs;
    int npt;
    if (G <= 0) {
        // resource scores are ~150 FP64 ops per pair: spread nodes thin; best-price is a compare: pack
        const int per_thread = c->o.priority == KSCHED_PRIORITY_BEST_PRICE ? 8 : 1;
        npt = 1;
        while (npt < 8 && (int64_t)kExactBlock * npt < (n + c->cus - 1) / c->cus) npt *= 2;
        while (npt < per_thread && npt < 8) npt *= 2;
        G = (int)std::max<int64_t>(1, (n + (int64_t)kExactBlock * npt - 1) / ((int64_t)kExactBlock * npt));
    } else {
        npt = 1;
        while (npt < 8 && (int64_t)G * kExactBlock * npt < n) npt *= 2;
    }
    const int64_t per_wg = (n + G - 1) / G;
    if (per_wg > (int64_t)kExactBlock * npt)
        return fail(c, KSCHED_E_INVALID, "exact mode: too many nodes per workgroup (raise exact_wgs)");
    if (G > c->cus) return fail(c, KSCHED_E_INVALID, "exact mode: more workgroups than CUs");
    HIPCHK(c, grow(&c->d_slots, &c->slots_cap, (int64_t)2 * G * 4, sizeof(uint64_t)));
    HIPCHK(c, hipMemsetAsync(c->d_slots, 0, (size_t)2 * G * 4 * sizeof(uint64_t), c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_err, 0, sizeof(int32_t), c->stream));
    ExactArgs a{};
    a.nodes = c->d_nodes; a.n = n; a.G = G; a.per_wg = (int32_t)per_wg;
    a.pods = PodArgs{c->d_rc, c->d_rm, c->d_rp, c->d_sel, c->p};
    a.out = OutArgs{c->d_oidx, c->d_osc, c->d_ofeas};
    a.slots = c->d_slots; a.err = c->d_err;
    a.timeout_ticks = c->diag.exchange_timeout_ms * 100000;  // 100 MHz wall clock
    int e0 = -1;
    HIPCHK(c, ev_begin(c, c->o.timing != 0, &e0, c->stream));
    HIPCHK(c, launch_exact(npt, c->o.priority, c->o.domain, c->o.use_labels != 0, c->fast53, a, kExactBlock,
                           G > 1 && !c->diag.plain_launch, c->stream));
    HIPCHK(c, ev_end(c, c->o.timing != 0, 0, e0, c->p * n, c->stream));
    c->st.pair_evals = c->p * n;
    c->st.batches = 0;
    c->st.truncations = 0;
    c->run_batches = 1;
    return KSCHED_OK;
}

}  // namespace

extern "C" {

int ksched_abi_version(void) { return KSCHED_ABI_VERSION; }

int ksched_default_opts(ksched_opts *o) {
    if (!o) return KSCHED_E_INVALID;
    std::memset(o, 0, sizeof(*o));
    o->struct_size = (int32_t)sizeof(ksched_opts);
    o->mode = KSCHED_MODE_AUTO;
    o->priority = KSCHED_PRIORITY_RESOURCE;
    o->domain = KSCHED_DOMAIN_ALL;
    o->device = -1;
    o->nranks = 1;
    return KSCHED_OK;
}

int ksched_create(const ksched_opts *opts, ksched_ctx **out) {
    if (!opts || !out || opts->struct_size != (int32_t)sizeof(ksched_opts)) return KSCHED_E_INVALID;
    *out = nullptr;
    if (opts->priority < 0 || opts->priority > 1 || opts->domain < 0 || opts->domain > 1 || opts->mode < 0 ||
        opts->mode > 2 || opts->nranks < 1 || opts->rank < 0 || opts->rank >= opts->nranks)
        return KSCHED_E_INVALID;
    if (opts->topk != 0 && opts->topk != 4 && opts->topk != 8 && opts->topk != 16) return KSCHED_E_INVALID;
    ksched_ctx *c = new (std::nothrow) ksched_ctx();
    if (!c) return KSCHED_E_NOMEM;
    c->o = *opts;
    c->K = opts->topk ? opts->topk : 16;
    if (opts->chunk_topk != 0 && opts->chunk_topk != 2 && opts->chunk_topk != 4 && opts->chunk_topk != 8 &&
        opts->chunk_topk != 16) { delete c; return KSCHED_E_INVALID; }
    c->KC = std::min(c->K, opts->chunk_topk ? opts->chunk_topk : 4);
    c->B = opts->batch > 0 ? opts->batch : std::min(128, 8 * c->K);
    if (c->B > 128) { delete c; return KSCHED_E_INVALID; }
    if (opts->commit_impl < 0 || opts->commit_impl > 3) { delete c; return KSCHED_E_INVALID; }
    if (opts->pipeline < 0 || opts->pipeline > 1 || opts->pipe_wgs < 0) { delete c; return KSCHED_E_INVALID; }
    c->diag.trace = env_int("KSCHED_PERSIST_TRACE", 0) != 0;
    c->diag.commit_stamps = env_int("KSCHED_COMMIT_STAMPS", 0) != 0;
    c->diag.merge_stamps = env_int("KSCHED_MERGE_STAMPS", 0) != 0;
    c->diag.debug = env_int("KSCHED_DEBUG", 0) != 0;
    c->diag.no_screen = env_int("KSCHED_NO_SCREEN", 0) != 0;
    c->diag.no_pairs = env_int("KSCHED_NO_PAIRS", 0) != 0;
    c->diag.poison = env_int("KSCHED_POISON", 0) != 0;
    c->diag.plain_launch = env_int("KSCHED_PLAIN_LAUNCH", 0) != 0;
    c->diag.xchg_diag = env_int("KSCHED_XCHG_DIAG", 0);
    c->diag.epoch_base = env_int("KSCHED_XCHG_EPOCH_BASE", 0);
    c->diag.exact1_bs = env_int("KSCHED_EXACT1_BS", 1024);
    c->diag.rescue_max = env_int("KSCHED_RESCUE_MAX", 4);
    c->diag.rescue_rate = env_int("KSCHED_RESCUE_RATE", 4);
    c->diag.rescue_look = env_int("KSCHED_RESCUE_LOOK", 0);
    c->diag.rescue_cap = env_int("KSCHED_RESCUE_CAP", 16);
    c->diag.rescue_low = env_int("KSCHED_RESCUE_LOW", 2);
    c->diag.touch_screen = env_int("KSCHED_NO_TOUCH_SCREEN", 0) == 0;
    c->diag.jitter = (uint32_t)env_int("KSCHED_JITTER", 0);
    c->diag.persist_timeout_ms = env_int("KSCHED_PERSIST_TIMEOUT_MS", 10000);
    c->diag.exchange_timeout_ms = env_int("KSCHED_EXCHANGE_TIMEOUT_MS", 2000);
    // KSCHED_COMMIT_LANE_PER_POD (round 1) is retired: accepted as the speculative commit  // touched table: 2B <= 256 = 4 slots per lane
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) { delete c; return KSCHED_E_DEVICE; }
    if (opts->device >= 0) {
        if (opts->device >= ndev || hipSetDevice(opts->device) != hipSuccess) { delete c; return KSCHED_E_DEVICE; }
        c->dev = opts->device;
    } else {
        hipGetDevice(&c->dev);
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, c->dev) == hipSuccess) c->cus = prop.multiProcessorCount;
    bool ev_ok = true;
    for (int i = 0; i < 4; ++i)
        ev_ok = ev_ok && hipEventCreateWithFlags(&c->ev_lists[i], hipEventDisableTiming) == hipSuccess &&
                hipEventCreateWithFlags(&c->ev_commit[i], hipEventDisableTiming) == hipSuccess &&
                hipEventCreateWithFlags(&c->ev_scored[i], hipEventDisableTiming) == hipSuccess;
    for (int i = 0; i < 3; ++i) ev_ok = ev_ok && hipEventCreateWithFlags(&c->ev_pipe[i], hipEventDisableTiming) == hipSuccess;
    if (!ev_ok || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipMalloc((void **)&c->d_cursor, sizeof(Ctl)) != hipSuccess ||
        hipMalloc((void **)&c->d_err, sizeof(int32_t)) != hipSuccess ||
        hipHostMalloc((void **)&c->h_cursor, sizeof(Ctl)) != hipSuccess) {
        ksched_destroy(c);
        return KSCHED_E_DEVICE;
    }
    if (hipMemsetAsync(c->d_err, 0, sizeof(int32_t), c->stream) != hipSuccess ||  // error word read by every sync
        hipStreamSynchronize(c->stream) != hipSuccess) {
        ksched_destroy(c);
        return KSCHED_E_DEVICE;
    }
    *out = c;
    return KSCHED_OK;
}

int ksched_destroy(ksched_ctx *c) {
    if (!c) return KSCHED_OK;
    hipSetDevice(c->dev);
    if (c->stream) hipStreamSynchronize(c->stream);
    if (c->stream2) hipStreamSynchronize(c->stream2);
    if (c->comm) ncclCommDestroy(c->comm);
    hipFree(c->d_nodes); hipFree(c->d_snap);
    hipFree(c->d_rc); hipFree(c->d_rm); hipFree(c->d_rp); hipFree(c->d_sel);
    hipFree(c->d_oidx); hipFree(c->d_osc); hipFree(c->d_ofeas);
    hipFree(c->d_ws); hipFree(c->d_cursor); hipFree(c->d_dbg); hipFree(c->d_mdbg); hipFree(c->d_slots); hipFree(c->d_perm); hipFree(c->d_err);
    if (c->h_cursor) hipHostFree(c->h_cursor);
    for (hipEvent_t e : c->ev_pool) hipEventDestroy(e);
    if (c->ev0) hipEventDestroy(c->ev0);
    if (c->ev1) hipEventDestroy(c->ev1);
    for (int i = 0; i < 4; ++i) {
        if (c->ev_lists[i]) hipEventDestroy(c->ev_lists[i]);
        if (c->ev_commit[i]) hipEventDestroy(c->ev_commit[i]);
        if (c->ev_scored[i]) hipEventDestroy(c->ev_scored[i]);
    }
    for (int i = 0; i < 3; ++i) if (c->ev_pipe[i]) hipEventDestroy(c->ev_pipe[i]);
    hipFree(c->d_xring); hipFree(c->d_lring);
    hipFree(c->d_xws); hipFree(c->d_xbuf); hipFree(c->d_pws); hipFree(c->d_trace); hipFree(c->d_trace_wg); hipFree(c->d_xdbg); hipFree(c->d_xmin);
    rx_unmap_peers(c);
    c->lg.reset();
    rx_free(c);
    if (c->stream) hipStreamDestroy(c->stream);
    if (c->stream2) hipStreamDestroy(c->stream2);
    delete c;
    return KSCHED_OK;
}

const char *ksched_last_error(const ksched_ctx *c) { return c ? c->err.c_str() : "null context"; }

int ksched_get_unique_id(uint8_t out_id[128]) {
    if (!out_id) return KSCHED_E_INVALID;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return KSCHED_E_DEVICE;
    static_assert(sizeof(ncclUniqueId) == 128, "nccl id size");
    std::memcpy(out_id, &id, 128);
    return KSCHED_OK;
}

int ksched_set_comm(ksched_ctx *c, const uint8_t id[128]) {
    if (!c || !id) return KSCHED_E_INVALID;
    HIPCHK(c, hipSetDevice(c->dev));
    ncclUniqueId uid;
    std::memcpy(&uid, id, 128);
    if (c->comm) { ncclCommDestroy(c->comm); c->comm = nullptr; }
    NCCLCHK(c, ncclCommInitRank(&c->comm, c->o.nranks, uid, c->o.rank));
    return KSCHED_OK;
}

int ksched_group_create(int32_t nranks, int32_t device, ksched_group **out) {
    if (!out || nranks < 1 || nranks > 1024) return KSCHED_E_INVALID;
    *out = nullptr;
    ksched_group *g = new (std::nothrow) ksched_group();
    if (!g) return KSCHED_E_NOMEM;
    g->nranks = nranks;
    g->send.assign((size_t)nranks, nullptr);
    if (device >= 0) {
        if (hipSetDevice(device) != hipSuccess) { delete g; return KSCHED_E_DEVICE; }
        g->dev = device;
    } else if (hipGetDevice(&g->dev) != hipSuccess) {
        delete g;
        return KSCHED_E_DEVICE;
    }
    *out = g;
    return KSCHED_OK;
}

int ksched_group_destroy(ksched_group *g) {
    delete g;
    return KSCHED_OK;
}

int ksched_set_group(ksched_ctx *c, ksched_group *g) {
    if (!c || !g) return KSCHED_E_INVALID;
    if (g->nranks != c->o.nranks) return fail(c, KSCHED_E_INVALID, "set_group: group size != opts.nranks");
    if (c->dev != g->dev) return fail(c, KSCHED_E_INVALID, "set_group: the group's contexts must share its device");
    if (c->comm) return fail(c, KSCHED_E_STATE, "set_group: context already has an RCCL communicator");
    const int64_t bytes = (int64_t)c->B * c->K * (int64_t)sizeof(Rec) + (int64_t)c->B * (int64_t)sizeof(int64_t);
    {
        std::lock_guard<std::mutex> lk(g->mu);
        if (g->block_bytes == 0) g->block_bytes = bytes;
        else if (g->block_bytes != bytes) return fail(c, KSCHED_E_INVALID, "set_group: ranks disagree on batch / topk");
    }
    c->group = g;
    return KSCHED_OK;
}

// The settings every rank of a node-sharded group must share, because every rank replays the same commit and takes
// the same rescue-or-truncate decisions (the rescue policy) or lays out the same messages: carried in the handle
// blob after the IPC handle and the epoch hint, checked by every importer (a rank with other
// KSCHED_RESCUE_* settings would wait for rescue records no peer sends).
constexpr int kPolicyWords = 8;
constexpr size_t kPolicyOff = 72;
static_assert(sizeof(hipIpcMemHandle_t) + 4 <= kPolicyOff && kPolicyOff + 4 * kPolicyWords <= KSCHED_XCHG_HANDLE_BYTES,
              "handle blob layout");
void policy_words(const ksched_ctx *c, uint32_t *w) {
    w[0] = 0x4b534331u;  // "KSC1": a blob of this layout
    w[1] = (uint32_t)c->diag.rescue_max;
    w[2] = (uint32_t)c->diag.rescue_rate;
    w[3] = (uint32_t)c->diag.rescue_cap;
    w[4] = (uint32_t)c->diag.rescue_low;
    w[5] = (uint32_t)c->diag.rescue_look;
    w[6] = (uint32_t)c->B | (uint32_t)c->K << 16;
    w[7] = (uint32_t)c->KC | (uint32_t)c->o.priority << 8 | (uint32_t)c->o.domain << 16 | (uint32_t)(c->o.use_labels != 0) << 24;
}

int ksched_xchg_export(ksched_ctx *c, uint8_t handle[KSCHED_XCHG_HANDLE_BYTES]) {
    if (!c || !handle) return KSCHED_E_INVALID;
    const int R = c->o.nranks;
    if (R < 2 || R > kMaxXchgRanks) return fail(c, KSCHED_E_INVALID, "xchg_export: 2 <= nranks <= 8");
    if (c->B > 64) return fail(c, KSCHED_E_INVALID, "xchg_export: the persistent pipeline needs batch <= 64");
    if (c->group) return fail(c, KSCHED_E_STATE, "xchg_export: context uses an in-process rank group");
    if (c->lg) return fail(c, KSCHED_E_STATE, "xchg_export: context is in a local rank group (xchg_join_local)");
    HIPCHK(c, hipSetDevice(c->dev));
    // a re-export (a second setup_exchange) drops this rank's maps of the old peers before its ring is zeroed
    rx_unmap_peers(c);
    c->xchg_ready = false;
    if (int rc = rx_prepare(c, xchg_ring_bytes(R, c->B, c->K), true); rc != KSCHED_OK) return rc;
    if (!c->d_xmin) HIPCHK(c, hipMalloc((void **)&c->d_xmin, sizeof(int32_t)));
    hipIpcMemHandle_t h;
    HIPCHK(c, hipIpcGetMemHandle(&h, c->d_rx));
    // the blob: the IPC handle, then this process's first unused granule tag (the setup's tags start at the
    // largest hint of all ranks)
    std::memset(handle, 0, KSCHED_XCHG_HANDLE_BYTES);
    std::memcpy(handle, &h, sizeof(h));
    const uint32_t hint = g_epoch_next.load();
    std::memcpy(handle + sizeof(h), &hint, sizeof(hint));
    uint32_t pol[kPolicyWords];
    policy_words(c, pol);
    std::memcpy(handle + kPolicyOff, pol, sizeof(pol));
    return KSCHED_OK;
}

int ksched_xchg_import(ksched_ctx *c, const uint8_t *handles) {
    if (!c || !handles) return KSCHED_E_INVALID;
    if (!c->d_rx) return fail(c, KSCHED_E_STATE, "xchg_import before xchg_export");
    if (c->lg) return fail(c, KSCHED_E_STATE, "xchg_import: context is in a local rank group (xchg_join_local)");
    HIPCHK(c, hipSetDevice(c->dev));
    const int R = c->o.nranks;
    rx_unmap_peers(c);
    c->xchg_ready = false;
    {
        uint32_t mine[kPolicyWords];
        policy_words(c, mine);
        for (int r = 0; r < R; ++r)
            if (std::memcmp(handles + (size_t)r * KSCHED_XCHG_HANDLE_BYTES + kPolicyOff, mine, sizeof(mine)) != 0)
                return fail(c, KSCHED_E_INVALID, "xchg_import: rank " + std::to_string(r) +
                                                     " has other settings (batch, topk, priority, domain, labels or the "
                                                     "KSCHED_RESCUE_* policy): every rank must share them");
    }
    for (int r = 0; r < R; ++r) {
        if (r == c->o.rank) { c->rx_peer[r] = static_cast<char *>(c->d_rx); continue; }
        if (int rc = rx_map_peer(c, r, handles + (size_t)r * KSCHED_XCHG_HANDLE_BYTES); rc != KSCHED_OK) {
            rx_unmap_peers(c);
            return rc;
        }
    }
    // every ring was zeroed by its rank's export of this setup, before its handle left (rx_prepare), AND the tags
    // start at the largest hint of all ranks: beyond any tag any of their processes used, so no granule left in
    // reused memory can match (the same R blobs on every rank: the same epoch on every rank)
    uint32_t e0 = std::max<uint32_t>(1u, (uint32_t)c->diag.epoch_base);
    for (int r = 0; r < R; ++r) {
        uint32_t hint = 0;
        std::memcpy(&hint, handles + (size_t)r * KSCHED_XCHG_HANDLE_BYTES + sizeof(hipIpcMemHandle_t), sizeof(hint));
        e0 = std::max(e0, hint);
    }
    epoch_used_below(e0 + 1);
    c->xchg_ready = true;
    c->xchg_epoch = e0;
    return KSCHED_OK;
}

int ksched_xchg_ready(const ksched_ctx *c) { return c && c->xchg_ready ? 1 : 0; }

int ksched_xchg_join_local(ksched_ctx *const *ctxs, int32_t n) { return ksched_xchg_join_local_ex(ctxs, n, 0); }

int ksched_xchg_join_local_ex(ksched_ctx *const *ctxs, int32_t n, int32_t flags) {
    if (!ctxs || n < 2 || n > kMaxLocalRanks) return KSCHED_E_INVALID;
    if (flags & ~(KSCHED_XCHG_RINGS_UNCACHED | KSCHED_XCHG_RINGS_IPC)) return KSCHED_E_INVALID;
    for (int r = 0; r < n; ++r)
        if (!ctxs[r]) return KSCHED_E_INVALID;
    const bool ipc = (flags & KSCHED_XCHG_RINGS_IPC) != 0;
    const bool uncached = ipc || (flags & KSCHED_XCHG_RINGS_UNCACHED) != 0;
    ksched_ctx *c0 = ctxs[0];
    for (int r = 0; r < n; ++r) {
        ksched_ctx *c = ctxs[r];
        if (c->o.nranks != n || c->o.rank != r)
            return fail(c, KSCHED_E_INVALID, "xchg_join_local: ctxs[r] must be rank r of nranks = n");
        if (c->dev != c0->dev) return fail(c, KSCHED_E_INVALID, "xchg_join_local: the ranks must share one device");
        if (c->B > 64) return fail(c, KSCHED_E_INVALID, "xchg_join_local: the persistent pipeline needs batch <= 64");
        if (c->group) return fail(c, KSCHED_E_STATE, "xchg_join_local: context uses an in-process rank group");
        uint32_t pc[kPolicyWords], p0[kPolicyWords];
        policy_words(c, pc);
        policy_words(c0, p0);
        if (std::memcmp(pc, p0, sizeof(pc)) != 0)
            return fail(c, KSCHED_E_INVALID, "xchg_join_local: the ranks' options or rescue policies differ");
    }
    auto g = std::make_shared<ksched_lgroup>();
    g->R = n;
    g->dev = c0->dev;
    HIPCHK(c0, hipSetDevice(c0->dev));
    for (int r = 0; r < n; ++r) HIPCHK(c0, hipEventCreateWithFlags(&g->ready[r], hipEventDisableTiming));
    HIPCHK(c0, hipEventCreateWithFlags(&g->done, hipEventDisableTiming));
    // every ring through rx_prepare, as xchg_export's: (re)allocated, zeroed at this setup and finished before
    // any rank of the group can see it.  Plain device memory by default (one device, one kernel: the granules
    // are sc1 traffic inside one device's memory, like the score -> merge records); uncached as export's on request
    for (int r = 0; r < n; ++r) {
        ksched_ctx *c = ctxs[r];
        rx_unmap_peers(c);
        c->lg.reset();
        c->xchg_ready = false;
        if (int rc = rx_prepare(c, xchg_ring_bytes(n, c0->B, c0->K), uncached); rc != KSCHED_OK) return rc;
    }
    std::vector<uint8_t> handles;
    if (ipc) {  // the multi-process path's handles: each ring exported, every peer's opened from its handle
        handles.resize((size_t)n * KSCHED_XCHG_HANDLE_BYTES);
        for (int r = 0; r < n; ++r) {
            hipIpcMemHandle_t h;
            HIPCHK(ctxs[r], hipIpcGetMemHandle(&h, ctxs[r]->d_rx));
            std::memcpy(handles.data() + (size_t)r * KSCHED_XCHG_HANDLE_BYTES, &h, sizeof(h));
        }
    }
    for (int r = 0; r < n; ++r) {
        ksched_ctx *c = ctxs[r];
        for (int q = 0; q < n; ++q) {
            if (q == r || !ipc) {
                c->rx_peer[q] = static_cast<char *>(ctxs[q]->d_rx);
            } else if (int rc = rx_map_peer(c, q, handles.data() + (size_t)q * KSCHED_XCHG_HANDLE_BYTES); rc != KSCHED_OK) {
                for (int u = 0; u <= r; ++u) rx_unmap_peers(ctxs[u]);
                return rc;
            }
        }
    }
    // the same epoch rule as xchg_import: the process's first unused tag (one process: one hint)
    const uint32_t e0 = (c0->diag.xchg_diag & 2) ? 1u : std::max<uint32_t>({1u, g_epoch_next.load(), (uint32_t)c0->diag.epoch_base});
    epoch_used_below(e0 + 1);
    for (int r = 0; r < n; ++r) {
        ksched_ctx *c = ctxs[r];
        c->lg = g;
        c->xchg_ready = true;
        c->xchg_epoch = e0;
    }
    return KSCHED_OK;
}

int ksched_xchg_close(ksched_ctx *c) {
    if (!c) return KSCHED_E_INVALID;
    c->xchg_ready = false;
    c->xchg_run = false;
    rx_unmap_peers(c);  // the peers' rings are no longer used (IPC maps closed); the own ring stays allocated
    return KSCHED_OK;
}

int ksched_load_nodes(ksched_ctx *c, int64_t n, const int64_t *ac, const int64_t *am, const int64_t *ap,
                      const uint64_t *labels, const float *price) {
    if (!c) return KSCHED_E_INVALID;
    if (n < 0 || (n > 0 && (!ac || !am || !ap))) return fail(c, KSCHED_E_INVALID, "load_nodes: bad arguments");
    if (c->o.use_labels && n > 0 && !labels) return fail(c, KSCHED_E_INVALID, "load_nodes: use_labels needs labels");
    if (c->o.priority == KSCHED_PRIORITY_BEST_PRICE && n > 0 && !price)
        return fail(c, KSCHED_E_INVALID, "load_nodes: best-price priority needs prices");
    // node indices are int32 on the device and kNoIdx (INT32_MAX) marks "no candidate": every global
    // index this rank produces (node_offset + local) must stay below it
    if (c->o.node_offset < 0 || n > 0x7ffffff0LL || c->o.node_offset + n > 0x7ffffff0LL)
        return fail(c, KSCHED_E_INVALID, "load_nodes: node_offset + n must stay below 2^31 - 16");
    std::vector<NodeRec> h((size_t)std::max<int64_t>(n, 0));
    uint64_t mx = 0;
    for (int64_t i = 0; i < n; ++i) {
        NodeRec &r = h[(size_t)i];
        r.a[0] = ac[i]; r.a[1] = am[i]; r.a[2] = ap[i];
        r.af[0] = r.af[1] = r.af[2] = 0.0;  // derived on the device (k_prep_nodes) with the reciprocals
        r.y[0] = r.y[1] = r.y[2] = 0.0;
        r.labels = labels ? labels[i] : 0;
        r.price = (price && price[i] != 0.f) ? price[i] : 0.f;  // "-0" == "0": canonical +0 (price_key)
        r.ys[0] = r.ys[1] = r.ys[2] = 0.f;
        mx = std::max(mx, std::max(uabs(ac[i]), std::max(uabs(am[i]), uabs(ap[i]))));
        if (price && !std::isfinite(price[i])) return fail(c, KSCHED_E_INVALID, "load_nodes: non-finite price");
    }
    HIPCHK(c, hipSetDevice(c->dev));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, grow(&c->d_nodes, &c->node_cap, n, sizeof(NodeRec)));
    if (c->d_snap) { hipFree(c->d_snap); c->d_snap = nullptr; }
    // in the stream of the kernels that read it (a legacy hipMemcpy from pageable memory may return before its DMA
    // lands, and nothing orders it with this non-blocking stream: k_prep_nodes read the memory's earlier contents --
    // the round-4 exchange failure)
    if (n > 0) HIPCHK(c, hipMemcpyAsync(c->d_nodes, h.data(), (size_t)n * sizeof(NodeRec), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, launch_prep_nodes(c->d_nodes, n, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->max_abs_alloc = mx;
    c->n_local = n;
    c->explain_valid = false;
    c->n_global = c->o.nranks > 1 ? c->o.nodes_global : (c->o.nodes_global > 0 ? c->o.nodes_global : n);
    if (c->n_global < c->o.node_offset + n) return fail(c, KSCHED_E_INVALID, "load_nodes: nodes_global too small");
    c->has_labels = labels != nullptr;
    c->has_price = price != nullptr;
    if (price && n > 0 && n <= (int64_t)kExact1Block * 16) {
        // exact mode on one workgroup (k_exact1): the nodes in the best-price argmax's order -- price ascending,
        // node index ascending on ties (prices are finite, -0 canonical: the order of price_key descending)
        std::vector<int32_t> perm((size_t)n);
        for (int64_t i = 0; i < n; ++i) perm[(size_t)i] = (int32_t)i;
        std::stable_sort(perm.begin(), perm.end(), [&](int32_t x, int32_t y) { return h[(size_t)x].price < h[(size_t)y].price; });
        HIPCHK(c, grow(&c->d_perm, &c->perm_cap, n, sizeof(int32_t)));
        HIPCHK(c, hipMemcpyAsync(c->d_perm, perm.data(), (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    } else if (c->d_perm) {
        hipFree(c->d_perm);
        c->d_perm = nullptr;
        c->perm_cap = 0;
    }
    return KSCHED_OK;
}

int ksched_apply_delta(ksched_ctx *c, int64_t k, const int32_t *idx, const int64_t *dc, const int64_t *dm,
                       const int64_t *dp) {
    if (!c) return KSCHED_E_INVALID;
    if (c->n_local < 0) return fail(c, KSCHED_E_STATE, "apply_delta before load_nodes");
    if (k < 0 || (k > 0 && (!idx || !dc || !dm || !dp))) return fail(c, KSCHED_E_INVALID, "apply_delta: bad arguments");
    if (k == 0) return KSCHED_OK;
    for (int64_t i = 0; i < k; ++i) {
        if (idx[i] < 0 || idx[i] >= c->n_local) return fail(c, KSCHED_E_INVALID, "apply_delta: node index out of range");
        c->max_abs_alloc = sat_add(c->max_abs_alloc, sat_add(uabs(dc[i]), sat_add(uabs(dm[i]), uabs(dp[i]))));
    }
    HIPCHK(c, hipSetDevice(c->dev));
    std::vector<int64_t> d((size_t)(3 * k));
    std::memcpy(d.data(), dc, (size_t)k * 8);
    std::memcpy(d.data() + k, dm, (size_t)k * 8);
    std::memcpy(d.data() + 2 * k, dp, (size_t)k * 8);
    int32_t *d_idx = nullptr;
    int64_t *d_d = nullptr;
    HIPCHK(c, hipMalloc(&d_idx, (size_t)k * 4));
    if (hipMalloc(&d_d, (size_t)k * 24) != hipSuccess) { hipFree(d_idx); return fail(c, KSCHED_E_DEVICE, "apply_delta: alloc"); }
    hipError_t e = hipMemcpyAsync(d_idx, idx, (size_t)k * 4, hipMemcpyHostToDevice, c->stream);  // the kernel's stream
    if (e == hipSuccess) e = hipMemcpyAsync(d_d, d.data(), (size_t)k * 24, hipMemcpyHostToDevice, c->stream);
    c->explain_valid = false;
    if (e == hipSuccess) e = launch_apply_delta(c->d_nodes, c->n_local, k, d_idx, d_d, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    hipFree(d_idx);
    hipFree(d_d);
    if (e != hipSuccess) return fail(c, KSCHED_E_DEVICE, std::string("apply_delta: ") + hipGetErrorString(e));
    return KSCHED_OK;
}

int ksched_explain(ksched_ctx *c, int64_t rc, int64_t rm, int64_t rp, uint64_t sel, int64_t out_counts[KSCHED_NUM_REASONS],
                   uint8_t *out_reason) {
    if (!c) return KSCHED_E_INVALID;
    if (c->n_local < 0) return fail(c, KSCHED_E_STATE, "explain before load_nodes");
    if (!out_counts) return fail(c, KSCHED_E_INVALID, "explain: out_counts is NULL");
    static_assert(KSCHED_NUM_REASONS == kNumReasons, "reason codes");
    HIPCHK(c, hipSetDevice(c->dev));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const int64_t n = c->n_local;
    unsigned long long *d_cnt = nullptr;
    HIPCHK(c, hipMalloc(&d_cnt, KSCHED_NUM_REASONS * sizeof(unsigned long long) + (size_t)(out_reason ? n : 0)));
    uint8_t *d_reason = out_reason ? (uint8_t *)(d_cnt + KSCHED_NUM_REASONS) : nullptr;
    unsigned long long h[KSCHED_NUM_REASONS] = {};
    hipError_t e = hipMemsetAsync(d_cnt, 0, KSCHED_NUM_REASONS * sizeof(unsigned long long), c->stream);
    if (e == hipSuccess)
        e = launch_explain(c->d_nodes, n, rc, rm, rp, sel, c->o.use_labels != 0, d_reason, d_cnt, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(h, d_cnt, sizeof(h), hipMemcpyDeviceToHost);
    if (e == hipSuccess && out_reason && n > 0) e = hipMemcpy(out_reason, d_reason, (size_t)n, hipMemcpyDeviceToHost);
    hipFree(d_cnt);
    if (e != hipSuccess) return fail(c, KSCHED_E_DEVICE, std::string("explain: ") + hipGetErrorString(e));
    for (int k = 0; k < KSCHED_NUM_REASONS; ++k) out_counts[k] = (int64_t)h[k];
    return KSCHED_OK;
}

namespace {
ExplainArgs explain_args(ksched_ctx *c) {
    ExplainArgs a{};
    a.idx = c->d_oidx; a.p = c->p;
    a.rc = c->d_rc; a.rm = c->d_rm; a.rp = c->d_rp; a.sel = c->d_sel;
    a.nodes = c->d_nodes; a.n_local = c->n_local; a.node_lo = c->o.node_offset;
    a.use_labels = c->o.use_labels != 0;
    return a;
}

hipError_t grow_bytes(void **p, size_t *cap, size_t need) {
    if (*p && *cap >= need) return hipSuccess;
    if (*p) hipFree(*p);
    *p = nullptr;
    *cap = 0;
    hipError_t e = hipMalloc(p, std::max<size_t>(need, 256));
    if (e == hipSuccess) *cap = std::max<size_t>(need, 256);
    return e;
}
}  // namespace

int ksched_explain_batch(ksched_ctx *c, int64_t p, int64_t *out_counts, int64_t *out_nofit) {
    if (!c) return KSCHED_E_INVALID;
    if (!out_counts && p > 0) return fail(c, KSCHED_E_INVALID, "explain_batch: out_counts is NULL");
    if (p != c->p) return fail(c, KSCHED_E_INVALID, "explain_batch: p differs from the last schedule call");
    if (!c->explain_valid) return fail(c, KSCHED_E_STATE, "explain_batch: the node state changed since the last schedule call");
    if (p >= 0x7fffffff) return fail(c, KSCHED_E_INVALID, "explain_batch: too many pods");
    HIPCHK(c, hipSetDevice(c->dev));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::memset(out_counts, 0, (size_t)p * KSCHED_NUM_REASONS * sizeof(int64_t));
    if (out_nofit) *out_nofit = 0;
    if (p == 0 || c->n_local == 0) return KSCHED_OK;
    const size_t cnt_bytes = (size_t)p * kNumReasons * sizeof(unsigned long long);
    HIPCHK(c, grow_bytes(&c->d_xbuf, &c->xbuf_bytes, cnt_bytes + (size_t)p * sizeof(int32_t)));
    unsigned long long *d_cnt = static_cast<unsigned long long *>(c->d_xbuf);
    int32_t *d_fpod = reinterpret_cast<int32_t *>(static_cast<char *>(c->d_xbuf) + cnt_bytes);
    HIPCHK(c, hipMemsetAsync(d_cnt, 0, cnt_bytes, c->stream));
    ExplainArgs a = explain_args(c);
    int64_t nf = 0;
    a.fpod_out = d_fpod;
    a.n_nofit = &nf;
    HIPCHK(c, explain_batch(a, &c->d_xws, &c->xws_bytes, d_cnt, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (nf == 0) return KSCHED_OK;
    std::vector<unsigned long long> h((size_t)nf * kNumReasons);
    std::vector<int32_t> fp((size_t)nf);
    HIPCHK(c, hipMemcpy(h.data(), d_cnt, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(fp.data(), d_fpod, fp.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
    for (int64_t f = 0; f < nf; ++f)
        for (int r = 0; r < kNumReasons; ++r)
            out_counts[(size_t)fp[(size_t)f] * kNumReasons + r] = (int64_t)h[(size_t)f * kNumReasons + r];
    if (out_nofit) *out_nofit = nf;
    return KSCHED_OK;
}

int ksched_explain_pod(ksched_ctx *c, int64_t pod, int64_t out_counts[KSCHED_NUM_REASONS], uint8_t *out_reason) {
    if (!c) return KSCHED_E_INVALID;
    if (!out_counts) return fail(c, KSCHED_E_INVALID, "explain_pod: out_counts is NULL");
    if (pod < 0 || pod >= c->p) return fail(c, KSCHED_E_INVALID, "explain_pod: pod out of range");
    if (!c->explain_valid) return fail(c, KSCHED_E_STATE, "explain_pod: the node state changed since the last schedule call");
    HIPCHK(c, hipSetDevice(c->dev));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const int64_t n = c->n_local;
    ExplainArgs a = explain_args(c);
    HIPCHK(c, hipMemcpy(&a.q_rc, c->d_rc + pod, 8, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(&a.q_rm, c->d_rm + pod, 8, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(&a.q_rp, c->d_rp + pod, 8, hipMemcpyDeviceToHost));
    if (c->o.use_labels) HIPCHK(c, hipMemcpy(&a.q_sel, c->d_sel + pod, 8, hipMemcpyDeviceToHost));
    const size_t st_bytes = (size_t)3 * std::max<int64_t>(n, 1) * sizeof(int64_t);
    HIPCHK(c, grow_bytes(&c->d_xbuf, &c->xbuf_bytes, st_bytes + 64 + (size_t)std::max<int64_t>(n, 1)));
    int64_t *d_state = static_cast<int64_t *>(c->d_xbuf);
    unsigned long long *d_cnt = reinterpret_cast<unsigned long long *>(static_cast<char *>(c->d_xbuf) + st_bytes);
    uint8_t *d_reason = reinterpret_cast<uint8_t *>(d_cnt + 8);
    HIPCHK(c, hipMemsetAsync(d_cnt, 0, kNumReasons * sizeof(unsigned long long), c->stream));
    HIPCHK(c, explain_pod_at(a, pod, d_state, out_reason ? d_reason : nullptr, d_cnt, c->stream));
    unsigned long long h[kNumReasons] = {};
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(h, d_cnt, sizeof(h), hipMemcpyDeviceToHost));
    if (out_reason && n > 0) HIPCHK(c, hipMemcpy(out_reason, d_reason, (size_t)n, hipMemcpyDeviceToHost));
    for (int r = 0; r < kNumReasons; ++r) out_counts[r] = (int64_t)h[r];
    return KSCHED_OK;
}

int ksched_read_nodes(ksched_ctx *c, int64_t n, int64_t *ac, int64_t *am, int64_t *ap) {
    if (!c) return KSCHED_E_INVALID;
    if (c->n_local < 0) return fail(c, KSCHED_E_STATE, "read_nodes before load_nodes");
    if (n != c->n_local) return fail(c, KSCHED_E_INVALID, "read_nodes: size mismatch");
    HIPCHK(c, hipSetDevice(c->dev));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::vector<NodeRec> h((size_t)n);
    if (n > 0) HIPCHK(c, hipMemcpy(h.data(), c->d_nodes, (size_t)n * sizeof(NodeRec), hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < n; ++i) {
        if (ac) ac[i] = h[(size_t)i].a[0];
        if (am) am[i] = h[(size_t)i].a[1];
        if (ap) ap[i] = h[(size_t)i].a[2];
    }
    return KSCHED_OK;
}

int ksched_save_state(ksched_ctx *c) {
    if (!c) return KSCHED_E_INVALID;
    if (c->n_local < 0) return fail(c, KSCHED_E_STATE, "save_state before load_nodes");
    HIPCHK(c, hipSetDevice(c->dev));
    if (!c->d_snap) HIPCHK(c, hipMalloc(&c->d_snap, (size_t)std::max<int64_t>(c->n_local, 1) * sizeof(NodeRec)));
    if (c->n_local > 0)
        HIPCHK(c, hipMemcpyAsync(c->d_snap, c->d_nodes, (size_t)c->n_local * sizeof(NodeRec), hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->snap_max_abs_alloc = c->max_abs_alloc;
    return KSCHED_OK;
}

int ksched_restore_state(ksched_ctx *c) {
    if (!c) return KSCHED_E_INVALID;
    if (!c->d_snap) return fail(c, KSCHED_E_STATE, "restore_state without save_state");
    HIPCHK(c, hipSetDevice(c->dev));
    if (c->n_local > 0)
        HIPCHK(c, hipMemcpyAsync(c->d_nodes, c->d_snap, (size_t)c->n_local * sizeof(NodeRec), hipMemcpyDeviceToDevice, c->stream));
    c->max_abs_alloc = c->snap_max_abs_alloc;
    c->explain_valid = false;
    return KSCHED_OK;
}

int ksched_upload_pods(ksched_ctx *c, int64_t p, const int64_t *rc, const int64_t *rm, const int64_t *rp,
                       const uint64_t *sel) {
    if (!c) return KSCHED_E_INVALID;
    if (p < 0 || (p > 0 && (!rc || !rm || !rp))) return fail(c, KSCHED_E_INVALID, "upload_pods: bad arguments");
    if (c->o.use_labels && p > 0 && !sel) return fail(c, KSCHED_E_INVALID, "upload_pods: use_labels needs selectors");
    HIPCHK(c, hipSetDevice(c->dev));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    int64_t cap = c->p_cap;
    if (cap < p) {
        hipFree(c->d_rc); hipFree(c->d_rm); hipFree(c->d_rp); hipFree(c->d_sel);
        hipFree(c->d_oidx); hipFree(c->d_osc); hipFree(c->d_ofeas);
        c->d_rc = c->d_rm = c->d_rp = nullptr; c->d_sel = nullptr;
        c->d_oidx = c->d_ofeas = nullptr; c->d_osc = nullptr;
        c->p_cap = 0;
        const size_t q = (size_t)std::max<int64_t>(p, 1);
        HIPCHK(c, hipMalloc(&c->d_rc, q * 8)); HIPCHK(c, hipMalloc(&c->d_rm, q * 8));
        HIPCHK(c, hipMalloc(&c->d_rp, q * 8)); HIPCHK(c, hipMalloc(&c->d_sel, q * 8));
        HIPCHK(c, hipMalloc(&c->d_oidx, q * 4)); HIPCHK(c, hipMalloc(&c->d_osc, q * 8));
        HIPCHK(c, hipMalloc(&c->d_ofeas, q * 4));
        c->p_cap = p;
    }
    if (p > 0) {
        // in the stream of the kernels that read them, finished before the caller's buffers may change (see
        // ksched_load_nodes)
        HIPCHK(c, hipMemcpyAsync(c->d_rc, rc, (size_t)p * 8, hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->d_rm, rm, (size_t)p * 8, hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->d_rp, rp, (size_t)p * 8, hipMemcpyHostToDevice, c->stream));
        if (sel) HIPCHK(c, hipMemcpyAsync(c->d_sel, sel, (size_t)p * 8, hipMemcpyHostToDevice, c->stream));
        else HIPCHK(c, hipMemsetAsync(c->d_sel, 0, (size_t)p * 8, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    uint64_t sum = 0;
    for (int64_t i = 0; i < p; ++i) sum = sat_add(sum, sat_add(uabs(rc[i]), sat_add(uabs(rm[i]), uabs(rp[i]) + 1)));
    c->sum_abs_req = sum;
    c->p = p;
    c->explain_valid = false;
    return KSCHED_OK;
}

int ksched_selftest_fastdiv(ksched_ctx *c, int64_t n, const double *a, const double *b, double *out_native,
                            double *out_fast) {
    if (!c || n < 0 || (n > 0 && (!a || !b || !out_native || !out_fast))) return KSCHED_E_INVALID;
    if (n == 0) return KSCHED_OK;
    HIPCHK(c, hipSetDevice(c->dev));
    double *d = nullptr;
    HIPCHK(c, hipMalloc(&d, (size_t)n * 32));
    hipError_t e = hipMemcpyAsync(d, a, (size_t)n * 8, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(d + n, b, (size_t)n * 8, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = launch_selftest_div(n, d, d + n, d + 2 * n, d + 3 * n, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(out_native, d + 2 * n, (size_t)n * 8, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(out_fast, d + 3 * n, (size_t)n * 8, hipMemcpyDeviceToHost);
    hipFree(d);
    if (e != hipSuccess) return fail(c, KSCHED_E_DEVICE, std::string("selftest_fastdiv: ") + hipGetErrorString(e));
    return KSCHED_OK;
}

int ksched_run(ksched_ctx *c) {
    if (!c) return KSCHED_E_INVALID;
    if (c->n_local < 0) return fail(c, KSCHED_E_STATE, "run before load_nodes");
    if (c->o.nranks > 1 && !c->comm && !c->group && !c->xchg_ready)
        return fail(c, KSCHED_E_STATE, "run: multi-rank context without ksched_set_comm / ksched_set_group / "
                                       "ksched_xchg_import");
    HIPCHK(c, hipSetDevice(c->dev));
    c->err.clear();
    c->st = ksched_stats{};
    c->timed.clear();
    c->ev_used = 0;
    c->st.pods = c->p;
    int mode = c->o.mode;
    if (mode == KSCHED_MODE_AUTO) mode = c->o.nranks > 1 ? KSCHED_MODE_BATCHED : KSCHED_MODE_EXACT;
    c->xchg_run = c->xchg_ready && mode == KSCHED_MODE_BATCHED && c->p > 0;
    // a multi-rank batched call needs a transport: the device exchange, an RCCL communicator or a rank group
    // (never a rank committing from its own shard alone)
    if (c->o.nranks > 1 && mode == KSCHED_MODE_BATCHED && c->p > 0 && !c->xchg_run && !c->comm && !c->group)
        return fail(c, KSCHED_E_STATE, "run: multi-rank context without an exchange transport");
    if (int rr = decide_fast53(c)) return rr;
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    int r = KSCHED_OK;
    if (c->p > 0) {
        c->persist_stats = false;
        if (mode == KSCHED_MODE_EXACT) {
            r = enqueue_exact(c);
            c->st.pipeline = KSCHED_PIPE_EXACT;
        } else {
            r = enqueue_persistent(c);
            c->st.pipeline = KSCHED_PIPE_PERSISTENT;
            if (r == 1 && c->xchg_run && !c->comm)
                r = fail(c, KSCHED_E_INVALID, "node-sharded exchange: the persistent pipeline does not fit this "
                                              "configuration and no RCCL communicator is set");
            if (r == 1) {  // not eligible: the stream pipeline
                c->xchg_run = false;
                r = enqueue_batched(c);
                c->st.pipeline = c->B > 64 || c->o.commit_impl == KSCHED_COMMIT_SEQUENTIAL ? KSCHED_PIPE_STREAM_SEQ
                                                                                          : KSCHED_PIPE_STREAM;
            }
        }
    }
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    c->running = r == KSCHED_OK;
    // the call's commits move every allocatable by at most the sum of the staged requests: keep the
    // FAST53 bound true of the state the NEXT call starts from
    if (r == KSCHED_OK) c->max_abs_alloc = sat_add(c->max_abs_alloc, c->sum_abs_req);
    c->explain_valid = r == KSCHED_OK;
    return r;
}

// KSCHED_PERSIST_TRACE: per score workgroup the summed scan time and poll-end -> arrival time, slowest first,
// with where it ran and whether a merger workgroup shared its CU (PersistArgs::prog words 2, 3).
static void print_wg_busy(ksched_ctx *c) {
    if (!c->d_prog) return;
    const int G = c->prog_G, B = c->prog_B, n = G + B + kCommitWGs;
    std::vector<uint64_t> w((size_t)kProgWords * n);
    if (hipMemcpy(w.data(), c->d_prog, w.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    auto where = [&](int i) { return (uint32_t)(w[kProgWords * i + 1] >> 32); };
    std::vector<int> order(G);
    for (int g = 0; g < G; ++g) order[g] = g;
    std::sort(order.begin(), order.end(), [&](int a, int b) { return w[kProgWords * a + 3] > w[kProgWords * b + 3]; });
    auto shares = [&](int g) {
        int k = 0;
        for (int m = 0; m < B; ++m) k += where(G + m) == where(g);
        return k;
    };
    double sum_busy = 0, sum_scan = 0, sum_busy_m = 0, sum_busy_nm = 0;
    int nm = 0;
    for (int g = 0; g < G; ++g) {
        sum_busy += (double)w[kProgWords * g + 3];
        sum_scan += (double)w[kProgWords * g + 2];
        if (shares(g)) { sum_busy_m += (double)w[kProgWords * g + 3]; ++nm; } else sum_busy_nm += (double)w[kProgWords * g + 3];
    }
    fprintf(stderr, "persist wg busy (ms, 100 MHz ticks): mean scan %.2f busy %.2f | with a merger on the CU (%d WGs) %.2f, "
                    "without %.2f | slowest:",
            sum_scan / G * 1e-5, sum_busy / G * 1e-5, nm, nm ? sum_busy_m / nm * 1e-5 : 0.0,
            G > nm ? sum_busy_nm / (G - nm) * 1e-5 : 0.0);
    for (int k = 0; k < 8 && k < G; ++k) {
        const int g = order[k];
        fprintf(stderr, " #%d(scan %.2f busy %.2f xcc %u se %u cu %u mergers %d)", g, w[kProgWords * g + 2] * 1e-5,
                w[kProgWords * g + 3] * 1e-5, (where(g) >> 8) & 0xf, (where(g) >> 4) & 0xf, where(g) & 0xf, shares(g));
    }
    fprintf(stderr, " | fastest: #%d(busy %.2f)\n", order[G - 1], w[kProgWords * order[G - 1] + 3] * 1e-5);
}

// After a persistent wait timed out: which workgroups are furthest behind, in which phase, on which XCD/SE/CU,
// and what their last wait saw (PersistArgs::prog).
static std::string progress_summary(ksched_ctx *c) {
    if (!c->d_prog) return "";
    const int n = c->prog_G + c->prog_B + kCommitWGs;
    std::vector<uint64_t> w((size_t)kProgWords * n);
    if (hipMemcpy(w.data(), c->d_prog, w.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return "";
    const Ctl *h = reinterpret_cast<const Ctl *>(c->h_cursor);
    std::string out = "; polls satisfied by the atomic read " + std::to_string(h->polls_rmw);
    auto group = [&](const char *name, int lo, int hi) {
        int64_t bmin = INT64_MAX, bmax = -1;
        for (int i = lo; i < hi; ++i) {
            const int64_t b = (int64_t)(w[kProgWords * i] >> 8);
            bmin = std::min(bmin, b); bmax = std::max(bmax, b);
        }
        char t[160];
        snprintf(t, sizeof t, "; %s batches %lld..%lld", name, (long long)bmin, (long long)bmax);
        out += t;
        int shown = 0;
        for (int i = lo; i < hi && shown < 6; ++i) {
            if ((int64_t)(w[kProgWords * i] >> 8) != bmin || bmin == bmax) continue;
            const uint32_t where = (uint32_t)(w[kProgWords * i + 1] >> 32);
            snprintf(t, sizeof t, " [#%d phase %#x xcc %u se %u cu %u saw %llu polls %llu]", i - lo,
                     (unsigned)(w[kProgWords * i] & 0xff), (where >> 8) & 0xf, (where >> 4) & 0xf, where & 0xf,
                     (unsigned long long)(w[kProgWords * i + 1] & 0xffffffffull),
                     (unsigned long long)w[kProgWords * i + 2]);
            out += t;
            if (i < c->prog_G && w[kProgWords * i + 4]) {
                out += " waves";
                for (int v = 0; v < 8; ++v) {
                    const uint64_t x = w[kProgWords * i + 4 + v];
                    snprintf(t, sizeof t, " %lld:%#x", (long long)(x >> 8), (unsigned)(x & 0xff));
                    out += t;
                }
            }
            ++shown;
        }
    };
    group("score", 0, c->prog_G);
    group("merge", c->prog_G, c->prog_G + c->prog_B);
    group("commit", c->prog_G + c->prog_B, n);
    for (int i = c->prog_G + c->prog_B; i < n; ++i) {
        const uint32_t where = (uint32_t)(w[kProgWords * i + 1] >> 32);
        char t[160];
        snprintf(t, sizeof t, "; commit workgroup %d: batch %lld phase %#x on xcc %u se %u cu %u", i - c->prog_G - c->prog_B,
                 (long long)(w[kProgWords * i] >> 8), (unsigned)(w[kProgWords * i] & 0xff), (where >> 8) & 0xf,
                 (where >> 4) & 0xf, where & 0xf);
        out += t;
    }
    return out;
}

static int sync_impl(ksched_ctx *c);

int ksched_sync(ksched_ctx *c) {
    if (!c) return KSCHED_E_INVALID;
    const int r = sync_impl(c);
    // a failed call left the node state partly committed: no FailedScheduling replay from it (callers
    // restore_state / load_nodes before retrying)
    if (r != KSCHED_OK) c->explain_valid = false;
    return r;
}

static int sync_impl(ksched_ctx *c) {
    HIPCHK(c, hipSetDevice(c->dev));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->running) {
        float ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        c->st.device_ms = ms;
        c->running = false;
        for (const auto &t : c->timed) {
            float km = 0.f;
            HIPCHK(c, hipEventElapsedTime(&km, c->ev_pool[(size_t)t.e0], c->ev_pool[(size_t)t.e1]));
            c->st.kernel_ms[t.fam] += km;
            c->st.kernel_launches[t.fam] += 1;
            c->st.kernel_pairs[t.fam] += t.pairs;
        }
        c->timed.clear();
    }
    if (c->persist_stats && c->d_trace && c->diag.trace) {
        print_persist_trace(c);
        print_wg_busy(c);
    }
    // KSCHED_XCHG_DUMP=<path>: the exchange's message hashes, to <path>.r<rank>.c<call> ([cap][B][R + 1] u64)
    if (c->persist_stats && c->d_xdbg && c->xchg_run) {
        if (const char *xd = std::getenv("KSCHED_XCHG_DUMP"); xd && *xd) {
            const size_t elems = xdbg_commit_off(c->xdbg_cap, c->B, c->o.nranks, c->K) + (size_t)c->xdbg_cap * 16;
            std::vector<uint64_t> t(elems);
            if (hipMemcpy(t.data(), c->d_xdbg, elems * 8, hipMemcpyDeviceToHost) == hipSuccess) {
                const std::string path = std::string(xd) + ".r" + std::to_string(c->o.rank) + ".c" + std::to_string(c->xdbg_calls);
                if (FILE *f = std::fopen(path.c_str(), "wb")) {
                    std::fwrite(t.data(), 8, t.size(), f);
                    std::fclose(f);
                }
            }
        }
        ++c->xdbg_calls;
    }
    // KSCHED_TRACE_WG=<path>: the raw per-workgroup stamps ([batches][G] u64: scan start | arrival << 32)
    if (c->persist_stats && c->d_trace_wg && c->prog_G > 0) {
        if (const char *wgp = std::getenv("KSCHED_TRACE_WG"); wgp && *wgp) {
            std::vector<uint64_t> t((size_t)c->trace_wg_elems);
            if (hipMemcpy(t.data(), c->d_trace_wg, t.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
                if (FILE *f = std::fopen(wgp, "wb")) {
                    const int64_t hdr[2] = {(int64_t)c->prog_G, c->trace_wg_elems / c->prog_G};
                    std::fwrite(hdr, 8, 2, f);
                    std::fwrite(t.data(), 8, t.size(), f);
                    std::fclose(f);
                }
            }
        }
    }
    if (c->persist_stats) {
        const Ctl *h = reinterpret_cast<const Ctl *>(c->h_cursor);
        c->st.batches = h->stats[0];
        c->st.truncations = h->stats[1];
        c->st.placed = h->stats[2];
        c->st.rescues = h->stats[4];
        c->st.pair_evals = (h->stats[0] + h->stats[3]) * c->persist_B * c->n_local;
        c->persist_stats = false;
        if (c->d_prog) {  // the score workgroups' exact / scanned row counts (progress words 4, 5)
            std::vector<uint64_t> w((size_t)kProgWords * c->prog_G);
            HIPCHK(c, hipMemcpy(w.data(), c->d_prog, w.size() * 8, hipMemcpyDeviceToHost));
            for (int g = 0; g < c->prog_G; ++g) {
                c->st.exact_rows += (int64_t)w[(size_t)kProgWords * g + 4];
                c->st.scan_rows += (int64_t)w[(size_t)kProgWords * g + 5];
            }
        }
    }
    int32_t e = 0;
    HIPCHK(c, hipMemcpy(&e, c->d_err, sizeof(e), hipMemcpyDeviceToHost));
    if (c->xchg_run) {
        // every rank counted the same active batches and rescues (batch tags epoch0 + a, rescue tags epoch0 + q):
        // the next call's tags start past this call's, and this process never uses them again
        const Ctl *h = reinterpret_cast<const Ctl *>(c->h_cursor);
        // (a step of a multiple of 2^15 would give the next call's barrier granules the tag of this call's:
        // gran_tag keeps 15 bits -- skip one more)
        const uint32_t step = (uint32_t)h->nact + (uint32_t)h->stats[4] + 2u;
        c->xchg_epoch += step + ((step & 0x7fffu) == 0 ? 1u : 0u);
        epoch_used_below(c->xchg_epoch);
        if (e) c->xchg_ready = false;  // the rings' state is unknown: later calls take the RCCL path
        c->xchg_run = false;
    }
    if (e >= 5 && e <= 11) {
        (void)hipMemsetAsync(c->d_err, 0, sizeof(int32_t), c->stream);
        static const std::string lagw = "a score or merger workgroup's wait for commit(b-" + std::to_string(kPipeLag) + ")";
        static const char *what[] = {"the commit's wait for the merges", lagw.c_str(),
                                     "a merger's wait for the score workgroups", "the score grid's plan (idle)",
                                     "the commit's plan (idle)",
                                     "a merger's wait for a peer rank's candidate lists (node-sharded exchange)",
                                     "the ranks' device barrier (node-sharded exchange)"};
        const Ctl *h = reinterpret_cast<const Ctl *>(c->h_cursor);
        char buf[400];
        snprintf(buf, sizeof buf,
                 "persistent pipeline: %s timed out (committed %llu, arrive %llu/%llu/%llu/%llu, merged "
                 "%llu/%llu/%llu/%llu, cursor %lld, merger-0 batches %lld, rank %d/%d)",
                 what[e - 5], h->committed, h->arrive[0].v, h->arrive[1].v, h->arrive[2].v, h->arrive[3].v, h->merged[0].v,
                 h->merged[1].v, h->merged[2].v, h->merged[3].v, (long long)h->cursor, (long long)h->nact, c->o.rank,
                 c->o.nranks);
        return fail(c, KSCHED_E_DEVICE, std::string(buf) + progress_summary(c));
    }
    if (e == 2 || e == 4) {
        (void)hipMemsetAsync(c->d_err, 0, sizeof(int32_t), c->stream);
        return fail(c, KSCHED_E_DEVICE, e == 2 ? "batched mode: the merge's wait for the score workgroups timed out"
                                               : "batched mode: the score's wait for commit(b-2) timed out");
    }
    if (e == 15) {
        std::vector<uint64_t> w((size_t)(c->prog_G + c->prog_B + kCommitWGs) * kProgWords);
        uint64_t where = 0;
        if (!w.empty() && hipMemcpy(w.data(), c->d_prog, w.size() * 8, hipMemcpyDeviceToHost) == hipSuccess)
            for (int i = c->prog_G + c->prog_B; i < c->prog_G + c->prog_B + 2; ++i) where |= w[(size_t)kProgWords * i + 2];
        (void)hipMemsetAsync(c->d_err, 0, sizeof(int32_t), c->stream);
        char buf[200];
        snprintf(buf, sizeof buf, "persistent pipeline: the commit's LDS canary changed (batch %llu, word %llu, low bits %#llx)",
                 (unsigned long long)(where >> 32), (unsigned long long)((where >> 16) & 0xffff),
                 (unsigned long long)(where & 0xffff));
        return fail(c, KSCHED_E_DEVICE, buf);
    }
    if (e == 14) {
        std::vector<uint64_t> w((size_t)(c->prog_G + c->prog_B + kCommitWGs) * kProgWords);
        uint64_t d = 0, v = 0;
        if (hipMemcpy(w.data(), c->d_prog, w.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
            d = w[(size_t)kProgWords * (c->prog_G + c->prog_B) + 3];
            v = w[(size_t)kProgWords * (c->prog_G + c->prog_B) + 4];
        }
        (void)hipMemsetAsync(c->d_err, 0, sizeof(int32_t), c->stream);
        char buf[240];
        snprintf(buf, sizeof buf, "persistent pipeline: the commit produced a node index outside every node (%#llx; batch %llu, "
                 "pod lane %llu, path %llu; a device protocol error, results discarded)", (unsigned long long)v,
                 (unsigned long long)(d >> 40), (unsigned long long)((d >> 32) & 0xff), (unsigned long long)(d & 0xffffffffu));
        return fail(c, KSCHED_E_DEVICE, buf);
    }
    if (e == 12 || e == 14) {
        (void)hipMemsetAsync(c->d_err, 0, sizeof(int32_t), c->stream);
        return fail(c, KSCHED_E_DEVICE, e == 12 ? "persistent pipeline: the commit's wait for a rescue timed out"
                                                : "persistent pipeline: the commit produced a node index outside every "
                                                  "node (a device protocol error; results discarded)");
    }
    if (e) return fail(c, KSCHED_E_DEVICE, "exact mode: cross-workgroup exchange timed out (workgroups not co-resident?)");
    return KSCHED_OK;
}

int ksched_download_results(ksched_ctx *c, int64_t p, int32_t *oi, double *os, int32_t *of) {
    if (!c) return KSCHED_E_INVALID;
    if (p != c->p) return fail(c, KSCHED_E_INVALID, "download_results: size mismatch");
    HIPCHK(c, hipSetDevice(c->dev));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (p == 0) return KSCHED_OK;
    if (oi) HIPCHK(c, hipMemcpy(oi, c->d_oidx, (size_t)p * 4, hipMemcpyDeviceToHost));
    if (os) HIPCHK(c, hipMemcpy(os, c->d_osc, (size_t)p * 8, hipMemcpyDeviceToHost));
    if (of) HIPCHK(c, hipMemcpy(of, c->d_ofeas, (size_t)p * 4, hipMemcpyDeviceToHost));
    if (oi && c->st.placed == 0) {
        int64_t placed = 0;
        for (int64_t i = 0; i < p; ++i) placed += oi[i] >= 0;
        c->st.placed = placed;
    }
    return KSCHED_OK;
}

int ksched_get_stats(const ksched_ctx *c, ksched_stats *out) {
    if (!c || !out) return KSCHED_E_INVALID;
    *out = c->st;
    return KSCHED_OK;
}

int ksched_set_timeout(ksched_ctx *c, int32_t persist_ms) {
    if (!c || persist_ms < 0) return KSCHED_E_INVALID;
    c->diag.persist_timeout_ms = persist_ms;
    return KSCHED_OK;
}

int ksched_set_timing(ksched_ctx *c, int32_t timing, int32_t every) {
    if (!c || every < 0) return KSCHED_E_INVALID;
    c->o.timing = timing ? 1 : 0;
    if (every > 0) c->o.timing_every = every;
    return KSCHED_OK;
}

int ksched_schedule(ksched_ctx *c, int64_t p, const int64_t *rc, const int64_t *rm, const int64_t *rp,
                    const uint64_t *sel, int32_t *oi, double *os, int32_t *of) {
    int r = ksched_upload_pods(c, p, rc, rm, rp, sel);
    if (r != KSCHED_OK) return r;
    if ((r = ksched_run(c)) != KSCHED_OK) { ksched_sync(c); return r; }
    if ((r = ksched_sync(c)) != KSCHED_OK) return r;
    return ksched_download_results(c, p, oi, os, of);
}

}  // extern "C"
