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
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ksched.h"
#include "ksched_kernels.h"

using namespace ksched;

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
    NodeRec *d_nodes = nullptr, *d_snap = nullptr;
    int64_t node_cap = 0;
    // pods
    int64_t p = 0, p_cap = 0;
    int64_t *d_rc = nullptr, *d_rm = nullptr, *d_rp = nullptr;
    uint64_t *d_sel = nullptr;
    int32_t *d_oidx = nullptr, *d_ofeas = nullptr;
    double *d_osc = nullptr;
    // batched workspace
    int K = 16, B = 128;
    int64_t ws_bytes = 0;
    void *d_ws = nullptr;
    int64_t *d_cursor = nullptr;  // [0] cursor, [1..3] stats
    int64_t *h_cursor = nullptr;  // pinned
    // exact workspace
    uint64_t *d_slots = nullptr;
    int32_t *d_err = nullptr;
    int64_t slots_cap = 0;
    // multi-GPU
    ncclComm_t comm = nullptr;
    // timing
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool running = false;
    std::vector<hipEvent_t> ev_pool;  // sampled per-family event pairs (opts.timing)
    struct Timed { int fam; int e0, e1; int64_t pairs; };
    std::vector<Timed> timed;
    size_t ev_used = 0;
    ksched_stats st{};
    int64_t run_batches = 0;
};

namespace {

int fail(ksched_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    return code;
}

#define HIPCHK(c, expr)                                                                        \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail((c), KSCHED_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
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

hipError_t ev_begin(ksched_ctx *c, bool on, int *e0) {
    if (!on) return hipSuccess;
    hipError_t r = ev_take(c, e0);
    if (r != hipSuccess) return r;
    return hipEventRecord(c->ev_pool[(size_t)*e0], c->stream);
}

hipError_t ev_end(ksched_ctx *c, bool on, int fam, int e0, int64_t pairs) {
    if (!on) return hipSuccess;
    int e1;
    hipError_t r = ev_take(c, &e1);
    if (r != hipSuccess) return r;
    r = hipEventRecord(c->ev_pool[(size_t)e1], c->stream);
    if (r == hipSuccess) c->timed.push_back({fam, e0, e1, pairs});
    return r;
}

// Batched-mode geometry for one schedule call.
struct BatchPlan {
    int K, B, pod_groups;
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
    pl.B = c->B;
    pl.pod_groups = (pl.B + 63) / 64;
    const int64_t n = std::max<int64_t>(c->n_local, 1);
    // enough waves to cover the chip (>= 8 waves per CU) while keeping >= 16 nodes per wave
    const int target_waves = env_int("KSCHED_TARGET_WAVES", c->cus * 8);
    int64_t chunks = std::max<int64_t>(1, target_waves / pl.pod_groups);
    const int min_s = env_int("KSCHED_MIN_CHUNK", 16);
    chunks = std::min<int64_t>(chunks, (n + min_s - 1) / min_s);
    chunks = std::min<int64_t>(chunks, 4096);
    pl.S = (int)((n + chunks - 1) / chunks);
    pl.n_chunks = (int)((n + pl.S - 1) / pl.S);
    pl.C[0] = pl.n_chunks;
    pl.stages = 1;
    while (pl.C[pl.stages - 1] > 64) {
        pl.C[pl.stages] = (pl.C[pl.stages - 1] + 63) / 64;
        pl.stages++;
    }
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off = align_up(off + bytes, 256); return o; };
    pl.off_part = take((size_t)pl.B * pl.n_chunks * pl.K * sizeof(Cand));
    pl.off_pcnt = take((size_t)pl.B * pl.n_chunks * sizeof(int64_t));
    const int c1 = pl.stages > 1 ? pl.C[1] : 1;
    pl.off_m1 = take((size_t)pl.B * c1 * pl.K * sizeof(Cand) * 2);  // ping-pong for stage >= 1
    pl.off_m1cnt = take((size_t)pl.B * c1 * sizeof(int64_t) * 2);
    pl.send_bytes = (size_t)pl.B * pl.K * sizeof(Rec) + (size_t)pl.B * sizeof(int64_t);
    pl.off_send = take(pl.send_bytes);  // local lists + fc (also the single-GPU final lists)
    const int R = std::max(1, c->o.nranks);
    pl.off_recv = take(pl.send_bytes * R);
    pl.off_glists = take((size_t)pl.B * pl.K * sizeof(Rec));
    pl.off_gfc = take((size_t)pl.B * sizeof(int64_t));
    pl.off_lists = pl.off_send;
    pl.off_fc = pl.off_send + (size_t)pl.B * pl.K * sizeof(Rec);
    pl.total = off;
    return pl;
}

int64_t commit_lds_bytes(const ksched_ctx *c, int B, int *words) {
    const int64_t w = (c->n_global + 31) / 32;
    *words = (int)align_up((size_t)w, 4);
    return (int64_t)*words * 4 + (int64_t)B * (int64_t)(sizeof(Touched) + kPodStageBytes);
}

int enqueue_batched(ksched_ctx *c) {
    const BatchPlan pl = plan_batch(c);
    if (c->ws_bytes < (int64_t)pl.total) {
        if (c->d_ws) hipFree(c->d_ws);
        c->d_ws = nullptr;
        c->ws_bytes = 0;
        HIPCHK(c, hipMalloc(&c->d_ws, pl.total));
        c->ws_bytes = (int64_t)pl.total;
    }
    int words = 0;
    const int64_t lds = commit_lds_bytes(c, pl.B, &words);
    if (lds > 160 * 1024 - 4096)
        return fail(c, KSCHED_E_INVALID, "batched mode: node bitmap + touched table exceed LDS (nodes_global too large or batch too big)");
    char *ws = static_cast<char *>(c->d_ws);
    const int prio = c->o.priority, dom = c->o.domain;
    const bool lab = c->o.use_labels != 0;
    const int R = std::max(1, c->o.nranks);
    PodArgs pods{c->d_rc, c->d_rm, c->d_rp, c->d_sel, c->p};

    HIPCHK(c, hipMemsetAsync(c->d_cursor, 0, 4 * sizeof(int64_t), c->stream));
    int64_t resolved = 0, batches = 0;
    double avg_progress = std::max(1.0, pl.K * 2.0);
    const int poll = env_int("KSCHED_POLL_BATCHES", 0);
    const bool single_wave = env_int("KSCHED_COMMIT_WAVES", 1) == 1;
    while (resolved < c->p) {
        int64_t m = (int64_t)std::ceil((double)(c->p - resolved) / avg_progress);
        m = std::max<int64_t>(1, std::min<int64_t>(m, poll > 0 ? poll : 256));
        for (int64_t it = 0; it < m; ++it) {
            const bool tm = c->o.timing && (batches % (c->o.timing_every > 0 ? c->o.timing_every : 16) == 0);
            int e0 = -1;
            ScoreArgs sa{};
            sa.nodes = c->d_nodes; sa.n_local = c->n_local; sa.node_offset = c->o.node_offset;
            sa.S = pl.S; sa.n_chunks = pl.n_chunks; sa.pods = pods; sa.cursor = c->d_cursor; sa.B = pl.B;
            sa.part = reinterpret_cast<Cand *>(ws + pl.off_part);
            sa.part_cnt = reinterpret_cast<int64_t *>(ws + pl.off_pcnt);
            // (an empty shard runs one empty chunk: the kernel writes empty lists and zero counts)
            HIPCHK(c, ev_begin(c, tm, &e0));
            HIPCHK(c, launch_score_topk(pl.K, prio, dom, lab, sa, pl.pod_groups, c->stream));
            HIPCHK(c, ev_end(c, tm, 0, e0, (int64_t)pl.B * c->n_local));
            HIPCHK(c, ev_begin(c, tm, &e0));
            // merge stages
            const void *in = sa.part;
            const int64_t *in_cnt = sa.part_cnt;
            for (int s = 0; s < pl.stages; ++s) {
                MergeArgs ma{};
                ma.in = in; ma.in_cnt = in_cnt; ma.C_in = pl.C[s];
                ma.C_out = (pl.C[s] + 63) / 64;
                ma.cursor = c->d_cursor; ma.P = c->p; ma.B = pl.B;
                ma.nodes = c->d_nodes; ma.node_offset = c->o.node_offset;
                const bool fin = (s == pl.stages - 1);
                if (fin) {
                    ma.out_rec = reinterpret_cast<Rec *>(ws + pl.off_lists);
                    ma.out_fc = reinterpret_cast<int64_t *>(ws + pl.off_fc);
                } else {
                    const int pp = s & 1;
                    const int c1 = pl.C[1];
                    ma.out = reinterpret_cast<Cand *>(ws + pl.off_m1) + (size_t)pp * pl.B * c1 * pl.K;
                    ma.out_cnt = reinterpret_cast<int64_t *>(ws + pl.off_m1cnt) + (size_t)pp * pl.B * c1;
                }
                HIPCHK(c, launch_merge(pl.K, false, fin, ma, c->stream));
                in = ma.out; in_cnt = ma.out_cnt;
            }
            HIPCHK(c, ev_end(c, tm, 1, e0, 0));
            const Rec *lists = reinterpret_cast<const Rec *>(ws + pl.off_lists);
            const int64_t *fc0 = reinterpret_cast<const int64_t *>(ws + pl.off_fc);
            if (R > 1) {
                HIPCHK(c, ev_begin(c, tm, &e0));
                NCCLCHK(c, ncclAllGather(ws + pl.off_send, ws + pl.off_recv, pl.send_bytes, ncclUint8, c->comm, c->stream));
                MergeArgs ma{};
                ma.in = ws + pl.off_recv; ma.rank_stride = (int64_t)pl.send_bytes; ma.C_in = R; ma.C_out = 1;
                ma.cursor = c->d_cursor; ma.P = c->p; ma.B = pl.B;
                ma.out_rec = reinterpret_cast<Rec *>(ws + pl.off_glists);
                ma.out_fc = reinterpret_cast<int64_t *>(ws + pl.off_gfc);
                HIPCHK(c, launch_merge(pl.K, true, true, ma, c->stream));
                lists = ma.out_rec;
                fc0 = ma.out_fc;
                HIPCHK(c, ev_end(c, tm, 3, e0, 0));
            }
            CommitArgs ca{};
            ca.lists = lists; ca.fc0 = fc0; ca.pods = pods; ca.cursor = c->d_cursor; ca.B = pl.B;
            ca.nodes = c->d_nodes; ca.node_lo = c->o.node_offset; ca.n_local = c->n_local;
            ca.n_global = c->n_global; ca.bitmap_words = words;
            ca.out = OutArgs{c->d_oidx, c->d_osc, c->d_ofeas};
            ca.stats = c->d_cursor + 1;
            HIPCHK(c, ev_begin(c, tm, &e0));
            HIPCHK(c, launch_commit(pl.K, prio, dom, lab, ca, (size_t)lds, single_wave, c->stream));
            HIPCHK(c, ev_end(c, tm, 2, e0, 0));
            ++batches;
        }
        HIPCHK(c, hipMemcpyAsync(c->h_cursor, c->d_cursor, 4 * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        const int64_t now = c->h_cursor[0];
        if (now <= resolved) return fail(c, KSCHED_E_DEVICE, "batched mode made no progress");
        resolved = now;
        if (c->h_cursor[1] > 0) avg_progress = std::max(1.0, (double)resolved / (double)c->h_cursor[1]);
    }
    c->st.batches = c->h_cursor[1];
    c->st.truncations = c->h_cursor[2];
    c->st.placed = c->h_cursor[3];
    c->st.pair_evals = c->h_cursor[1] * (int64_t)pl.B * c->n_local;
    c->run_batches = batches;
    return KSCHED_OK;
}

int enqueue_exact(ksched_ctx *c) {
    if (c->o.nranks > 1) return fail(c, KSCHED_E_INVALID, "exact mode is single-GPU; use batched mode across ranks");
    const int64_t n = c->n_local;
    int G = c->o.exact_wgs > 0 ? c->o.exact_wgs : env_int("KSCHED_EXACT_WGS", 0);
    int npt;
    if (G <= 0) {
        // resource scores are ~150 FP64 ops per pair: spread nodes thin; best-price is a compare: pack
        const int per_thread = c->o.priority == KSCHED_PRIORITY_BEST_PRICE ? 8 : 1;
        npt = 1;
        while (npt < 16 && (int64_t)kExactBlock * npt < (n + c->cus - 1) / c->cus) npt *= 2;
        while (npt < per_thread && npt < 16) npt *= 2;
        G = (int)std::max<int64_t>(1, (n + (int64_t)kExactBlock * npt - 1) / ((int64_t)kExactBlock * npt));
    } else {
        npt = 1;
        while (npt < 16 && (int64_t)G * kExactBlock * npt < n) npt *= 2;
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
    a.timeout_ticks = (int64_t)env_int("KSCHED_EXCHANGE_TIMEOUT_MS", 2000) * 100000;  // 100 MHz wall clock
    int e0 = -1;
    HIPCHK(c, ev_begin(c, c->o.timing != 0, &e0));
    HIPCHK(c, launch_exact(npt, c->o.priority, c->o.domain, c->o.use_labels != 0, a, kExactBlock, G > 1, c->stream));
    HIPCHK(c, ev_end(c, c->o.timing != 0, 0, e0, c->p * n));
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
    c->B = opts->batch > 0 ? opts->batch : 8 * c->K;
    if (c->B > 4096) { delete c; return KSCHED_E_INVALID; }
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
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipMalloc((void **)&c->d_cursor, 8 * sizeof(int64_t)) != hipSuccess ||
        hipMalloc((void **)&c->d_err, sizeof(int32_t)) != hipSuccess ||
        hipHostMalloc((void **)&c->h_cursor, 8 * sizeof(int64_t)) != hipSuccess) {
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
    if (c->comm) ncclCommDestroy(c->comm);
    hipFree(c->d_nodes); hipFree(c->d_snap);
    hipFree(c->d_rc); hipFree(c->d_rm); hipFree(c->d_rp); hipFree(c->d_sel);
    hipFree(c->d_oidx); hipFree(c->d_osc); hipFree(c->d_ofeas);
    hipFree(c->d_ws); hipFree(c->d_cursor); hipFree(c->d_slots); hipFree(c->d_err);
    if (c->h_cursor) hipHostFree(c->h_cursor);
    for (hipEvent_t e : c->ev_pool) hipEventDestroy(e);
    if (c->ev0) hipEventDestroy(c->ev0);
    if (c->ev1) hipEventDestroy(c->ev1);
    if (c->stream) hipStreamDestroy(c->stream);
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
    if (c->o.nranks <= 1) return KSCHED_OK;
    HIPCHK(c, hipSetDevice(c->dev));
    ncclUniqueId uid;
    std::memcpy(&uid, id, 128);
    if (c->comm) { ncclCommDestroy(c->comm); c->comm = nullptr; }
    NCCLCHK(c, ncclCommInitRank(&c->comm, c->o.nranks, uid, c->o.rank));
    return KSCHED_OK;
}

int ksched_load_nodes(ksched_ctx *c, int64_t n, const int64_t *ac, const int64_t *am, const int64_t *ap,
                      const uint64_t *labels, const float *price) {
    if (!c) return KSCHED_E_INVALID;
    if (n < 0 || (n > 0 && (!ac || !am || !ap))) return fail(c, KSCHED_E_INVALID, "load_nodes: bad arguments");
    if (c->o.use_labels && n > 0 && !labels) return fail(c, KSCHED_E_INVALID, "load_nodes: use_labels needs labels");
    if (c->o.priority == KSCHED_PRIORITY_BEST_PRICE && n > 0 && !price)
        return fail(c, KSCHED_E_INVALID, "load_nodes: best-price priority needs prices");
    if (n > 0x7ffffff0LL) return fail(c, KSCHED_E_INVALID, "load_nodes: too many nodes");
    std::vector<NodeRec> h((size_t)std::max<int64_t>(n, 0));
    for (int64_t i = 0; i < n; ++i) {
        NodeRec &r = h[(size_t)i];
        r.a[0] = ac[i]; r.a[1] = am[i]; r.a[2] = ap[i];
        r.af[0] = (double)ac[i]; r.af[1] = (double)am[i]; r.af[2] = (double)ap[i];
        r.labels = labels ? labels[i] : 0;
        r.price = price ? price[i] : 0.f;
        r.pad = 0;
        if (price && !std::isfinite(price[i])) return fail(c, KSCHED_E_INVALID, "load_nodes: non-finite price");
    }
    HIPCHK(c, hipSetDevice(c->dev));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, grow(&c->d_nodes, &c->node_cap, n, sizeof(NodeRec)));
    if (c->d_snap) { hipFree(c->d_snap); c->d_snap = nullptr; }
    if (n > 0) HIPCHK(c, hipMemcpy(c->d_nodes, h.data(), (size_t)n * sizeof(NodeRec), hipMemcpyHostToDevice));
    c->n_local = n;
    c->n_global = c->o.nranks > 1 ? c->o.nodes_global : (c->o.nodes_global > 0 ? c->o.nodes_global : n);
    if (c->n_global < c->o.node_offset + n) return fail(c, KSCHED_E_INVALID, "load_nodes: nodes_global too small");
    c->has_labels = labels != nullptr;
    c->has_price = price != nullptr;
    return KSCHED_OK;
}

int ksched_apply_delta(ksched_ctx *c, int64_t k, const int32_t *idx, const int64_t *dc, const int64_t *dm,
                       const int64_t *dp) {
    if (!c) return KSCHED_E_INVALID;
    if (c->n_local < 0) return fail(c, KSCHED_E_STATE, "apply_delta before load_nodes");
    if (k < 0 || (k > 0 && (!idx || !dc || !dm || !dp))) return fail(c, KSCHED_E_INVALID, "apply_delta: bad arguments");
    if (k == 0) return KSCHED_OK;
    for (int64_t i = 0; i < k; ++i)
        if (idx[i] < 0 || idx[i] >= c->n_local) return fail(c, KSCHED_E_INVALID, "apply_delta: node index out of range");
    HIPCHK(c, hipSetDevice(c->dev));
    std::vector<int64_t> d((size_t)(3 * k));
    std::memcpy(d.data(), dc, (size_t)k * 8);
    std::memcpy(d.data() + k, dm, (size_t)k * 8);
    std::memcpy(d.data() + 2 * k, dp, (size_t)k * 8);
    int32_t *d_idx = nullptr;
    int64_t *d_d = nullptr;
    HIPCHK(c, hipMalloc(&d_idx, (size_t)k * 4));
    if (hipMalloc(&d_d, (size_t)k * 24) != hipSuccess) { hipFree(d_idx); return fail(c, KSCHED_E_DEVICE, "apply_delta: alloc"); }
    hipError_t e = hipMemcpy(d_idx, idx, (size_t)k * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_d, d.data(), (size_t)k * 24, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch_apply_delta(c->d_nodes, c->n_local, k, d_idx, d_d, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    hipFree(d_idx);
    hipFree(d_d);
    if (e != hipSuccess) return fail(c, KSCHED_E_DEVICE, std::string("apply_delta: ") + hipGetErrorString(e));
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
    return KSCHED_OK;
}

int ksched_restore_state(ksched_ctx *c) {
    if (!c) return KSCHED_E_INVALID;
    if (!c->d_snap) return fail(c, KSCHED_E_STATE, "restore_state without save_state");
    HIPCHK(c, hipSetDevice(c->dev));
    if (c->n_local > 0)
        HIPCHK(c, hipMemcpyAsync(c->d_nodes, c->d_snap, (size_t)c->n_local * sizeof(NodeRec), hipMemcpyDeviceToDevice, c->stream));
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
        HIPCHK(c, hipMemcpy(c->d_rc, rc, (size_t)p * 8, hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->d_rm, rm, (size_t)p * 8, hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->d_rp, rp, (size_t)p * 8, hipMemcpyHostToDevice));
        if (sel) HIPCHK(c, hipMemcpy(c->d_sel, sel, (size_t)p * 8, hipMemcpyHostToDevice));
        else HIPCHK(c, hipMemset(c->d_sel, 0, (size_t)p * 8));
    }
    c->p = p;
    return KSCHED_OK;
}

int ksched_run(ksched_ctx *c) {
    if (!c) return KSCHED_E_INVALID;
    if (c->n_local < 0) return fail(c, KSCHED_E_STATE, "run before load_nodes");
    if (c->o.nranks > 1 && !c->comm) return fail(c, KSCHED_E_STATE, "run: multi-rank context without ksched_set_comm");
    HIPCHK(c, hipSetDevice(c->dev));
    c->err.clear();
    c->st = ksched_stats{};
    c->timed.clear();
    c->ev_used = 0;
    c->st.pods = c->p;
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    int r = KSCHED_OK;
    if (c->p > 0) {
        int mode = c->o.mode;
        if (mode == KSCHED_MODE_AUTO) mode = c->o.nranks > 1 ? KSCHED_MODE_BATCHED : KSCHED_MODE_EXACT;
        r = mode == KSCHED_MODE_EXACT ? enqueue_exact(c) : enqueue_batched(c);
    }
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    c->running = r == KSCHED_OK;
    return r;
}

int ksched_sync(ksched_ctx *c) {
    if (!c) return KSCHED_E_INVALID;
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
    int32_t e = 0;
    HIPCHK(c, hipMemcpy(&e, c->d_err, sizeof(e), hipMemcpyDeviceToHost));
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

int ksched_schedule(ksched_ctx *c, int64_t p, const int64_t *rc, const int64_t *rm, const int64_t *rp,
                    const uint64_t *sel, int32_t *oi, double *os, int32_t *of) {
    int r = ksched_upload_pods(c, p, rc, rm, rp, sel);
    if (r != KSCHED_OK) return r;
    if ((r = ksched_run(c)) != KSCHED_OK) { ksched_sync(c); return r; }
    if ((r = ksched_sync(c)) != KSCHED_OK) return r;
    return ksched_download_results(c, p, oi, os, of);
}

}  // extern "C"
