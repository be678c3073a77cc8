/*
 * ksched.h -- C ABI of the MI355X-native scheduling core (libksched.so).
 *
 * Drop-in boundary for the hot path of yinwoods/k8s-scheduler (paths relative to the reference):
 *   func predicate(pod *Pod) ([]*Node, error)              anchor/predicate.go:107-176
 *   func priorities(pod *Pod, nodes []*Node) (*Node, error) anchor/priorities.go:25-63
 *   the per-pod commit that the next pod observes           anchor/schedule.go:68-89, 185-197
 *                                                           (used += request, anchor/predicate.go:83-105)
 * The Go caller keeps getNodes/getPods (anchor/tools.go:53-108) and bind/postEvent
 * (anchor/schedule.go:200-261) unchanged; see INTEGRATION.md for the cgo shim.
 *
 * Plain C types only.  Caller-owned arrays are read (or written) during the call only and never
 * retained, so Go slices of scalars may be passed directly under the cgo pointer rules.
 * Every function returns an int status (KSCHED_OK == 0), never throws across the ABI and never
 * exits the process.  A context is not reentrant: callers serialise calls on one context exactly as
 * the reference serialises schedulePod under processorLock (anchor/schedule.go:29,55,186).
 */
#ifndef KSCHED_H
#define KSCHED_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KSCHED_ABI_VERSION 6

/* status codes */
#define KSCHED_OK 0
#define KSCHED_E_INVALID (-1)   /* bad argument / shape / option */
#define KSCHED_E_DEVICE (-2)    /* HIP or RCCL failure, or a device-side timeout */
#define KSCHED_E_PARSE (-3)     /* the reference's errFatal parse paths (anchor/predicate.go:15,31,39,49) */
#define KSCHED_E_STATE (-4)     /* call out of order (e.g. schedule before load_nodes) */
#define KSCHED_E_NOMEM (-5)
#define KSCHED_E_UNKNOWN_NODE (-6) /* a bound pod names a node not in the node list (reference: nil deref panic, anchor/predicate.go:94-99) */

/* per-pod outcome in out_idx[] */
#define KSCHED_NO_FIT (-1)            /* predicate found no node: reference returns "failed to fit" (anchor/schedule.go:74-76) */
#define KSCHED_NO_POSITIVE_SCORE (-2) /* no node scored > 0: reference binds a nil node and panics (anchor/priorities.go:55-62, anchor/schedule.go:208); documented divergence */

/* options */
#define KSCHED_MODE_EXACT 0     /* pod-by-pod: one full node scan + grid-wide arg-best per pod (persistent kernel) */
#define KSCHED_MODE_BATCHED 1   /* speculative top-K for a batch of pods + ordered commit with exact re-score */
#define KSCHED_MODE_AUTO 2

#define KSCHED_PRIORITY_RESOURCE 0    /* (balanced + least-requested) / 2, anchor/priorities.go:45-50 */
#define KSCHED_PRIORITY_BEST_PRICE 1  /* lowest node price among feasible nodes (README.md:37-64; build-defined) */

/* ordered-commit implementations (batched mode; all produce the sequential result) */
#define KSCHED_COMMIT_SEQUENTIAL 1    /* one wave re-scores the touched set per pod (batch <= 128) */
#define KSCHED_COMMIT_LANE_PER_POD 2  /* retired (round 1 variant): treated as KSCHED_COMMIT_SPECULATIVE */
#define KSCHED_COMMIT_SPECULATIVE 3   /* guess first touches, check all pods in parallel, resolve the first miss (batch <= 64) */

/* batched-mode pipelines (all produce the same results) */
#define KSCHED_PIPELINE_AUTO 0    /* the persistent kernel where the configuration fits it, else the stream pipeline */
#define KSCHED_PIPELINE_STREAM 1  /* always the stream pipeline (per-batch score / merge / commit launches) */

#define KSCHED_DOMAIN_ALL 0       /* argmax over ALL nodes, feasible or not (the reference, anchor/priorities.go:45) */
#define KSCHED_DOMAIN_FEASIBLE 1  /* argmax over feasible nodes only (build extension) */

typedef struct ksched_opts {
    int32_t struct_size; /* = sizeof(ksched_opts) */
    int32_t mode;        /* KSCHED_MODE_* */
    int32_t priority;    /* KSCHED_PRIORITY_* */
    int32_t domain;      /* KSCHED_DOMAIN_* (best-price always ranges over feasible nodes) */
    int32_t use_labels;  /* 1: feasible &= (node_labels & pod_selector) == pod_selector (build extension) */
    int32_t batch;       /* batched mode: pods per speculative batch (0 = auto) */
    int32_t topk;        /* batched mode: candidates kept per pod, one of 4, 8, 16 (0 = auto) */
    int32_t device;      /* HIP device ordinal (-1 = current) */
    /* node sharding across ranks (multi-GPU); single GPU: rank 0, nranks 1 */
    int32_t rank;
    int32_t nranks;
    int64_t node_offset;  /* global index of this rank's first node */
    int64_t nodes_global; /* total nodes across ranks (0 = local count when nranks == 1) */
    int32_t exact_wgs;    /* exact mode: workgroups (0 = auto) */
    int32_t timing;       /* 1: time kernel families with HIP events on the engine stream (sampled) */
    int32_t timing_every; /* batched mode: time one batch in every N (0 = 16) */
    int32_t chunk_topk;   /* batched mode: candidates kept per node chunk before the merge, 2/4/8/16 (0 = auto);
                             capped at topk.  The merge keeps the exact prefix. */
    int32_t commit_impl;  /* batched mode: KSCHED_COMMIT_* (0 = auto: speculative when batch <= 64) */
    int32_t pipeline;     /* batched mode: KSCHED_PIPELINE_AUTO (0) or KSCHED_PIPELINE_STREAM (ABI 4) */
    int32_t pipe_wgs;     /* persistent pipeline: at most this many workgroups, one per CU (0 = every CU).
                             The launch is always cooperative (the runtime admits the grid only if every
                             workgroup is resident at once); ranks that share ONE device are joined by
                             ksched_xchg_join_local and split its CUs in one such launch. (ABI 4) */
    int32_t reserved[1];
} ksched_opts;

typedef struct ksched_ctx ksched_ctx;

typedef struct ksched_stats {
    int64_t pods;          /* pods resolved by the last schedule call */
    int64_t placed;        /* pods bound to a node */
    int64_t batches;       /* speculative batches launched (batched mode) */
    int64_t truncations;   /* batches cut short by a candidate-list overflow */
    int64_t pair_evals;    /* pod-node pairs evaluated by the score kernels */
    double device_ms;      /* device time of the last schedule call (HIP events) */
    double kernel_ms[4];   /* timed device ms per kernel family: [0] score (or the exact kernel),
                              [1] merge, [2] commit, [3] collective (all-gather + rank merge) */
    int64_t kernel_launches[4]; /* number of timed batches (launch groups) behind kernel_ms */
    int64_t kernel_pairs[4];    /* pod-node pairs evaluated by the timed family-0 launches */
    int64_t pipeline;           /* which device pipeline ran the last call: KSCHED_PIPE_* (ABI 2) */
    int64_t rescues;            /* persistent pipeline (ABI 5): exhausted candidate lists resolved by a full scan
                                   of the untouched nodes instead of truncating their batch */
    int64_t exact_rows;         /* persistent pipeline: node rows scored exactly (f64) by the score workgroups,
                                   summed over batches -- the screened scan's survivors plus unscreened batches */
    int64_t scan_rows;          /* ... and node rows scanned (each row once per active batch) */
} ksched_stats;

enum {
    KSCHED_PIPE_NONE = 0,       /* no pods */
    KSCHED_PIPE_EXACT = 1,      /* the exact persistent kernel, one pod at a time */
    KSCHED_PIPE_STREAM = 2,     /* batched: score / merge / speculative commit kernels per batch, stream-linked */
    KSCHED_PIPE_STREAM_SEQ = 3, /* batched with the sequential one-pod-at-a-time commit kernel */
    KSCHED_PIPE_PERSISTENT = 4  /* batched: ONE persistent kernel (commit workgroup + score/merge workgroups) */
};

/* ---- lifecycle ---- */
int ksched_abi_version(void);
int ksched_default_opts(ksched_opts *opts);
int ksched_create(const ksched_opts *opts, ksched_ctx **out);
int ksched_destroy(ksched_ctx *ctx);
const char *ksched_last_error(const ksched_ctx *ctx); /* never NULL; "" when no error */

/* Multi-GPU: rank 0 creates a 128-byte RCCL unique id; every rank passes it to ksched_set_comm
 * before the first schedule call (opts.nranks > 1). */
int ksched_get_unique_id(uint8_t out_id[128]);
int ksched_set_comm(ksched_ctx *ctx, const uint8_t id[128]);

/* In-process rank group: the same node-sharded batched path with R contexts of ONE process on ONE
 * device (one host thread per context), the per-batch all-gather done by host-coordinated device
 * copies instead of RCCL (RCCL admits one rank per device).  It runs the multi-rank code on a single
 * GPU (a test vehicle, one host round trip per batch); contexts set opts.rank / nranks / node_offset /
 * nodes_global as for ksched_set_comm, call ksched_set_group instead of it, and must run the same
 * schedule calls concurrently. */
/* Device-side candidate exchange for the node-sharded batched path (one process per GPU, 2..8 ranks,
 * batch <= 64): instead of one RCCL all-gather per batch launched from the host, the persistent
 * pipeline's merger workgroups write each pod's candidate list straight into every rank's receive
 * ring over xGMI (tagged 8-byte granules in uncached device memory) and rank-merge the R lists they
 * receive -- no launch, no host round trip, no collective per batch.  Setup, on every rank:
 *   ksched_xchg_export(ctx, h)          allocates (or reuses) this rank's ring and zeroes it (a device kernel
 *                                       of system-scope stores, the granules' own path) at EVERY export;
 *                                       h = its IPC handle and the first granule tag this process has never
 *                                       used (128 bytes)
 *   (all-gather the R blobs in rank order, e.g. torch.distributed)
 *   ksched_xchg_import(ctx, handles)    maps every rank's ring (R * 128 bytes, own entry ignored); the tags
 *                                       of the setup start at the largest of the R hints, so no tag repeats
 *                                       in any process's memory
 * Batched runs then take the exchange path on every rank (an RCCL communicator is optional: it is
 * the fallback when a device timeout disables the exchange; ksched_xchg_ready reports the state).
 * Replaces the same all-gather as ksched_set_comm; the call sequence is unchanged. */
#define KSCHED_XCHG_HANDLE_BYTES 128
int ksched_xchg_export(ksched_ctx *ctx, uint8_t handle[KSCHED_XCHG_HANDLE_BYTES]);
int ksched_xchg_import(ksched_ctx *ctx, const uint8_t *handles);
int ksched_xchg_ready(const ksched_ctx *ctx);
/* Turns the exchange off on this rank (later batched calls take the RCCL path).  Every rank calls it when
 * any rank failed to import (ABI 4): the ranks must agree on the transport. */
int ksched_xchg_close(ksched_ctx *ctx);
/* Ranks as threads of ONE process on ONE device (ABI 5): joins ctxs[0..n-1] (rank r at ctxs[r], each created
 * with nranks = n, 2 <= n <= 8, batch <= 64 and the same options) into the device exchange.  Their persistent
 * pipelines then run as ONE cooperative launch -- rank r's workgroups a contiguous block range, the ranks sharing
 * the CUs equally -- so every rank's grid is resident at once by construction; separate launches (of separate
 * processes) sharing a device guarantee no such thing.  The contexts' threads call
 * ksched_run concurrently, as with ksched_set_group; destroy all of them together.  Every rank's grid must fit
 * its share of the CUs: at 8 ranks on one MI355X (31 CUs each) that needs batch <= 32.
 * ksched_xchg_join_local_ex (ABI 6) takes flags: KSCHED_XCHG_RINGS_UNCACHED allocates the rings exactly as
 * ksched_xchg_export does (hipDeviceMallocUncached, zeroed at every setup, tags from the process's next unused
 * one); KSCHED_XCHG_RINGS_IPC
 * (implies UNCACHED) also maps every peer's ring through its IPC handle, as ksched_xchg_import does -- the
 * multi-process transport's allocation, zeroing, handles and epoch rule on one device (it fails where the
 * runtime does not open a handle of the same process). */
int ksched_xchg_join_local(ksched_ctx *const *ctxs, int32_t n);
#define KSCHED_XCHG_RINGS_UNCACHED 1
#define KSCHED_XCHG_RINGS_IPC 2
int ksched_xchg_join_local_ex(ksched_ctx *const *ctxs, int32_t n, int32_t flags);

typedef struct ksched_group ksched_group;
int ksched_group_create(int32_t nranks, int32_t device, ksched_group **out);
int ksched_group_destroy(ksched_group *g); /* after every context using it is destroyed */
int ksched_set_group(ksched_ctx *ctx, ksched_group *g);

/* ---- node state (allocatable = capacity - used, anchor/predicate.go:56-67) ---- */
/* Loads this rank's n nodes (node order = nodeList.Items order).  labels / price may be NULL
 * unless the options need them.  Prices must be finite. */
int ksched_load_nodes(ksched_ctx *ctx, int64_t n, const int64_t *alloc_cpu, const int64_t *alloc_mem,
                      const int64_t *alloc_pods, const uint64_t *labels, const float *price);
/* alloc[node_idx[i]] += (d_cpu[i], d_mem[i], d_pods[i]) for binds / deletions made by others,
 * or to undo a bind that failed (anchor/schedule.go:200-237).  node_idx is local to this rank. */
int ksched_apply_delta(ksched_ctx *ctx, int64_t k, const int32_t *node_idx, const int64_t *d_cpu,
                       const int64_t *d_mem, const int64_t *d_pods);
/* FailedScheduling diagnostics (anchor/predicate.go:127-157): evaluates the predicate of ONE pod
 * against the current (local) node state and reports, per node, the first failing check in the
 * reference's order -- the "fit failure on node (%s): Insufficient CPU|Memory|Pod" lines of the
 * FailedScheduling event -- then the build-defined label check.  out_counts[KSCHED_REASON_*] counts
 * nodes per outcome (out_counts[KSCHED_REASON_FIT] == the pod's feasible count); out_reason (n_local
 * bytes, may be NULL) receives each node's code.  Multi-rank: counts cover this rank's shard. */
#define KSCHED_REASON_FIT 0
#define KSCHED_REASON_CPU 1     /* "Insufficient CPU"    anchor/predicate.go:134-138 */
#define KSCHED_REASON_MEMORY 2  /* "Insufficient Memory" anchor/predicate.go:139-143 */
#define KSCHED_REASON_POD 3     /* "Insufficient Pod"    anchor/predicate.go:144-148 */
#define KSCHED_REASON_LABELS 4  /* label selector not satisfied (build extension) */
#define KSCHED_NUM_REASONS 5
int ksched_explain(ksched_ctx *ctx, int64_t req_cpu, int64_t req_mem, int64_t req_pods, uint64_t selector,
                   int64_t out_counts[KSCHED_NUM_REASONS], uint8_t *out_reason);
/* The same diagnostics for EVERY pod of the last schedule call (ksched_schedule / ksched_run) that
 * ended KSCHED_NO_FIT, each against the node state it saw at its turn -- the state after the
 * placements of all pods before it (anchor/schedule.go:185-197 re-reads the cluster per pod) -- with
 * no host replay: out_counts[i * KSCHED_NUM_REASONS + r] for pod i (rows of the other pods are
 * zero); *out_nofit (may be NULL) = their number.  Valid only while the last call's placements are
 * the last change to the node state (KSCHED_E_STATE after load_nodes / apply_delta / restore_state /
 * upload_pods).  Multi-rank: counts cover this rank's shard (sum them over ranks). */
int ksched_explain_batch(ksched_ctx *ctx, int64_t p, int64_t *out_counts, int64_t *out_nofit);
/* Per-node reasons of pod `pod` of the last schedule call at its turn: the "fit failure on node"
 * lines of its FailedScheduling event (out_reason: n_local bytes, may be NULL). */
int ksched_explain_pod(ksched_ctx *ctx, int64_t pod, int64_t out_counts[KSCHED_NUM_REASONS], uint8_t *out_reason);
/* Copies the current (local) node state back to the host. */
int ksched_read_nodes(ksched_ctx *ctx, int64_t n, int64_t *alloc_cpu, int64_t *alloc_mem, int64_t *alloc_pods);
/* Device-side snapshot / restore of the node state (bench: identical start state every step). */
int ksched_save_state(ksched_ctx *ctx);
int ksched_restore_state(ksched_ctx *ctx);

/* ---- scheduling: schedulePods over p pending pods, in order (anchor/schedule.go:185-197) ----
 * req_pods is the container count (anchor/predicate.go:78); each placed pod commits
 * alloc[node] -= (req_cpu, req_mem, 1) (anchor/predicate.go:102).  Outputs per pod:
 *   out_idx      node index (global across ranks) | KSCHED_NO_FIT | KSCHED_NO_POSITIVE_SCORE
 *   out_score    winning score (resource priority) or price (best-price); 0 when not placed
 *   out_feasible number of nodes passing predicate() for that pod at its turn
 * Any output pointer may be NULL. */
int ksched_schedule(ksched_ctx *ctx, int64_t p, const int64_t *req_cpu, const int64_t *req_mem,
                    const int64_t *req_pods, const uint64_t *selector,
                    int32_t *out_idx, double *out_score, int32_t *out_feasible);

/* Same, in two halves, with the pods staged in HBM: upload once, run many times (bench). */
int ksched_upload_pods(ksched_ctx *ctx, int64_t p, const int64_t *req_cpu, const int64_t *req_mem,
                       const int64_t *req_pods, const uint64_t *selector);
int ksched_run(ksched_ctx *ctx);                 /* schedules the staged pods; results stay on device */
/* Bound of every device-side wait of the persistent pipeline, in ms (default 10000, or the
 * KSCHED_PERSIST_TIMEOUT_MS environment variable at create).  A wait that exceeds it ends the call with
 * KSCHED_E_DEVICE naming the wait and where every workgroup stood (ABI 4). */
int ksched_set_timeout(ksched_ctx *ctx, int32_t persist_ms);
int ksched_sync(ksched_ctx *ctx);                /* waits for the run; fills stats */
int ksched_download_results(ksched_ctx *ctx, int64_t p, int32_t *out_idx, double *out_score, int32_t *out_feasible);
int ksched_get_stats(const ksched_ctx *ctx, ksched_stats *out);
/* Turns the sampled per-kernel HIP-event timing (opts.timing / opts.timing_every) on or off for the
 * following calls (every = 0: keep the current sampling period). */
int ksched_set_timing(ksched_ctx *ctx, int32_t timing, int32_t every);

/* Diagnostics: out_native[i] = a[i] / b[i] (hipcc's f64 division) and out_fast[i] = the engine's
 * hoisted-reciprocal division of the same operands, both computed on the device (bit-exactness
 * check of the division used by every score kernel). */
int ksched_selftest_fastdiv(ksched_ctx *ctx, int64_t n, const double *a, const double *b, double *out_native,
                            double *out_fast);

/* ---- host packer: Go-exact Kubernetes quantity parsing ----
 * s == NULL means the key is absent from the ResourceList.  KSCHED_E_PARSE on the reference's
 * errFatal paths; otherwise KSCHED_OK with the reference's value (0 for unparseable floats and for
 * memory suffixes other than Ki/Mi). */
int ksched_parse_cpu(const char *s, int64_t *out);    /* parseCpu, anchor/predicate.go:10-24 */
int ksched_parse_memory(const char *s, int64_t *out); /* parseMemory, anchor/predicate.go:26-44 */
int ksched_parse_pods(const char *s, int64_t *out);   /* parsePod, anchor/predicate.go:46-53 */
int ksched_parse_price(const char *s, float *out);    /* node price annotation (README.md:43-48), f32 */

/* Packs a Kubernetes-shaped cluster into the SoA inputs above.
 *   nodes: n names + capacity strings (cpu/mem/pods, NULL = absent)       anchor/predicate.go:56-67
 *   bound pods: nb pods with node name, container range [cont_off[i], cont_off[i+1]) into the
 *     container request arrays (cpu/mem strings, NULL = absent)          anchor/predicate.go:83-105
 * Writes alloc_* (n).  KSCHED_E_UNKNOWN_NODE if a bound pod names an unknown node. */
int ksched_pack_nodes(int64_t n, const char *const *names, const char *const *cap_cpu,
                      const char *const *cap_mem, const char *const *cap_pods,
                      int64_t nb, const char *const *bound_node, const int64_t *cont_off,
                      const char *const *cont_cpu, const char *const *cont_mem,
                      int64_t *alloc_cpu, int64_t *alloc_mem, int64_t *alloc_pods);
/* requestedResource (anchor/predicate.go:69-81) for p pending pods (container ranges as above). */
int ksched_pack_pods(int64_t p, const int64_t *cont_off, const char *const *cont_cpu,
                     const char *const *cont_mem, int64_t *req_cpu, int64_t *req_mem, int64_t *req_pods);

#ifdef __cplusplus
}
#endif
#endif /* KSCHED_H */
