// ksched_kernels.h -- HIP kernels of the scheduling core (gfx950 / CDNA4).
//
// Exact mode  : k_exact        persistent, node-per-lane, node state in registers, one grid-wide
//                              arg-best per pod through tagged 8-byte granules (no host round trip).
// Batched mode: k_score_topk   pod-per-lane fused predicate + score + per-lane top-K over a node
//                              chunk (node rows are wave-uniform -> scalar loads);
//               k_merge        sorted-list merge, one wave per (pod, <=64 lists), DPP/shuffle arg-best;
//               k_commit       one workgroup replays the batch in pod order: re-scores the nodes
//                              already committed in the batch, takes the first untouched candidate,
//                              commits, stops at the first candidate-list overflow.
// See DESIGN.md for the correctness argument of the batched commit.
#pragma once

#include "ksched_device.h"

namespace ksched {

struct alignas(8) Touched {
    int32_t idx;
    int32_t pad;
    int64_t s0[3];   // state at the batch snapshot
    int64_t cur[3];  // current state
    uint64_t labels;
    float price;
    int32_t pad2;
};
static_assert(sizeof(Touched) == 72, "Touched layout");

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
};

struct ScoreArgs {
    const NodeRec *nodes;
    int64_t n_local;
    int64_t node_offset;
    int32_t S;         // nodes per chunk (one wave per chunk and 64 pods)
    int32_t n_chunks;
    PodArgs pods;
    const int64_t *cursor;
    int32_t B;
    Cand *part;        // [B][n_chunks][K]
    int64_t *part_cnt; // [B][n_chunks]
};

struct MergeArgs {
    const void *in;         // Cand [B][C_in][K]  or, INPUT_REC, C_in rank blocks of rank_stride bytes,
                            // each {Rec [B][K]; int64 fc[B]} (the RCCL all-gather layout)
    const int64_t *in_cnt;  // [B][C_in] (Cand input only)
    int64_t rank_stride;    // bytes per rank block (INPUT_REC)
    int32_t C_in;
    int32_t C_out;          // ceil(C_in / 64)
    Cand *out;              // [B][C_out][K] (non-final)
    int64_t *out_cnt;       // [B][C_out]
    Rec *out_rec;           // [B][K]  (final)
    int64_t *out_fc;        // [B]
    const NodeRec *nodes;   // final + !INPUT_REC: gather node snapshot state
    int64_t node_offset;
    const int64_t *cursor;
    int64_t P;
    int32_t B;
};

struct CommitArgs {
    const Rec *lists;       // [B][K]
    const int64_t *fc0;     // [B]
    PodArgs pods;
    int64_t *cursor;
    int32_t B;
    NodeRec *nodes;         // local shard
    int64_t node_lo;        // global index of the first local node
    int64_t n_local;
    int64_t n_global;       // bitmap bits
    int32_t bitmap_words;
    OutArgs out;
    int64_t *stats;         // [0] batches [1] truncations [2] placed
};

// host-side launchers (ksched_kernels.hip)
hipError_t launch_exact(int npt, int prio, int dom, bool lab, const ExactArgs &a, int block, bool cooperative,
                        hipStream_t s);
hipError_t launch_score_topk(int K, int prio, int dom, bool lab, const ScoreArgs &a, int pod_groups, hipStream_t s);
hipError_t launch_merge(int K, bool input_rec, bool final_stage, const MergeArgs &a, hipStream_t s);
hipError_t launch_commit(int K, int prio, int dom, bool lab, const CommitArgs &a, size_t lds_bytes, bool single_wave,
                         hipStream_t s);
constexpr size_t kPodStageBytes = 40;  // LDS per batch pod staged by the single-wave commit
hipError_t launch_apply_delta(NodeRec *nodes, int64_t n, int64_t k, const int32_t *idx, const int64_t *d,
                              hipStream_t s);

constexpr int kExactBlock = 256;
constexpr int kCommitBlock = 256;

}  // namespace ksched
