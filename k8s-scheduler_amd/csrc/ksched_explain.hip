// ksched_explain.hip -- FailedScheduling diagnostics for a whole schedule call, on the device.
//
// The reference posts, for a pod that fits nowhere, one line per node with the FIRST failing check
// in the order CPU, Memory, Pod (anchor/predicate.go:127-173), evaluated against the cluster state
// that pod saw at its turn -- i.e. after every placement of the pods before it.  After a batched call
// only the final state is on the device; for a NO_FIT pod i the state it saw is
//     state_j(i) = final_j + sum of the requests of the pods after i that were placed on node j.
// So its reason histogram is
//     hist(i) = H_final(i) + sum over placements k > i of [onehot(r_i(before_k)) - onehot(r_i(after_k))]
// where before_k / after_k are node n_k's state just before / after placement k (the sum over the
// placements on one node telescopes to onehot(r_i(state at i)) - onehot(r_i(final))).  Three steps:
//   1. placements in pod order (stable compaction) and, per placement, the node's state before it:
//      a stable sort by node, then within each node's run a backward walk from the final state;
//   2. k_hist_final: every NO_FIT pod against every node's final state (lane = pod, rows scalar-loaded);
//   3. k_hist_correct: every NO_FIT pod against the placements after it (lane = pod, placements
//      wave-uniform), only the reason changes counted.
// Work: F x N + F x (placements after each NO_FIT pod) integer compares, no host replay.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "ksched_kernels.h"

namespace ksched {

namespace {

// first failing check (anchor/predicate.go:134-148), then the build-defined label check; 0 = fits
__device__ __forceinline__ int reason_of(int64_t rc, int64_t rm, int64_t rp, uint64_t sel, int64_t ac, int64_t am,
                                         int64_t ap, uint64_t lab, bool use_labels) {
    return ac < rc ? 1 : am < rm ? 2 : ap < rp ? 3 : (use_labels && (lab & sel) != sel) ? 4 : 0;
}

// placed-and-owned flag per pod, local node key per pod (sort key; non-placed pods sort last)
__global__ void k_commit_flags(const int32_t *idx, int64_t p, int64_t node_lo, int64_t n_local, uint8_t *placed,
                               uint8_t *nofit) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p) return;
    const int64_t j = (int64_t)idx[i] - node_lo;
    placed[i] = idx[i] >= 0 && j >= 0 && j < n_local;
    nofit[i] = idx[i] == -1;
}

__global__ void k_commit_keys(const int32_t *cpod, const int32_t *idx, int64_t nc, int64_t node_lo, int32_t *key,
                              int32_t *pos) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nc) return;
    key[c] = (int32_t)((int64_t)idx[cpod[c]] - node_lo);
    pos[c] = (int32_t)c;
}

// One thread per node run of the node-sorted placements: walk the run backwards from the final state.
// before[c] (c = position in pod order) = final + the requests of this and every later placement there.
__global__ void k_commit_before(const int32_t *skey, const int32_t *spos, int64_t nc, const int32_t *cpod,
                                const NodeRec *nodes, const int64_t *rc, const int64_t *rm, int64_t *before) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nc) return;
    if (t + 1 < nc && skey[t + 1] == skey[t]) return;  // not the last placement of its node
    const NodeRec &nd = nodes[skey[t]];
    int64_t a0 = nd.a[0], a1 = nd.a[1], a2 = nd.a[2];
    for (int64_t u = t; u >= 0 && skey[u] == skey[t]; --u) {
        const int32_t c = spos[u];
        const int32_t pod = cpod[c];
        a0 = (int64_t)((uint64_t)a0 + (uint64_t)rc[pod]);  // undo used += request (wrapping, like the commit)
        a1 = (int64_t)((uint64_t)a1 + (uint64_t)rm[pod]);
        a2 = (int64_t)((uint64_t)a2 + 1ull);
        before[c] = a0;
        before[nc + c] = a1;
        before[2 * nc + c] = a2;
    }
}

// H_final: lane = NO_FIT pod, node rows wave-uniform (scalar loads), nodes split over blockIdx.y.
template <bool LAB>
__global__ __launch_bounds__(256) void k_hist_final(const int32_t *fpod, int64_t nf, const int64_t *rc, const int64_t *rm,
                                                    const int64_t *rp, const uint64_t *sel, const NodeRec *nodes,
                                                    int64_t n, unsigned long long *counts) {
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = f < nf;
    const int32_t pod = in ? fpod[f] : 0;
    const int64_t qc = in ? rc[pod] : 0, qm = in ? rm[pod] : 0, qp = in ? rp[pod] : 0;
    const uint64_t qs = (LAB && in) ? sel[pod] : 0;
    const int64_t per = (n + gridDim.y - 1) / gridDim.y;
    const int64_t lo = (int64_t)blockIdx.y * per;
    const int64_t hi = lo + per < n ? lo + per : n;
    const NodeRecC *rows = (const NodeRecC *)nodes;
    uint32_t c1 = 0, c2 = 0, c3 = 0, c4 = 0;
    for (int64_t j = lo; j < hi; ++j) {
        const NodeRec nd = load_row(rows + j);
        const bool f1 = nd.a[0] < qc;
        const bool f2 = !f1 && nd.a[1] < qm;
        const bool f3 = !f1 && !f2 && nd.a[2] < qp;
        const bool f4 = LAB && !f1 && !f2 && !f3 && (nd.labels & qs) != qs;
        c1 += f1; c2 += f2; c3 += f3; c4 += f4;
    }
    if (!in || hi <= lo) return;
    unsigned long long *o = counts + (size_t)f * kNumReasons;
    const uint32_t nfit = (uint32_t)(hi - lo) - c1 - c2 - c3 - c4;
    atomicAdd(o + 0, (unsigned long long)nfit);
    atomicAdd(o + 1, (unsigned long long)c1);
    atomicAdd(o + 2, (unsigned long long)c2);
    atomicAdd(o + 3, (unsigned long long)c3);
    if (LAB) atomicAdd(o + 4, (unsigned long long)c4);
}

// Corrections: lane = NO_FIT pod i; the placements after it (in pod order) move node n_k from
// after_k (its final-side state) back to before_k.  Placements are wave-uniform.
template <bool LAB>
__global__ __launch_bounds__(64) void k_hist_correct(const int32_t *fpod, int64_t nf, const int32_t *cpod, int64_t nc,
                                                     const int64_t *before, const int32_t *idx, int64_t node_lo,
                                                     const int64_t *rc, const int64_t *rm, const int64_t *rp,
                                                     const uint64_t *sel, const NodeRec *nodes,
                                                     unsigned long long *counts) {
    const int64_t f = (int64_t)blockIdx.x * 64 + threadIdx.x;
    const bool in = f < nf;
    const int32_t pod = in ? fpod[f] : 0x7fffffff;
    const int64_t qc = in ? rc[pod] : 0, qm = in ? rm[pod] : 0, qp = in ? rp[pod] : 0;
    const uint64_t qs = (LAB && in) ? sel[pod] : 0;
    // first placement after this lane's pod: binary search in the pod-ordered placements
    int64_t lo = 0, hi = nc;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (cpod[mid] > pod) hi = mid; else lo = mid + 1;
    }
    // the wave walks from its earliest start (NO_FIT pods are in pod order: lane 0's)
    const int32_t start = __builtin_amdgcn_readfirstlane((int32_t)lo);
    const int32_t ncu = (int32_t)nc;
    int32_t d[kNumReasons] = {0, 0, 0, 0, 0};
    for (int32_t c = start; c < ncu; ++c) {
        const int32_t kp = cpod[c];               // wave-uniform
        const int64_t b0 = before[c], b1 = before[nc + c], b2 = before[2 * nc + c];
        const int64_t a0 = wsub(b0, rc[kp]), a1 = wsub(b1, rm[kp]), a2 = wsub(b2, 1);
        const uint64_t lab = LAB ? nodes[(int64_t)idx[kp] - node_lo].labels : 0;
        const int rb = reason_of(qc, qm, qp, qs, b0, b1, b2, lab, LAB);
        const int ra = reason_of(qc, qm, qp, qs, a0, a1, a2, lab, LAB);
        const bool on = c >= lo && rb != ra;
#pragma unroll
        for (int r = 0; r < kNumReasons; ++r) d[r] += on ? (int)(rb == r) - (int)(ra == r) : 0;
    }
    if (!in) return;
    unsigned long long *o = counts + (size_t)f * kNumReasons;
#pragma unroll
    for (int r = 0; r < kNumReasons; ++r)
        if (d[r]) atomicAdd(o + r, (unsigned long long)(long long)d[r]);
}

// State one pod saw at its turn: final + the placements after it (on this rank's nodes).
__global__ void k_credit_after(const int32_t *idx, int64_t p, int64_t pod, int64_t node_lo, int64_t n_local,
                               const int64_t *rc, const int64_t *rm, unsigned long long *state) {
    const int64_t k = pod + 1 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= p) return;
    const int64_t j = (int64_t)idx[k] - node_lo;
    if (idx[k] < 0 || j < 0 || j >= n_local) return;
    atomicAdd(state + j, (unsigned long long)rc[k]);
    atomicAdd(state + n_local + j, (unsigned long long)rm[k]);
    atomicAdd(state + 2 * n_local + j, 1ull);
}

__global__ void k_state_of(const NodeRec *nodes, int64_t n, int64_t *state) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    state[j] = nodes[j].a[0];
    state[n + j] = nodes[j].a[1];
    state[2 * n + j] = nodes[j].a[2];
}

__global__ void k_explain_state(const int64_t *state, const NodeRec *nodes, int64_t n, int64_t rc, int64_t rm,
                                int64_t rp, uint64_t sel, int use_labels, uint8_t *reason,
                                unsigned long long *counts) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int r = -1;
    if (j < n) {
        r = reason_of(rc, rm, rp, sel, state[j], state[n + j], state[2 * n + j], nodes[j].labels, use_labels != 0);
        if (reason) reason[j] = (uint8_t)r;
    }
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < kNumReasons; ++k) {
        const unsigned long long m = __ballot(r == k);
        if (lane == 0 && m) atomicAdd(counts + k, (unsigned long long)__popcll(m));
    }
}

size_t al(size_t x) { return (x + 255) / 256 * 256; }

}  // namespace

hipError_t explain_batch(const ExplainArgs &a, void **ws, size_t *ws_bytes, unsigned long long *counts, hipStream_t s) {
    const int64_t p = a.p, n = a.n_local;
    // workspace: flags, compacted pod lists, sort keys/values, before states, cub temp
    size_t cub_sel = 0, cub_sort = 0;
    hipError_t e;
    e = hipcub::DeviceSelect::Flagged(nullptr, cub_sel, (const int32_t *)nullptr, (const uint8_t *)nullptr,
                                      (int32_t *)nullptr, (int64_t *)nullptr, (int)p, s);
    if (e != hipSuccess) return e;
    e = hipcub::DeviceRadixSort::SortPairs(nullptr, cub_sort, (const int32_t *)nullptr, (int32_t *)nullptr,
                                           (const int32_t *)nullptr, (int32_t *)nullptr, (int)p, 0, 32, s);
    if (e != hipSuccess) return e;
    const size_t off_placed = 0, off_nofit = al(off_placed + p), off_cpod = al(off_nofit + p), off_fpod = al(off_cpod + 4 * p), off_nsel = al(off_fpod + 4 * p),
                 off_key = al(off_nsel + 16), off_pos = al(off_key + 4 * p), off_skey = al(off_pos + 4 * p),
                 off_spos = al(off_skey + 4 * p), off_before = al(off_spos + 4 * p),
                 off_cub = al(off_before + 24 * p), total = al(off_cub + std::max(cub_sel, cub_sort));
    if (*ws_bytes < total) {
        if (*ws) hipFree(*ws);
        *ws = nullptr;
        *ws_bytes = 0;
        if ((e = hipMalloc(ws, total)) != hipSuccess) return e;
        *ws_bytes = total;
    }
    char *w = static_cast<char *>(*ws);
    uint8_t *placed = (uint8_t *)(w + off_placed), *nofit = (uint8_t *)(w + off_nofit);
    int32_t *cpod = (int32_t *)(w + off_cpod), *fpod = (int32_t *)(w + off_fpod);
    int64_t *nsel = (int64_t *)(w + off_nsel);
    int32_t *key = (int32_t *)(w + off_key), *pos = (int32_t *)(w + off_pos);
    int32_t *skey = (int32_t *)(w + off_skey), *spos = (int32_t *)(w + off_spos);
    int64_t *before = (int64_t *)(w + off_before);
    void *cub = w + off_cub;
    const unsigned gp = (unsigned)((p + 255) / 256);
    hipLaunchKernelGGL(k_commit_flags, dim3(gp), dim3(256), 0, s, a.idx, p, a.node_lo, n, placed, nofit);
    hipcub::CountingInputIterator<int32_t> it(0);  // selecting over pod indices writes the pod lists
    size_t t1 = cub_sel;
    if ((e = hipcub::DeviceSelect::Flagged(cub, t1, it, placed, cpod, nsel, (int)p, s)) != hipSuccess) return e;
    t1 = cub_sel;
    if ((e = hipcub::DeviceSelect::Flagged(cub, t1, it, nofit, fpod, nsel + 1, (int)p, s)) != hipSuccess) return e;
    int64_t hn[2] = {0, 0};
    if ((e = hipMemcpyAsync(hn, nsel, sizeof(hn), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    const int64_t nc = hn[0], nf = hn[1];
    if (nf == 0) return hipSuccess;
    if (nc > 0) {
        const unsigned gc = (unsigned)((nc + 255) / 256);
        hipLaunchKernelGGL(k_commit_keys, dim3(gc), dim3(256), 0, s, cpod, a.idx, nc, a.node_lo, key, pos);
        size_t t2 = cub_sort;
        int bits = 1;
        while (bits < 31 && ((int64_t)1 << bits) <= n) ++bits;
        if ((e = hipcub::DeviceRadixSort::SortPairs(cub, t2, key, skey, pos, spos, (int)nc, 0, bits, s)) != hipSuccess)
            return e;
        hipLaunchKernelGGL(k_commit_before, dim3(gc), dim3(256), 0, s, skey, spos, nc, cpod, a.nodes, a.rc, a.rm,
                           before);
    }
    const unsigned gf = (unsigned)((nf + 255) / 256);
    const unsigned ych = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, std::max<int64_t>(1, 8192 / gf)));
    if (a.use_labels)
        hipLaunchKernelGGL(k_hist_final<true>, dim3(gf, ych), dim3(256), 0, s, fpod, nf, a.rc, a.rm, a.rp, a.sel,
                           a.nodes, n, counts);
    else
        hipLaunchKernelGGL(k_hist_final<false>, dim3(gf, ych), dim3(256), 0, s, fpod, nf, a.rc, a.rm, a.rp, a.sel,
                           a.nodes, n, counts);
    if (nc > 0) {
        const unsigned gw = (unsigned)((nf + 63) / 64);
        if (a.use_labels)
            hipLaunchKernelGGL(k_hist_correct<true>, dim3(gw), dim3(64), 0, s, fpod, nf, cpod, nc, before, a.idx,
                               a.node_lo, a.rc, a.rm, a.rp, a.sel, a.nodes, counts);
        else
            hipLaunchKernelGGL(k_hist_correct<false>, dim3(gw), dim3(64), 0, s, fpod, nf, cpod, nc, before, a.idx,
                               a.node_lo, a.rc, a.rm, a.rp, a.sel, a.nodes, counts);
    }
    *a.n_nofit = nf;
    return hipMemcpyAsync(a.fpod_out, fpod, (size_t)nf * sizeof(int32_t), hipMemcpyDeviceToDevice, s);
}

hipError_t explain_pod_at(const ExplainArgs &a, int64_t pod, int64_t *state, uint8_t *reason,
                          unsigned long long *counts, hipStream_t s) {
    const int64_t n = a.n_local;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_state_of, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a.nodes, n, state);
    const int64_t rest = a.p - pod - 1;
    if (rest > 0)
        hipLaunchKernelGGL(k_credit_after, dim3((unsigned)((rest + 255) / 256)), dim3(256), 0, s, a.idx, a.p, pod,
                           a.node_lo, n, a.rc, a.rm, (unsigned long long *)state);
    hipLaunchKernelGGL(k_explain_state, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, state, a.nodes, n,
                       a.q_rc, a.q_rm, a.q_rp, a.q_sel, (int)a.use_labels, reason, counts);
    return hipGetLastError();
}

}  // namespace ksched
