// Microbenchmark of the screened scan's pass-1 row loop (exploration tool, not product code): one workgroup per
// CU, 8 (or W) waves, node rows in LDS as in k_pipe, each wave scanning its rows r = w (mod W) for many
// repetitions; cycles per row per wave from s_memtime.  Variants isolate the cost of the pieces:
//   V=0 full pass 1 (i64 fit compares + f32 screen + top-4 of lower bounds)
//   V=1 no i64 compares (fit assumed)          V=2 no screen math (fit + count only)
//   V=3 i64 compares replaced by f64 compares  V=4 only the LDS row loads (sum of words)
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I../k8s-scheduler_amd/csrc ubench_screen.hip -o ubench_screen
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ksched_device.h"

using namespace ksched;

template <int V, int PU>
__global__ __launch_bounds__(768) void k_bench(const NodeRec *nodes, int R, const int64_t *req, int reps, uint64_t *out,
                                               uint32_t *sink) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    NodeRec *rows = reinterpret_cast<NodeRec *>(smem);
    const int W = blockDim.x / 64;
    for (int e = threadIdx.x; e < R * 6; e += blockDim.x)
        reinterpret_cast<int4 *>(rows)[e] = reinterpret_cast<const int4 *>(nodes)[e];
    __syncthreads();
    for (int r = threadIdx.x; r < R; r += blockDim.x) {
        rows[r].ys[0] = screen_recip(rows[r].a[0]); rows[r].ys[1] = screen_recip(rows[r].a[1]);
        rows[r].ys[2] = screen_recip(rows[r].a[2]);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t rc = req[lane * 3], rm = req[lane * 3 + 1], rp = req[lane * 3 + 2];
    const double rcf = (double)rc, rmf = (double)rm, rpf = (double)rp;
    const float qc = screen_req(rc), qm = screen_req(rm), qp = screen_req(rp);
    uint32_t t[4] = {0, 0, 0, 0};
    int cnt = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < reps; ++it) {
        for (int r0 = wave; r0 < R; r0 += W * PU) {
            uint32_t xs[PU];
#pragma unroll
            for (int u = 0; u < PU; ++u) {
                const int r = r0 + u * W;
                const bool valid = r < R;
                const NodeRec &nd = rows[valid ? r : r0];
                uint32_t x = 0;
                if (V == 4) {
                    x = (uint32_t)nd.a[0] ^ (uint32_t)nd.a[1] ^ (uint32_t)nd.a[2] ^ __float_as_uint(nd.ys[0]) ^
                        __float_as_uint(nd.ys[1]) ^ __float_as_uint(nd.ys[2]);
                } else {
                    bool okc, okm, okp;
                    if (V == 1) { okc = okm = okp = true; }
                    else if (V == 3) { okc = nd.af[0] >= rcf; okm = nd.af[1] >= rmf; okp = nd.af[2] >= rpf; }
                    else { okc = nd.a[0] >= rc; okm = nd.a[1] >= rm; okp = nd.a[2] >= rp; }
                    const bool f = okc & okm & okp;
                    cnt += (valid && f) ? 1 : 0;
                    if (V != 2) {
                        bool lo_ok;
                        const float v = screen_pair(qc, qm, qp, nd.ys[0], nd.ys[1], nd.ys[2], okc, okm, okp, &lo_ok);
                        x = (valid && lo_ok) ? __float_as_uint(v + (1.0f - kScreenEps)) : 0u;
                    }
                }
                xs[u] = x;
            }
#pragma unroll
            for (int u = 0; u < PU; ++u) {
                uint32_t xv = xs[u];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t hi = t[q] > xv ? t[q] : xv;
                    xv = t[q] > xv ? xv : t[q];
                    t[q] = hi;
                }
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    sink[blockIdx.x * blockDim.x + threadIdx.x] = t[3] + cnt;
    if (lane == 0) out[blockIdx.x * W + wave] = t1 - t0;
}

template <int V, int PU>
double run(const NodeRec *d_nodes, int R, const int64_t *d_req, int W, int grid, uint64_t *d_out, uint32_t *d_sink) {
    const int reps = 200;
    const size_t lds = (size_t)R * sizeof(NodeRec);
    hipFuncSetAttribute((const void *)k_bench<V, PU>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((k_bench<V, PU>), dim3(grid), dim3(64 * W), lds, 0, d_nodes, R, d_req, reps, d_out, d_sink);
    if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); exit(1); }
    std::vector<uint64_t> h((size_t)grid * W);
    hipMemcpy(h.data(), d_out, h.size() * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (auto v : h) s += (double)v;
    s /= (double)h.size();
    const double rows_per_wave = (double)((R + W - 1) / W) * reps;
    return s / rows_per_wave;  // cycles per row per wave
}

int main() {
    const int R = 393, grid = 256;
    std::vector<NodeRec> nodes(R);
    srand(7);
    for (int i = 0; i < R; ++i) {
        NodeRec &n = nodes[i];
        n = NodeRec{};
        n.a[0] = 2000 + rand() % 60000; n.a[1] = (1 << 20) + rand() % (200 << 20); n.a[2] = 55 + rand() % 55;
        for (int k = 0; k < 3; ++k) n.af[k] = (double)n.a[k];
    }
    std::vector<int64_t> req(64 * 3);
    for (int l = 0; l < 64; ++l) { req[l * 3] = 50 + rand() % 6000; req[l * 3 + 1] = (64 << 10) + rand() % (12 << 20); req[l * 3 + 2] = 1 + rand() % 3; }
    NodeRec *d_nodes; int64_t *d_req; uint64_t *d_out; uint32_t *d_sink;
    hipMalloc(&d_nodes, R * sizeof(NodeRec)); hipMalloc(&d_req, req.size() * 8);
    hipMalloc(&d_out, grid * 16 * 8); hipMalloc(&d_sink, grid * 1024 * 4);
    hipMemcpy(d_nodes, nodes.data(), R * sizeof(NodeRec), hipMemcpyHostToDevice);
    hipMemcpy(d_req, req.data(), req.size() * 8, hipMemcpyHostToDevice);
    for (int W : {8, 12, 16}) {
        printf("W=%d waves/WG: cycles per row per wave | full %.1f | no-i64 %.1f | no-screen %.1f | f64-cmp %.1f | loads-only %.1f | full PU8 %.1f | full PU2 %.1f\n", W,
               run<0, 4>(d_nodes, R, d_req, W, grid, d_out, d_sink), run<1, 4>(d_nodes, R, d_req, W, grid, d_out, d_sink),
               run<2, 4>(d_nodes, R, d_req, W, grid, d_out, d_sink), run<3, 4>(d_nodes, R, d_req, W, grid, d_out, d_sink),
               run<4, 4>(d_nodes, R, d_req, W, grid, d_out, d_sink), run<0, 8>(d_nodes, R, d_req, W, grid, d_out, d_sink),
               run<0, 2>(d_nodes, R, d_req, W, grid, d_out, d_sink));
    }
    return 0;
}
