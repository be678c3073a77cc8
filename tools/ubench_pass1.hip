// Microbenchmark of the screened scan's pass 1 as k_pipe runs it (exploration tool, not product code): one
// workgroup per CU, 8 waves, f32 screen reciprocals in LDS ([R] float4), each wave scanning rows r = w (mod 8);
// cycles per row per wave from s_memtime.  Stages add the pieces of the real loop one at a time:
//   S=0 load + fractions + polynomial         S=1 + f32 predicate flags, non-fitting form, select
//   S=2 + top-4 of lower bounds               S=3 + f16 record store          S=4 + ambiguous-row queue (ballot)
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I../k8s-scheduler_amd/csrc ubench_pass1.hip -o ubench_pass1
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ksched_device.h"

using namespace ksched;

template <int S, int PU, int W>
__global__ __launch_bounds__(1024) void k_pass1(const float4 *ysrc, int R, const int64_t *req, int reps, uint64_t *out,
                                               uint32_t *sink) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float4 *ysq = reinterpret_cast<float4 *>(smem);
    const int QW = (R + W - 1) / W;
    uint16_t *hrec = reinterpret_cast<uint16_t *>(smem + (size_t)R * 16);
    uint16_t *arow = hrec + (size_t)W * QW * 64;
    for (int e = threadIdx.x; e < R; e += blockDim.x) ysq[e] = ysrc[e];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const float qc = screen_req(req[lane * 3]), qm = screen_req(req[lane * 3 + 1]), qp = screen_req(req[lane * 3 + 2]);
    uint16_t *hw = hrec + (size_t)wave * QW * 64 + lane;
    uint32_t t[4] = {0, 0, 0, 0};
    int cnt = 0, na = 0;
    float acc = 0.f;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < reps; ++it) {
        for (int r0 = wave; r0 < R; r0 += W * PU) {
            float4 yv[PU];
#pragma unroll
            for (int u = 0; u < PU; ++u) { const int r = r0 + u * W; yv[u] = ysq[r < R ? r : r0]; }
            uint32_t xs[PU];
#pragma unroll
            for (int u = 0; u < PU; ++u) {
                const int r = r0 + u * W;
                const bool valid = r < R;
                const float c = qc * yv[u].x, m = qm * yv[u].y, p = qp * (yv[u].z + yv[u].w);
                float v;
                bool lo_ok = true, amb = false, f = true;
                if (S == 0) {
                    const float Sx = (c + m) + p, Q = (c * c + m * m) + p * p;
                    v = ((10.0f - (5.0f / 3.0f) * Sx) - (5.0f / 3.0f) * Q) + (5.0f / 9.0f) * (Sx * Sx);
                } else {
                    const bool okc = c < kFracLo, okm = m < kFracLo, okp = p < kFracLo;
                    amb = !(okc || c > kFracHi) || !(okm || m > kFracHi) || !(okp || p > kFracHi);
                    f = okc & okm & okp;
                    v = screen_q(c, m, p, okc, okm, okp, &lo_ok);
                }
                cnt += (valid && f && !amb) ? 1 : 0;
                xs[u] = (valid && lo_ok && !amb) ? __float_as_uint(v + (1.0f - kScreenEps)) : 0u;
                if (S < 2) acc += v;
                if (S >= 3) {
                    const float w = 10.0f - v;
                    const float wd = w - __builtin_fabsf(w) * 0x1p-10f - 0x1p-24f;
                    if (valid) hw[(size_t)(r / W) * 64] = __half_as_ushort(__float2half_rn(amb ? __builtin_nanf("") : wd));
                }
                if (S >= 4) {
                    const bool anya = __ballot(valid && amb) != 0;
                    if (lane == 0) arow[wave * QW + (na & 31)] = (uint16_t)r;
                    na += anya ? 1 : 0;
                }
            }
            if (S >= 2) {
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
            } else {
#pragma unroll
                for (int u = 0; u < PU; ++u) t[0] ^= xs[u];
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    sink[blockIdx.x * blockDim.x + threadIdx.x] = t[3] + t[0] + cnt + na + __float_as_uint(acc);
    if (lane == 0) out[blockIdx.x * W + wave] = t1 - t0;
}

template <int S, int PU, int W = 8>
double run(const float4 *d_y, int R, const int64_t *d_req, int grid, uint64_t *d_out, uint32_t *d_sink) {
    const int reps = 200;
    const int QW = (R + W - 1) / W;
    const size_t lds = (size_t)R * 16 + (size_t)W * QW * 64 * 2 + W * QW * 2 + 64;
    (void)hipFuncSetAttribute((const void *)k_pass1<S, PU, W>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((k_pass1<S, PU, W>), dim3(grid), dim3(64 * W), lds, 0, d_y, R, d_req, reps, d_out, d_sink);
    if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); exit(1); }
    std::vector<uint64_t> h((size_t)grid * W);
    (void)hipMemcpy(h.data(), d_out, h.size() * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (auto v : h) s += (double)v;
    return s / (double)h.size() / ((double)QW * reps);  // cycles per row per wave
}

int main() {
    const int R = 393, grid = 256;
    std::vector<float4> y(R);
    srand(7);
    for (int i = 0; i < R; ++i)
        y[i] = make_float4(1.0f / (2000 + rand() % 60000), 1.0f / ((1 << 20) + rand() % (200 << 20)), 1.0f / (55 + rand() % 55), 0.0f);
    std::vector<int64_t> req(64 * 3);
    for (int l = 0; l < 64; ++l) { req[l * 3] = 50 + rand() % 6000; req[l * 3 + 1] = (64 << 10) + rand() % (12 << 20); req[l * 3 + 2] = 1 + rand() % 3; }
    float4 *d_y; int64_t *d_req; uint64_t *d_out; uint32_t *d_sink;
    (void)hipMalloc(&d_y, R * 16); (void)hipMalloc(&d_req, req.size() * 8);
    (void)hipMalloc(&d_out, grid * 16 * 8); (void)hipMalloc(&d_sink, grid * 1024 * 4);
    (void)hipMemcpy(d_y, y.data(), R * 16, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_req, req.data(), req.size() * 8, hipMemcpyHostToDevice);
    printf("cycles per row per wave (8 waves/WG, %d WGs): S0 %.1f | S1 %.1f | S2 %.1f | S3 %.1f | S4 %.1f | S4 PU8 %.1f | S4 PU2 %.1f\n",
           grid, run<0, 4>(d_y, R, d_req, grid, d_out, d_sink), run<1, 4>(d_y, R, d_req, grid, d_out, d_sink),
           run<2, 4>(d_y, R, d_req, grid, d_out, d_sink), run<3, 4>(d_y, R, d_req, grid, d_out, d_sink),
           run<4, 4>(d_y, R, d_req, grid, d_out, d_sink), run<4, 8>(d_y, R, d_req, grid, d_out, d_sink),
           run<4, 2>(d_y, R, d_req, grid, d_out, d_sink));
    printf("waves per SIMD 1/2/3/4 (W=4/8/12/16), cycles per row per wave: S0 %.1f %.1f %.1f %.1f | S2 %.1f %.1f %.1f %.1f\n",
           run<0, 4, 4>(d_y, R, d_req, grid, d_out, d_sink), run<0, 4, 8>(d_y, R, d_req, grid, d_out, d_sink),
           run<0, 4, 12>(d_y, R, d_req, grid, d_out, d_sink), run<0, 4, 16>(d_y, R, d_req, grid, d_out, d_sink),
           run<2, 4, 4>(d_y, R, d_req, grid, d_out, d_sink), run<2, 4, 8>(d_y, R, d_req, grid, d_out, d_sink),
           run<2, 4, 12>(d_y, R, d_req, grid, d_out, d_sink), run<2, 4, 16>(d_y, R, d_req, grid, d_out, d_sink));
    return 0;
}
