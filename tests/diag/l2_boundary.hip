// Kernel-boundary visibility on MI355X: does a kernel see the values an earlier kernel (or a hipMemsetAsync) on the
// same stream wrote, on every XCD, when its own XCD's L2 may still hold the line from before?  Each round: a
// reader grid touches the lines (sc1 and plain loads, every XCD), a writer (1 block, plain stores / sc1 stores /
// hipMemsetAsync) writes round-specific values, then a checker grid reads them back (sc1 and plain).  Prints the
// number of stale observations per writer kind.  hipcc --offload-arch=gfx950 -O2 l2_boundary.hip -o /tmp/l2b
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int kLines = 64;       // 128-byte lines, one u64 probed per line
constexpr int kBlocks = 2048;

__device__ __forceinline__ uint64_t ld_sc1(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_touch(const uint64_t *buf, uint64_t *sink) {
    uint64_t acc = 0;
    for (int l = threadIdx.x; l < kLines; l += blockDim.x) acc += ld_sc1(buf + l * 16) + buf[l * 16 + 1];
    if (acc == 0x123456789ull) sink[blockIdx.x] = acc;  // keep the loads
}
__global__ void k_write_plain(uint64_t *buf, uint64_t v) {
    for (int l = threadIdx.x; l < kLines; l += blockDim.x) { buf[l * 16] = v; buf[l * 16 + 1] = v; }
}
__global__ void k_write_sc1(uint64_t *buf, uint64_t v) {
    for (int l = threadIdx.x; l < kLines; l += blockDim.x) {
        __hip_atomic_store(buf + l * 16, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(buf + l * 16 + 1, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// stale[0]: sc1 loads that saw another value, stale[1]: plain loads
__global__ void k_check(const uint64_t *buf, uint64_t v, unsigned long long *stale) {
    unsigned long long s0 = 0, s1 = 0;
    for (int l = threadIdx.x; l < kLines; l += blockDim.x) {
        s0 += ld_sc1(buf + l * 16) != v;
        s1 += buf[l * 16 + 1] != v;
    }
    if (s0) atomicAdd(stale, s0);
    if (s1) atomicAdd(stale + 1, s1);
}

// an earlier grid's atomic stores of a large value from every XCD, a 1-block plain-store reset to 0, then atomic
// maxima of small values from every XCD: each must see the reset (result <= the small values)
__global__ void k_big(uint64_t *buf) {
    for (int l = threadIdx.x; l < kLines; l += blockDim.x)
        __hip_atomic_store(buf + l * 16, 1ull << 62, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void k_max(uint64_t *buf, uint64_t v, unsigned long long *stale) {
    unsigned long long s = 0;
    for (int l = threadIdx.x; l < kLines; l += blockDim.x) {
        const uint64_t old = __hip_atomic_fetch_max(buf + l * 16, v + blockIdx.x % 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s += old >= (1ull << 62);
    }
    if (s) atomicAdd(stale, s);
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 2000;
    uint64_t *buf = nullptr, *sink = nullptr;
    unsigned long long *stale = nullptr;
    CK(hipMalloc(&buf, kLines * 128));
    CK(hipMalloc(&sink, kBlocks * 8));
    CK(hipMalloc(&stale, 16));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const char *names[3] = {"plain-store kernel", "sc1-store kernel", "hipMemsetAsync"};
    for (int kind = 0; kind < 3; ++kind) {
        CK(hipMemsetAsync(stale, 0, 16, s));
        for (int r = 1; r <= rounds; ++r) {
            hipLaunchKernelGGL(k_touch, dim3(kBlocks), dim3(64), 0, s, buf, sink);
            const uint64_t v = kind == 2 ? (uint64_t)(r & 0xff) * 0x0101010101010101ull : (uint64_t)r * 7919u + kind;
            if (kind == 0) hipLaunchKernelGGL(k_write_plain, dim3(1), dim3(64), 0, s, buf, v);
            else if (kind == 1) hipLaunchKernelGGL(k_write_sc1, dim3(1), dim3(64), 0, s, buf, v);
            else CK(hipMemsetAsync(buf, (int)(r & 0xff), kLines * 128, s));
            hipLaunchKernelGGL(k_check, dim3(kBlocks), dim3(64), 0, s, buf, v, stale);
        }
        unsigned long long h[2];
        CK(hipMemcpyAsync(h, stale, 16, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        printf("%-20s rounds %d: stale sc1 loads %llu, stale plain loads %llu (of %llu each)\n", names[kind], rounds, h[0], h[1],
               (unsigned long long)rounds * kBlocks * kLines);
    }
    {
        CK(hipMemsetAsync(stale, 0, 16, s));
        for (int r = 1; r <= rounds; ++r) {
            hipLaunchKernelGGL(k_big, dim3(kBlocks), dim3(64), 0, s, buf);
            hipLaunchKernelGGL(k_write_plain, dim3(1), dim3(64), 0, s, buf, 0ull);
            hipLaunchKernelGGL(k_max, dim3(kBlocks), dim3(64), 0, s, buf, (uint64_t)r, stale);
        }
        unsigned long long h[2];
        CK(hipMemcpyAsync(h, stale, 16, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        printf("%-20s rounds %d: atomic maxima that saw the earlier value %llu\n", "atomic-after-reset", rounds, h[0]);
    }
    return 0;
}
