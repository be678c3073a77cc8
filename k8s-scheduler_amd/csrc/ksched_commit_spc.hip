// ksched_commit_spc.hip -- the stream pipeline's ordered commit kernel (one launch per batch); the commit
// itself is commit_spc_batch (ksched_commit.h), shared with the persistent pipeline's commit workgroup.
#include <hip/hip_runtime.h>

#include "ksched_commit.h"

namespace ksched {

// <= 192 VGPRs (amdgpu_num_vgpr counts half the unified gfx950 file): beside a resident score
// workgroup (two 64-VGPR waves per SIMD) the commit's two waves per SIMD must fit the 512-entry file,
// or a score grid polling for this commit would never let it in.
template <int K, int PRIO, int DOM, bool LAB, bool F53>
__global__ __launch_bounds__(kSpcThreads) __attribute__((amdgpu_num_vgpr(96))) void k_commit_spc(CommitArgs A) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical: win issue arbitration over co-resident score waves
    extern __shared__ __attribute__((aligned(16))) char smem[];
    commit_spc_batch<K, PRIO, DOM, LAB, F53, false>(A, smem);
}

namespace {

template <int K, int PRIO, int DOM, bool LAB, bool F53>
hipError_t commit_spc_one(const CommitArgs &a, hipStream_t s) {
    static bool attr_set = false;
    const size_t lds = spc_lds_bytes<K>();
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void *)k_commit_spc<K, PRIO, DOM, LAB, F53>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    hipLaunchKernelGGL((k_commit_spc<K, PRIO, DOM, LAB, F53>), dim3(1), dim3(kSpcThreads), lds, s, a);
    return hipGetLastError();
}

template <int PRIO, int DOM, bool LAB, bool F53>
hipError_t commit_spc_k(int K, const CommitArgs &a, hipStream_t s) {
    switch (K) {
        case 4: return commit_spc_one<4, PRIO, DOM, LAB, F53>(a, s);
        case 8: return commit_spc_one<8, PRIO, DOM, LAB, F53>(a, s);
        case 16: return commit_spc_one<16, PRIO, DOM, LAB, F53>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

namespace {
template <int K, int PRIO, int DOM, bool LAB, bool F53>
hipError_t spc_attr_one(hipFuncAttributes *at, size_t *lds) {
    *lds = spc_lds_bytes<K>();
    return hipFuncGetAttributes(at, (const void *)k_commit_spc<K, PRIO, DOM, LAB, F53>);
}
template <int PRIO, int DOM, bool LAB, bool F53>
hipError_t spc_attr_k(int K, hipFuncAttributes *at, size_t *lds) {
    switch (K) {
        case 4: return spc_attr_one<4, PRIO, DOM, LAB, F53>(at, lds);
        case 8: return spc_attr_one<8, PRIO, DOM, LAB, F53>(at, lds);
        case 16: return spc_attr_one<16, PRIO, DOM, LAB, F53>(at, lds);
        default: return hipErrorInvalidValue;
    }
}
}  // namespace

hipError_t commit_spc_attributes(int K, int prio, int dom, bool lab, bool f53, hipFuncAttributes *at, size_t *lds) {
    KSCHED_DISPATCH(prio, dom, lab, f53, (spc_attr_k<P_, D_, L_, F_>(K, at, lds)));
}

hipError_t launch_commit_spc(int K, int prio, int dom, bool lab, bool f53, const CommitArgs &a, hipStream_t s) {
    if (a.B > 64) return hipErrorInvalidValue;
    KSCHED_DISPATCH(prio, dom, lab, f53, (commit_spc_k<P_, D_, L_, F_>(K, a, s)));
}

}  // namespace ksched
