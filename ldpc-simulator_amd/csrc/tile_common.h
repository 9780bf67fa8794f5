// tile_common.h -- synchronisation helpers shared by the tile-resident parity
// decoders (tile_kernels.hip: 64 frames per workgroup; tile_sub.hip: 16 or 8).
// Wavefronts of one workgroup hand the check-row product along through LDS
// words guarded by flags (no workgroup barrier on the chain).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

#include "cn_common.h"
#include "spa_device.h"

namespace ldpc {
namespace {

__host__ __device__ inline size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

// End of a tile decoder (every wavefront arrives): the rare rows it took in
// kernel -- its LDS rare-row sequence counts one per wavefront and rare row --
// into the decoder's running total (DevState::rare_count[3], ldpc_rare_rows_read).
__device__ __forceinline__ void count_rare_rows(const DevState &st, const int *tseq, int waves) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const int n = *tseq / waves;
        if (n) atomicAdd(&st.rare_count[3], n);
    }
}

__device__ __forceinline__ int lds_ld(const int *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(int *p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// LDS-only fences: order this wavefront's LDS accesses around a flag without
// waiting for its outstanding global stores.
__device__ __forceinline__ void lds_release() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local"); }
__device__ __forceinline__ void lds_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local"); }
// Polls: kSleep sleeps (s_sleep 1) between flag reads (tile_kernel); the
// sub-tile decoder spins (measured 1.7 % faster there, profiles/r2q logs).
template <bool kSleep = true>
__device__ __forceinline__ void wait_flag(const int *p, int v) {
    while (uniform(lds_ld(p)) != v)
        if (kSleep) __builtin_amdgcn_s_sleep(1);
    lds_acquire();
}
template <bool kSleep = true>
__device__ __forceinline__ void wait_ge(const int *p, int v) {
    while (uniform(lds_ld(p)) < v)
        if (kSleep) __builtin_amdgcn_s_sleep(1);
    lds_acquire();
}
// A read-only table entry at a wavefront-uniform index by a scalar load (SMEM,
// lgkmcnt): the vector load's vmcnt wait would also wait for every store the
// wavefront has in flight (the P3 order tables: this row's E_new stores).
__device__ __forceinline__ int ld_table(const int *p, int i) {
    return *(const __attribute__((address_space(4))) int *)(p + uniform(i));
}
// Load through L2 (not this CU's L1): data another wavefront of the workgroup
// stored (posteriors, rare-row scratch).
__device__ __forceinline__ double ld_l2(const double *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


}  // namespace
}  // namespace ldpc
