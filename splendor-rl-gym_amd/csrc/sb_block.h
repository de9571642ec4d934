// sb_block.h — wave64 / workgroup primitives (gfx950: 64-lane wavefronts, 64-bit ballots).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sb {

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }
__device__ __forceinline__ uint64_t lanemask_lt() { return (1ull << lane_id()) - 1ull; }

// inclusive wave64 prefix sum
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int l = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(v, d, 64);
        if (l >= d) v += t;
    }
    return v;
}

// Exclusive scan across a workgroup of NT threads (NT multiple of 64, <= 1024).
// lds must hold NT/64 + 1 words.  Returns the exclusive prefix; *total = workgroup sum.
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* lds, uint32_t* total) {
    constexpr int NW = NT / 64;
    const int w = threadIdx.x >> 6;
    uint32_t inc = wave_incl_scan(v);
    if (lane_id() == 63) lds[w] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int i = 0; i < NW; i++) {
            uint32_t t = lds[i];
            lds[i] = run;
            run += t;
        }
        lds[NW] = run;
    }
    __syncthreads();
    uint32_t r = lds[w] + inc - v;
    *total = lds[NW];
    __syncthreads();
    return r;
}

}  // namespace sb
