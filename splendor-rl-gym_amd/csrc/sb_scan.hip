// sb_scan.hip — device-wide exclusive scan of u32 values (reduce-then-scan, 4096-element tiles).
// Used for next_queue offsets (the (parent rank, ordinal) order of src/solver.py:446-450), radix
// histogram columns and the MT accept compaction.
#include "sb_block.h"
#include "sb_internal.h"

namespace sb {

constexpr int SCAN_NT = 256;
constexpr int SCAN_IPT = SCAN_TILE / SCAN_NT;   // 16 items per thread, blocked

__global__ __launch_bounds__(SCAN_NT) void k_scan_reduce(const uint32_t* __restrict__ in, int64_t n,
                                                          uint32_t* __restrict__ tile_sums) {
    __shared__ uint32_t lds[SCAN_NT / 64 + 1];
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < SCAN_IPT; j++) {
        int64_t i = base + (int64_t)j * SCAN_NT + threadIdx.x;   // strided: coalesced
        if (i < n) s += in[i];
    }
    uint32_t tot;
    block_excl_scan<SCAN_NT>(s, lds, &tot);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
}

// single workgroup: exclusive scan of the tile sums in place; writes the grand total
__global__ __launch_bounds__(1024) void k_scan_tiles(uint32_t* __restrict__ tile_sums, int64_t ntiles,
                                                      uint32_t* __restrict__ total) {
    __shared__ uint32_t lds[1024 / 64 + 1];
    uint32_t carry = 0;
    for (int64_t b = 0; b < ntiles; b += 1024) {
        int64_t i = b + threadIdx.x;
        uint32_t v = i < ntiles ? tile_sums[i] : 0;
        uint32_t tot;
        uint32_t ex = block_excl_scan<1024>(v, lds, &tot);
        if (i < ntiles) tile_sums[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0 && total) *total = carry;
}

// Wave w of a tile scans its contiguous quarter (1024 values) 64 at a time: every load and store is one
// coalesced 256-byte row (the blocked layout, 16 consecutive values per thread, spread a wave's accesses
// over 64 rows per instruction: 25.7 us for 4M values against a 5 us read + write)
#ifndef SB_SCAN_BLOCKED
#define SB_SCAN_BLOCKED 0
#endif
__global__ __launch_bounds__(SCAN_NT) void k_scan_apply(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                         int64_t n, const uint32_t* __restrict__ tile_sums) {
    __shared__ uint32_t lds[SCAN_NT / 64 + 1];
    if (SB_SCAN_BLOCKED) {
        const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_IPT;   // blocked
        uint32_t v[SCAN_IPT];
        uint32_t s = 0;
#pragma unroll
        for (int j = 0; j < SCAN_IPT; j++) {
            int64_t i = base + j;
            v[j] = i < n ? in[i] : 0;
            s += v[j];
        }
        uint32_t tot;
        uint32_t run = block_excl_scan<SCAN_NT>(s, lds, &tot) + tile_sums[blockIdx.x];
#pragma unroll
        for (int j = 0; j < SCAN_IPT; j++) {
            int64_t i = base + j;
            if (i < n) out[i] = run;
            run += v[j];
        }
        return;
    }
    constexpr int NW = SCAN_NT / 64, WSPAN = SCAN_TILE / NW;   // 1024 values per wave
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t wbase = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)w * WSPAN + lane;
    uint32_t v[SCAN_IPT];
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < SCAN_IPT; j++) {
        const int64_t i = wbase + (int64_t)j * 64;
        v[j] = i < n ? in[i] : 0;
        s += v[j];
    }
    const uint32_t ws = wave_incl_scan(s);
    if (lane == 63) lds[w] = ws;
    __syncthreads();
    uint32_t carry = tile_sums[blockIdx.x];
    for (int x = 0; x < w; x++) carry += lds[x];
#pragma unroll
    for (int j = 0; j < SCAN_IPT; j++) {
        const uint32_t inc = wave_incl_scan(v[j]);
        const int64_t i = wbase + (int64_t)j * 64;
        if (i < n) out[i] = carry + inc - v[j];
        carry += (uint32_t)__shfl((int)inc, 63, 64);
    }
}

void scan_tiles_inplace(uint32_t* tiles, int64_t ntiles, uint32_t* total_dev, hipStream_t st) {
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(1024), 0, st, tiles, ntiles, total_dev);
}

void scan_exclusive_u32_sums(const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total_dev, ScanScratch& s,
                             hipStream_t st) {
    const int64_t ntiles = (n + SCAN_TILE - 1) / SCAN_TILE;
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(1024), 0, st, s.tiles.p, ntiles, total_dev);
    hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)ntiles), dim3(SCAN_NT), 0, st, in, out, n, s.tiles.p);
    SB_HIP(hipGetLastError());
}

void scan_exclusive_u32(const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total_dev, ScanScratch& s,
                        hipStream_t st) {
    if (n <= 0) {
        if (total_dev) SB_HIP(hipMemsetAsync(total_dev, 0, 4, st));
        return;
    }
    int64_t ntiles = (n + SCAN_TILE - 1) / SCAN_TILE;
    s.tiles.ensure((size_t)ntiles);
    hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)ntiles), dim3(SCAN_NT), 0, st, in, n, s.tiles.p);
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(1024), 0, st, s.tiles.p, ntiles, total_dev);
    hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)ntiles), dim3(SCAN_NT), 0, st, in, out, n, s.tiles.p);
    SB_HIP(hipGetLastError());
}

}  // namespace sb
