// FETCH_SIZE calibration for the visited set's access pattern: does the
// guide's gfx950 doubling (MI355X_MICROARCH.md HBM section: FETCH_SIZE reports half the bytes of a wide
// coalesced streaming read) also hold for random 16-B loads of a table far beyond the Infinity Cache?
//   fetchcal <table_GiB> <n_millions>   under rocprofv3 --pmc FETCH_SIZE (and TCC_EA0_RDREQ_sum ...)
// kernel 1 k_stream: a coalesced 16-B/lane read of exactly S bytes (the guide's calibrated case)
// kernel 2 k_rand:   n random 16-B loads (the visited-set probe), one per thread iteration
// kernel 3 k_rand64: n random 64-B aligned loads (4 x 16 B of one line per 4 lanes)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
__global__ void k_stream(const ulonglong2* tab, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const ulonglong2 e = tab[i];
        acc += e.x ^ e.y;
    }
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_rand(const ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const ulonglong2 e = tab[mix(i) & mask];
        acc += e.x ^ e.y;
    }
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_rand64(const ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < 4 * n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t line = mix(i >> 2) & (mask >> 2);   // 4 consecutive lanes share one 64-B block
        const ulonglong2 e = tab[line * 4 + (i & 3)];
        acc += e.x ^ e.y;
    }
    if (acc == 42) atomicAdd(sink, acc);
}

// write side of a visited-set insert (tab filled with ~0 first): tag CAS on an empty slot, the key's
// write-through store, both on one line (the insert), a returning atomicMin (a same-turn duplicate)
__global__ void k_cas(ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        acc += atomicCAS(&tab[mix(i) & mask].y, ~0ull, (unsigned long long)i);
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_st(ulonglong2* tab, uint64_t mask, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        __hip_atomic_store(&tab[mix(i + 0x1234567) & mask].x, (unsigned long long)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void k_insert(ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t h = mix(i + 0x7654321) & mask;
        const ulonglong2 e = tab[h];
        if (e.y == ~0ull) {
            const uint64_t prev = atomicCAS(&tab[h].y, ~0ull, (unsigned long long)i);
            __hip_atomic_store(&tab[h].x, (unsigned long long)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            acc += prev;
        }
        acc += e.x;
    }
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_amin(ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        acc += atomicMin(&tab[mix(i + 0x55555) & mask].y, (unsigned long long)i);
    if (acc == 42) atomicAdd(sink, acc);
}

int main(int argc, char** argv) {

    const double gib = argc > 1 ? atof(argv[1]) : 32;
    const int64_t n = (int64_t)((argc > 2 ? atof(argv[2]) : 100) * 1e6);
    uint64_t entries = 1;
    while ((double)entries * 32 <= gib * (1ull << 30)) entries <<= 1;
    ulonglong2* tab;
    unsigned long long* sink;
    if (hipMalloc(&tab, entries * 16) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMalloc(&sink, 8);
    hipMemset(tab, 0x5A, entries * 16);
    hipDeviceSynchronize();
    const int grid = 256 * 32, nt = 256;
    const int64_t ns = (int64_t)((uint64_t)4 << 30) / 16;   // 4 GiB streamed
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float ms;
    hipEventRecord(a);
    hipLaunchKernelGGL(k_stream, dim3(grid), dim3(nt), 0, 0, tab, ns, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("k_stream  %lld B read coalesced (16 B/lane)        %8.3f ms\n", (long long)(ns * 16), ms);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_rand, dim3(grid), dim3(nt), 0, 0, tab, entries - 1, n, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("k_rand    %lld random 16-B loads, table %.1f GiB  %8.3f ms  %.2f G/s\n", (long long)n, entries * 16.0 / (1 << 30),
           ms, n / ms / 1e6);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_rand64, dim3(grid), dim3(nt), 0, 0, tab, entries - 1, n, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("k_rand64  %lld random 64-B blocks (4 lanes each)   %8.3f ms  %.2f G/s\n", (long long)n, ms, n / ms / 1e6);
    hipMemset(tab, 0xFF, entries * 16);
    hipDeviceSynchronize();
    auto timed = [&](const char* what, auto launch) {
        hipEventRecord(a);
        launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        printf("%-9s %lld random ops                          %8.3f ms  %.2f G/s\n", what, (long long)n, ms, n / ms / 1e6);
    };
    timed("k_cas", [&] { hipLaunchKernelGGL(k_cas, dim3(grid), dim3(nt), 0, 0, tab, entries - 1, n, sink); });
    timed("k_st", [&] { hipLaunchKernelGGL(k_st, dim3(grid), dim3(nt), 0, 0, tab, entries - 1, n); });
    timed("k_insert", [&] { hipLaunchKernelGGL(k_insert, dim3(grid), dim3(nt), 0, 0, tab, entries - 1, n, sink); });
    timed("k_amin", [&] { hipLaunchKernelGGL(k_amin, dim3(grid), dim3(nt), 0, 0, tab, entries - 1, n, sink); });
    return 0;

}
