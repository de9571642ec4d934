// Random-access throughput for the visited-set pattern under different allocation / load policies
// (diagnostic, round 2): is a random 16-B probe bound by 128-B line fetches (then an uncached or
// non-temporal access that moves less per request would raise the rate) or by request count?
//   randaccess2 <table_GiB> <n_millions>
// For each allocation (hipMalloc, hipDeviceMallocUncached, hipDeviceMallocFinegrained):
//   load16 / load8 (plain), load16_nt (nontemporal), load16_sc1 (agent-scope relaxed), cas8, cas8+st8
//   (the tag-first insert), two16 (two 16-B loads in one 128-B line per access).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
#define LOOP for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
__global__ void k_load16(const ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    LOOP { const ulonglong2 e = tab[mix(i) & mask]; acc += e.x ^ e.y; }
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_load8(const ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    LOOP { acc += tab[mix(i) & mask].x; }
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_load16_nt(const ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    LOOP {
        const ulonglong2* p = &tab[mix(i) & mask];
        acc += __builtin_nontemporal_load(&p->x) ^ __builtin_nontemporal_load(&p->y);
    }
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_load16_sc1(ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    LOOP {
        ulonglong2* p = &tab[mix(i) & mask];
        acc += __hip_atomic_load(&p->x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_two16(const ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    LOOP {
        const uint64_t h = mix(i) & mask & ~7ull;
        const ulonglong2 a = tab[h], b = tab[h + 4];
        acc += a.x ^ b.y;
    }
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_cas(ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    LOOP { acc += atomicCAS(&tab[mix(i) & mask].y, ~0ull, (unsigned long long)i); }
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_cas_st(ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    LOOP {
        ulonglong2* p = &tab[mix(i) & mask];
        acc += atomicCAS(&p->y, ~0ull, (unsigned long long)i);
        __hip_atomic_store(&p->x, (unsigned long long)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (acc == 42) atomicAdd(sink, acc);
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 32;
    const int64_t n = (int64_t)((argc > 2 ? atof(argv[2]) : 100) * 1e6);
    uint64_t entries = 1;
    while ((double)entries * 32 <= gib * (1ull << 30)) entries <<= 1;
    unsigned long long* sink;
    hipMalloc(&sink, 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grid = 256 * 32, nt = 256;
    const uint64_t mask = entries - 1;
    const char* names[3] = {"hipMalloc", "uncached", "finegrained"};
    for (int mode = 0; mode < 3; mode++) {
        ulonglong2* tab = nullptr;
        hipError_t e = mode == 0 ? hipMalloc(&tab, entries * 16)
                     : hipExtMallocWithFlags((void**)&tab, entries * 16,
                                             mode == 1 ? hipDeviceMallocUncached : hipDeviceMallocFinegrained);
        if (e != hipSuccess) { printf("%s: alloc failed (%s)\n", names[mode], hipGetErrorString(e)); continue; }
        hipMemset(tab, 0xFF, entries * 16);
        hipDeviceSynchronize();
        auto run = [&](const char* name, auto launch) {
            launch();
            hipEventRecord(a);
            launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            printf("%-11s %-11s table %6.2f GiB  n %lld  %8.3f ms  %7.2f G acc/s\n", names[mode], name,
                   entries * 16.0 / (1 << 30), (long long)n, ms, n / ms / 1e6);
            fflush(stdout);
        };
        run("load16", [&] { hipLaunchKernelGGL(k_load16, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); });
        run("load8", [&] { hipLaunchKernelGGL(k_load8, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); });
        run("load16_nt", [&] { hipLaunchKernelGGL(k_load16_nt, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); });
        run("load8_sc1", [&] { hipLaunchKernelGGL(k_load16_sc1, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); });
        run("two16", [&] { hipLaunchKernelGGL(k_two16, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); });
        run("cas8", [&] { hipLaunchKernelGGL(k_cas, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); });
        hipMemset(tab, 0xFF, entries * 16);
        run("cas8+st8", [&] { hipLaunchKernelGGL(k_cas_st, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); });
        hipFree(tab);
    }
    return 0;
}
