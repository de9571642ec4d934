// Cost of the visited-set insertion forms on MI355X (diagnostic for k_expand's claim).
//   claimcost <table_GiB> <n_millions>
// Each form runs on a freshly emptied table (all 0xFF) over n random slots of 16-B entries {key, tag}:
//   cas            CAS key EMPTY -> k                                  (1 atomic)
//   cas+amin       CAS key, then atomicMin tag once the CAS returned    (2 atomics, same line)
//   cas+amin_nr    CAS key and a no-return atomicMin issued together
//   cas+st_sc1     CAS key, then a write-through (sc1) 8-B store of tag
//   cas+st         CAS key, then a plain 8-B store of tag
//   st_sc1 / st    8-B stores alone; amin alone
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
#define LOOP for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)

__global__ void k_cas(ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    LOOP acc += atomicCAS(&tab[mix(i) & mask].x, ~0ull, (unsigned long long)i);
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_cas_amin(ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    LOOP {
        const uint64_t h = mix(i) & mask;
        const uint64_t p = atomicCAS(&tab[h].x, ~0ull, (unsigned long long)i);
        if (p == ~0ull) acc += atomicMin(&tab[h].y, (unsigned long long)i);
    }
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_cas_amin_nr(ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    LOOP {
        const uint64_t h = mix(i) & mask;
        acc += atomicCAS(&tab[h].x, ~0ull, (unsigned long long)i);
        __hip_atomic_fetch_min(&tab[h].y, (unsigned long long)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_cas_st1(ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    LOOP {
        const uint64_t h = mix(i) & mask;
        const uint64_t p = atomicCAS(&tab[h].x, ~0ull, (unsigned long long)i);
        if (p == ~0ull) __hip_atomic_store(&tab[h].y, (unsigned long long)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        acc += p;
    }
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_cas_st(ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    LOOP {
        const uint64_t h = mix(i) & mask;
        const uint64_t p = atomicCAS(&tab[h].x, ~0ull, (unsigned long long)i);
        if (p == ~0ull) tab[h].y = i;
        acc += p;
    }
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_st1(ulonglong2* tab, uint64_t mask, int64_t n) {
    LOOP __hip_atomic_store(&tab[mix(i) & mask].y, (unsigned long long)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void k_st(ulonglong2* tab, uint64_t mask, int64_t n) {
    LOOP tab[mix(i) & mask].y = i;
}
__global__ void k_st16(ulonglong2* tab, uint64_t mask, int64_t n) {
    LOOP tab[mix(i) & mask] = make_ulonglong2(i, i);
}
__global__ void k_amin(ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    LOOP acc += atomicMin(&tab[mix(i) & mask].y, (unsigned long long)i);
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_load(const ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    LOOP {
        const ulonglong2 e = tab[mix(i) & mask];
        acc += e.x ^ e.y;
    }
    if (acc == 42) atomicAdd(sink, acc);
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 32;
    const int64_t n = (int64_t)((argc > 2 ? atof(argv[2]) : 50) * 1e6);
    uint64_t entries = 1;
    while ((double)entries * 32 <= gib * (1ull << 30)) entries <<= 1;
    ulonglong2* tab;
    unsigned long long* sink;
    if (hipMalloc(&tab, entries * 16) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMalloc(&sink, 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grid = 256 * 32, nt = 256;
    const uint64_t mask = entries - 1;
    auto run = [&](const char* name, auto launch) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            hipMemset(tab, 0xFF, entries * 16);
            hipDeviceSynchronize();
            hipEventRecord(a);
            launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
        }
        printf("%-12s table %6.2f GiB  n %lld  %8.3f ms  %7.2f G ops/s\n", name, entries * 16.0 / (1 << 30),
               (long long)n, best, n / best / 1e6);
    };
    run("load16", [&] { hipLaunchKernelGGL(k_load, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); });
    run("cas", [&] { hipLaunchKernelGGL(k_cas, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); });
    run("amin", [&] { hipLaunchKernelGGL(k_amin, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); });
    run("cas+amin", [&] { hipLaunchKernelGGL(k_cas_amin, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); });
    run("cas+amin_nr", [&] { hipLaunchKernelGGL(k_cas_amin_nr, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); });
    run("cas+st_sc1", [&] { hipLaunchKernelGGL(k_cas_st1, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); });
    run("cas+st", [&] { hipLaunchKernelGGL(k_cas_st, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); });
    run("st_sc1", [&] { hipLaunchKernelGGL(k_st1, dim3(grid), dim3(nt), 0, 0, tab, mask, n); });
    run("st", [&] { hipLaunchKernelGGL(k_st, dim3(grid), dim3(nt), 0, 0, tab, mask, n); });
    run("st16", [&] { hipLaunchKernelGGL(k_st16, dim3(grid), dim3(nt), 0, 0, tab, mask, n); });
    return 0;
}
