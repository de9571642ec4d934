// Random-access throughput of MI355X HBM for the visited-set access pattern (diagnostic).
//   randaccess <table_GiB> <n_millions>
// reports: 16-B random loads, 8-B random atomicMin (returning), load+atomic on the same line.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
__global__ void k_load(const ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const ulonglong2 e = tab[mix(i) & mask];
        acc += e.x ^ e.y;
    }
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_amin(ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        acc += atomicMin(&tab[mix(i) & mask].y, (unsigned long long)i);
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_load_amin(ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t h = mix(i) & mask;
        const ulonglong2 e = tab[h];
        if (e.y > (uint64_t)i) acc += atomicMin(&tab[h].y, (unsigned long long)i);
        acc += e.x;
    }
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_amin_nr(ulonglong2* tab, uint64_t mask, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        __hip_atomic_fetch_min(&tab[mix(i) & mask].y, (unsigned long long)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void k_cas(ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        acc += atomicCAS(&tab[mix(i) & mask].x, ~0ull, (unsigned long long)i);
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_amin32(ulonglong2* tab, uint64_t mask, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        acc += atomicMin((unsigned int*)&tab[mix(i) & mask].y, (unsigned int)i);
    if (acc == 42) atomicAdd(sink, acc);
}
__global__ void k_stream(const ulonglong2* tab, int64_t n, unsigned long long* sink) {
    uint64_t acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const ulonglong2 e = tab[i];
        acc += e.x ^ e.y;
    }
    if (acc == 42) atomicAdd(sink, acc);
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 32;
    const int64_t n = (int64_t)((argc > 2 ? atof(argv[2]) : 100) * 1e6);
    uint64_t entries = 1;
    while ((double)entries * 32 <= gib * (1ull << 30)) entries <<= 1;   // entries * 16 B <= gib
    ulonglong2* tab;
    unsigned long long* sink;
    if (hipMalloc(&tab, entries * 16) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMalloc(&sink, 8);
    hipMemset(tab, 0xFF, entries * 16);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grid = 256 * 32, nt = 256;
    auto run = [&](const char* name, auto launch, double bytes_per) {
        launch();
        hipEventRecord(a);
        launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        printf("%-12s table %6.2f GiB  n %lld  %8.3f ms  %7.2f G acc/s  (x%g B = %7.1f GB/s)\n", name,
               entries * 16.0 / (1 << 30), (long long)n, ms, n / ms / 1e6, bytes_per, n * bytes_per / ms / 1e6);
    };
    const uint64_t mask = entries - 1;
    run("load16", [&] { hipLaunchKernelGGL(k_load, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); }, 128);
    run("amin8", [&] { hipLaunchKernelGGL(k_amin, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); }, 128);
    run("load+amin", [&] { hipLaunchKernelGGL(k_load_amin, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); }, 128);
    run("amin8_nr", [&] { hipLaunchKernelGGL(k_amin_nr, dim3(grid), dim3(nt), 0, 0, tab, mask, n); }, 128);
    run("cas8", [&] { hipLaunchKernelGGL(k_cas, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); }, 128);
    run("amin4", [&] { hipLaunchKernelGGL(k_amin32, dim3(grid), dim3(nt), 0, 0, tab, mask, n, sink); }, 128);
    const int64_t ns = (int64_t)(entries < (uint64_t)n * 4 ? entries : (uint64_t)n * 4);
    run("stream16", [&] { hipLaunchKernelGGL(k_stream, dim3(grid), dim3(nt), 0, 0, tab, ns, sink); }, 16.0 * ns / n);
    return 0;
}
