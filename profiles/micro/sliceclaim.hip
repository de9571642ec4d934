// A/B of where the visited-set claims land (diagnostic, round 2; VERDICT r1 "attack k_expand's
// random-touch bound"): k_expand claims every raw child straight from the block that owns its parent
// (random lines of a 32 GiB table; the answer goes to LDS).  The alternative partitions the children by
// the slot's high bits into 128 slices (256 MiB of table each, the Infinity Cache's size), claims slice by
// slice (the table lines a slice touches are cache-resident), and sends the answers back to the parents'
// candidate masks (a random 8-B atomicOr into 96 MB per surviving child).
//   sliceclaim <children_millions> <distinct_millions> [answers 0/1]   (-DSLICE_SHIFT=23: 256 slices)
// Both variants run the same claim (tag-first probe_insert restated, first occurrence = smallest tag) on
// the same children.  rocprofv3 --pmc passes give FETCH/WRITE/TCC per kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

struct alignas(16) Entry {
    unsigned long long key, tag;
};
constexpr unsigned long long EMPTY = ~0ull;
#ifndef SLICE_SHIFT
#define SLICE_SHIFT 24   // 2^31 slots / 2^7 slices = 2^24 slots (256 MiB) per slice; 23: 256 slices of 128 MiB
#endif
constexpr int NSL = 1 << (31 - SLICE_SHIFT);

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
__device__ __forceinline__ uint64_t child_key(uint64_t i, uint64_t distinct) { return mix(mix(i * 0x9E3779B97F4A7C15ull) % distinct + 1); }

// claim: 1 = inserted, 0 = this child holds the key (a larger same-turn tag displaced), -1 = lost
__device__ int claim(Entry* tab, uint64_t mask, uint64_t key, uint64_t tag) {
    uint64_t h = mix(key) & mask;
    for (int probe = 0; probe < 4096; probe++) {
        const ulonglong2 e = *reinterpret_cast<const ulonglong2*>(&tab[h]);
        unsigned long long k = e.x, tg = e.y;
        if (tg == EMPTY) {
            const unsigned long long prev = atomicCAS(&tab[h].tag, EMPTY, (unsigned long long)tag);
            if (prev == EMPTY) {
                __hip_atomic_store(&tab[h].key, (unsigned long long)key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return 1;
            }
            tg = prev;
        }
        if (k == EMPTY) k = __hip_atomic_load(&tab[h].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == EMPTY) continue;   // key store in flight: read again
        if (k == key) {
            if (tg < tag) return -1;
            const unsigned long long old = atomicMin(&tab[h].tag, (unsigned long long)tag);
            return old < tag ? -1 : 0;
        }
        h = (h + 1) & mask;
    }
    return -1;
}

// A: claims in child order (as k_expand hands out parent groups), answer counted (LDS in k_expand)
__global__ void k_direct(Entry* tab, uint64_t mask, int64_t n, uint64_t distinct, unsigned long long* won) {
    uint32_t c = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        c += claim(tab, mask, child_key(i, distinct), (uint64_t)i) >= 0;
    atomicAdd(won, (unsigned long long)c);
}
// B1: children -> slices: per-block LDS counts, one global atomic per (block, slice) for the count and
// one per (block, slice) to reserve the block's range at scatter time (order inside a slice is free:
// the tag decides)
__global__ void k_slice_count(uint64_t mask, int64_t n, uint64_t distinct, unsigned int* cnt) {
    __shared__ unsigned int c[NSL];
    for (int t = threadIdx.x; t < NSL; t += blockDim.x) c[t] = 0;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&c[(mix(child_key(i, distinct)) & mask) >> SLICE_SHIFT], 1u);
    __syncthreads();
    for (int t = threadIdx.x; t < NSL; t += blockDim.x)
        if (c[t]) atomicAdd(&cnt[t], c[t]);
}
__global__ void k_slice_scatter(uint64_t mask, int64_t n, uint64_t distinct, unsigned int* cur, ulonglong2* rec) {
    __shared__ unsigned int c[NSL], base[NSL];
    const int64_t per = (n + gridDim.x - 1) / gridDim.x, lo = blockIdx.x * per, hi = lo + per < n ? lo + per : n;
    for (int t = threadIdx.x; t < NSL; t += blockDim.x) c[t] = 0;
    __syncthreads();
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) atomicAdd(&c[(mix(child_key(i, distinct)) & mask) >> SLICE_SHIFT], 1u);
    __syncthreads();
    for (int t = threadIdx.x; t < NSL; t += blockDim.x) {
        base[t] = c[t] ? atomicAdd(&cur[t], c[t]) : 0;
        c[t] = 0;
    }
    __syncthreads();
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        const uint64_t k = child_key(i, distinct);
        const unsigned int s = (unsigned int)((mix(k) & mask) >> SLICE_SHIFT);
        rec[base[s] + atomicAdd(&c[s], 1u)] = make_ulonglong2(k, (unsigned long long)i);
    }
}
// B2: claims slice after slice (records grouped by slice; the grid sweeps them in order)
__global__ void k_slice_claim(Entry* tab, uint64_t mask, int64_t n, const ulonglong2* rec, unsigned long long* cand,
                              int answers) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const ulonglong2 r = rec[i];
        if (claim(tab, mask, r.x, r.y) >= 0 && answers) {   // B3: the answer back to the parent's candidate mask
            const uint64_t parent = r.y / 24, bit = r.y % 24 * 8;   // ~24 children per parent, 192-bit masks
            atomicOr(&cand[parent * 3 + (bit >> 6)], 1ull << (bit & 63));
        }
    }
}

int main(int argc, char** argv) {
    const int64_t n = (int64_t)((argc > 1 ? atof(argv[1]) : 96) * 1e6);
    const uint64_t distinct = (uint64_t)((argc > 2 ? atof(argv[2]) : 40) * 1e6);
    const uint64_t slots = 1ull << 31, mask = slots - 1;
    Entry* tab;
    ulonglong2* rec;
    unsigned int *cnt, *cur;
    unsigned long long *cand, *won;
    if (hipMalloc(&tab, slots * sizeof(Entry)) != hipSuccess || hipMalloc(&rec, n * 16) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    const int64_t parents = n / 24 + 1;
    hipMalloc(&cand, parents * 24);
    hipMalloc(&cnt, NSL * 4);
    hipMalloc(&cur, NSL * 4);
    const int answers = argc > 3 ? atoi(argv[3]) : 1;
    hipMalloc(&won, 8);
    hipEvent_t ev[6];
    for (auto& e : ev) hipEventCreate(&e);
    const int grid = 256 * 16, nt = 256;
    float best_a = 1e9, best_b[3] = {1e9, 1e9, 1e9};
    unsigned long long wa = 0;
    for (int rep = 0; rep < 3; rep++) {
        hipMemset(tab, 0xFF, slots * sizeof(Entry));
        hipMemset(won, 0, 8);
        hipEventRecord(ev[0]);
        hipLaunchKernelGGL(k_direct, dim3(grid), dim3(nt), 0, 0, tab, mask, n, distinct, won);
        hipEventRecord(ev[1]);
        hipEventSynchronize(ev[1]);
        float ms;
        hipEventElapsedTime(&ms, ev[0], ev[1]);
        best_a = ms < best_a ? ms : best_a;
        hipMemcpy(&wa, won, 8, hipMemcpyDeviceToHost);

        hipMemset(tab, 0xFF, slots * sizeof(Entry));
        hipMemset(cnt, 0, NSL * 4);
        hipMemset(cand, 0, parents * 24);
        hipEventRecord(ev[2]);
        hipLaunchKernelGGL(k_slice_count, dim3(grid), dim3(nt), 0, 0, mask, n, distinct, cnt);
        std::vector<unsigned int> h(NSL), s(NSL);
        hipMemcpy(h.data(), cnt, NSL * 4, hipMemcpyDeviceToHost);
        unsigned int acc = 0;
        for (int i = 0; i < NSL; i++) {
            s[i] = acc;
            acc += h[i];
        }
        hipMemcpy(cur, s.data(), NSL * 4, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_slice_scatter, dim3(grid), dim3(nt), 0, 0, mask, n, distinct, cur, rec);
        hipEventRecord(ev[3]);
        hipLaunchKernelGGL(k_slice_claim, dim3(grid), dim3(nt), 0, 0, tab, mask, n, rec, cand, answers);
        hipEventRecord(ev[4]);
        hipEventSynchronize(ev[4]);
        float p, c;
        hipEventElapsedTime(&p, ev[2], ev[3]);
        hipEventElapsedTime(&c, ev[3], ev[4]);
        if (p + c < best_b[0] + best_b[1]) {
            best_b[0] = p;
            best_b[1] = c;
        }
    }
    printf("children %lld distinct %llu table 32 GiB (2^31 slots), %d slices of %d MiB, answers %s\n", (long long)n,
           (unsigned long long)distinct, NSL, 1 << (SLICE_SHIFT + 4 - 20), answers ? "on" : "off (timing only)");
    printf("A direct claims (k_expand's pattern)          %8.3f ms   winners %llu\n", best_a, wa);
    printf("B partition into slices (count+scatter)       %8.3f ms\n", best_b[0]);
    printf("B slice-ordered claims + answers to the masks %8.3f ms\n", best_b[1]);
    printf("B total                                       %8.3f ms\n", best_b[0] + best_b[1]);
    return 0;
}
