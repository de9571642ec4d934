// Claim-protocol variants on a synthetic turn with k_expand's dedup structure (diagnostic).
//   claimproto [n_children_M=96] [distinct_pool_M=50] [filler_M=400]
// Child i has key id mix(i) % pool (≈46% same-turn duplicates at the defaults); ids below 3% of the
// pool were inserted by an "earlier turn"; `filler` further old keys set the table's load.  Every
// variant computes, per child, "first occurrence in index order and not old" — checked against V0.
//   V0  16-B {key, tag}: probe load, CAS key, atomicMin tag, displaced holder marked lost   (current)
//   V2  8-B packed {remainder | tag} in 16-slot buckets (one 128-B line): probe load, one CAS per
//       insert or displacement, displaced holder marked lost                                (1 atomic)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define EMPTY (~0ull)
__device__ __host__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
__device__ __forceinline__ uint64_t child_key(int64_t i, uint64_t pool) { return mix(0x1234567ull + mix((uint64_t)i) % pool); }

// ---------------- V0
__global__ void v0_fill(ulonglong2* tab, uint64_t mask, int64_t n, uint64_t pool, uint64_t nold) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t key = i < (int64_t)nold ? mix(0x1234567ull + (uint64_t)i) : mix(0xABCDEF0000000ull + (uint64_t)i);
        uint64_t h = mix(key) & mask;
        while (true) {
            const uint64_t p = atomicCAS(&tab[h].x, EMPTY, key);
            if (p == EMPTY || p == key) break;
            h = (h + 1) & mask;
        }
        tab[h].y = 0;
    }
}
__global__ void v0_claim(ulonglong2* tab, uint64_t mask, int64_t n, uint64_t pool, uint64_t turn,
                         unsigned long long* cand, unsigned long long* lost) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t key = child_key(i, pool), tag = turn | (uint64_t)i;
        uint64_t h = mix(key) & mask, cur;
        ulonglong2 ent = tab[h];
        while (true) {
            if (ent.x == EMPTY) {
                const uint64_t p = atomicCAS(&tab[h].x, EMPTY, key);
                if (p == EMPTY) { cur = EMPTY; break; }
                if (p == key) { cur = tab[h].y; break; }
                ent.x = p;
            }
            if (ent.x == key) { cur = ent.y; break; }
            h = (h + 1) & mask;
            ent = tab[h];
        }
        if (cur != EMPTY && cur < tag) continue;
        const uint64_t old = atomicMin(&tab[h].y, tag);
        if (old < tag) continue;
        if (old != EMPTY) {
            const uint64_t j = old & 0xFFFFFFFFFFull;
            atomicOr(&lost[j >> 6], 1ull << (j & 63));
        }
        atomicOr(&cand[i >> 6], 1ull << (i & 63));
    }
}

// ---------------- V2: B-bit bucket index, remainder 64-B bits, tag B bits (tag 0 = old)
constexpr int BB = 28;
constexpr uint64_t TAGM = (1ull << BB) - 1;
__device__ __forceinline__ void v2_split(uint64_t key, uint64_t* bucket, uint64_t* rem) {
    const uint64_t f = mix(key);
    *bucket = f >> (64 - BB);
    *rem = f & ((1ull << (64 - BB)) - 1);
}
__global__ void v2_fill(uint64_t* tab, int64_t n, uint64_t nold) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t key = i < (int64_t)nold ? mix(0x1234567ull + (uint64_t)i) : mix(0xABCDEF0000000ull + (uint64_t)i);
        uint64_t b, r;
        v2_split(key, &b, &r);
        const uint64_t w = r << BB;   // tag 0: old
        uint64_t* line = tab + b * 16;
        int s = (int)(r & 15);
        for (int k = 0; k < 16; k++, s = (s + 1) & 15) {
            const uint64_t p = atomicCAS(&line[s], EMPTY, w);
            if (p == EMPTY || (p >> BB) == r) break;
        }
    }
}
__global__ void v2_claim(uint64_t* tab, int64_t n, uint64_t pool, unsigned long long* cand, unsigned long long* lost,
                         unsigned* err) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t key = child_key(i, pool), tag = (uint64_t)i + 1;
        uint64_t b, r;
        v2_split(key, &b, &r);
        uint64_t* line = tab + b * 16;
        const uint64_t mine = (r << BB) | tag;
        int s = (int)(r & 15), k = 0;
        uint64_t w = line[s];
        bool won = false;
        while (true) {
            if (w == EMPTY) {
                const uint64_t p = atomicCAS(&line[s], EMPTY, mine);
                if (p == EMPTY) { won = true; break; }
                w = p;
                continue;
            }
            if ((w >> BB) != r) {
                if (++k == 16) { atomicOr(err, 1u); break; }
                s = (s + 1) & 15;
                w = line[s];
                continue;
            }
            if (w <= mine) break;   // old (tag 0) or an earlier claimant
            const uint64_t p = atomicCAS(&line[s], w, mine);
            if (p == w) {
                const uint64_t j = (w & TAGM) - 1;
                atomicOr(&lost[j >> 6], 1ull << (j & 63));
                won = true;
                break;
            }
            w = p;
        }
        if (won) atomicOr(&cand[i >> 6], 1ull << (i & 63));
    }
}

__global__ void k_survivors(const unsigned long long* cand, const unsigned long long* lost, int64_t nw,
                            unsigned long long* out, unsigned long long* cnt) {
    unsigned long long c = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nw; i += (int64_t)gridDim.x * blockDim.x) {
        out[i] = cand[i] & ~lost[i];
        c += __popcll(out[i]);
    }
    atomicAdd(cnt, c);
}

int main(int argc, char** argv) {
    const int64_t n = (int64_t)((argc > 1 ? atof(argv[1]) : 96) * 1e6);
    const uint64_t pool = (uint64_t)((argc > 2 ? atof(argv[2]) : 50) * 1e6);
    const int64_t filler = (int64_t)((argc > 3 ? atof(argv[3]) : 400) * 1e6);
    const uint64_t nold = pool * 3 / 100;
    const uint64_t bytes = 32ull << 30;
    void* tabv;
    if (hipMalloc(&tabv, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
    const int64_t nw = (n + 63) / 64;
    unsigned long long *cand, *lost, *s0, *s2, *cnt;
    unsigned* err;
    hipMalloc(&cand, nw * 8); hipMalloc(&lost, nw * 8); hipMalloc(&s0, nw * 8); hipMalloc(&s2, nw * 8);
    hipMalloc(&cnt, 16); hipMalloc(&err, 4);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const int grid = 256 * 32, nt = 256;
    float ms;
    unsigned long long hc[2];
    unsigned herr;
    for (int rep = 0; rep < 2; rep++) {
        // V0
        hipMemset(tabv, 0xFF, bytes);
        hipLaunchKernelGGL(v0_fill, dim3(grid), dim3(nt), 0, 0, (ulonglong2*)tabv, (bytes / 16) - 1, (int64_t)(nold + filler), pool, nold);
        hipMemset(cand, 0, nw * 8); hipMemset(lost, 0, nw * 8); hipMemset(cnt, 0, 16);
        hipDeviceSynchronize();
        hipEventRecord(a);
        hipLaunchKernelGGL(v0_claim, dim3(grid), dim3(nt), 0, 0, (ulonglong2*)tabv, (bytes / 16) - 1, n, pool, 1ull << 40, cand, lost);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        hipLaunchKernelGGL(k_survivors, dim3(1024), dim3(256), 0, 0, cand, lost, nw, s0, cnt);
        hipMemcpy(hc, cnt, 8, hipMemcpyDeviceToHost);
        printf("V0 16-B cas+amin     %8.3f ms  survivors %llu\n", ms, hc[0]);
        // V2
        hipMemset(tabv, 0xFF, bytes);
        hipLaunchKernelGGL(v2_fill, dim3(grid), dim3(nt), 0, 0, (uint64_t*)tabv, (int64_t)(nold + filler), nold);
        hipMemset(cand, 0, nw * 8); hipMemset(lost, 0, nw * 8); hipMemset(cnt, 0, 16); hipMemset(err, 0, 4);
        hipDeviceSynchronize();
        hipEventRecord(a);
        hipLaunchKernelGGL(v2_claim, dim3(grid), dim3(nt), 0, 0, (uint64_t*)tabv, n, pool, cand, lost, err);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        hipLaunchKernelGGL(k_survivors, dim3(1024), dim3(256), 0, 0, cand, lost, nw, s2, cnt + 1);
        hipMemcpy(hc, cnt, 16, hipMemcpyDeviceToHost);
        hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost);
        // compare masks
        unsigned long long* h0 = (unsigned long long*)malloc(nw * 8);
        unsigned long long* h2 = (unsigned long long*)malloc(nw * 8);
        hipMemcpy(h0, s0, nw * 8, hipMemcpyDeviceToHost);
        hipMemcpy(h2, s2, nw * 8, hipMemcpyDeviceToHost);
        int64_t diff = 0;
        for (int64_t i = 0; i < nw; i++) diff += h0[i] != h2[i];
        free(h0); free(h2);
        printf("V2 8-B packed 1 CAS  %8.3f ms  survivors %llu  err %u  mask words differing from V0: %lld\n", ms, hc[1],
               herr, (long long)diff);
    }
    return 0;
}
