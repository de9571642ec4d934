// sb_mt.hip — the randint(1,100) noise stream of the heuristics, on the device.
//
// The reference draws one `randint(1, 100)` per scored state (src/solver.py:215,247,260,284),
// in next_queue order (the order sorted() calls its key).  CPython implements it as MT19937
// words w with rejection: value = 1 + (w >> 25), redrawing while (w >> 25) >= 100.  The stream is
// data-independent, so the engine produces it ahead of use:
//   k_mt_gen      one workgroup runs the MT19937 twist (3 dependent phases of <= 227 words) and
//                 writes tempered words;
//   k_mt_count/k_mt_write   order-preserving compaction of accepted draws into a ring of u8
//                 values, so next_queue element k reads ring[(consumed + k) & mask].
#include <string.h>

#include "sb_block.h"
#include "sb_internal.h"

namespace sb {

constexpr uint32_t MT_UPPER = 0x80000000u, MT_LOWER = 0x7fffffffu, MT_A = 0x9908b0dfu;

__host__ __device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}
__host__ __device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t m) {
    uint32_t y = (a & MT_UPPER) | (b & MT_LOWER);
    return m ^ (y >> 1) ^ ((y & 1u) ? MT_A : 0u);
}

uint32_t HostMT::next() {
    if (idx >= 624) {
        int kk;
        for (kk = 0; kk < 624 - 397; kk++) mt[kk] = mt_mix(mt[kk], mt[kk + 1], mt[kk + 397]);
        for (; kk < 623; kk++) mt[kk] = mt_mix(mt[kk], mt[kk + 1], mt[kk - 227]);
        mt[623] = mt_mix(mt[623], mt[0], mt[396]);
        idx = 0;
    }
    return mt_temper(mt[idx++]);
}

// One workgroup of 640 threads; state in LDS ping-pong buffers; ntw twists.
__global__ __launch_bounds__(640) void k_mt_gen(uint32_t* __restrict__ state, uint32_t* __restrict__ out, int64_t ntw) {
    __shared__ uint32_t buf[2][624];
    const int t = threadIdx.x;
    if (t < 624) buf[0][t] = state[t];
    __syncthreads();
    int cur = 0;
    for (int64_t w = 0; w < ntw; w++) {
        uint32_t* A = buf[cur];
        uint32_t* B = buf[cur ^ 1];
        if (t < 227) B[t] = mt_mix(A[t], A[t + 1], A[t + 397]);                    // new[i], i < 227
        __syncthreads();
        if (t < 227) B[227 + t] = mt_mix(A[227 + t], A[228 + t], B[t]);          // i in [227, 454)
        __syncthreads();
        if (t < 169) B[454 + t] = mt_mix(A[454 + t], A[455 + t], B[227 + t]);   // i in [454, 623)
        else if (t == 169) B[623] = mt_mix(A[623], B[0], B[396]);               // i = 623
        __syncthreads();
        if (t < 624) out[w * 624 + t] = mt_temper(B[t]);
        cur ^= 1;
    }
    if (t < 624) state[t] = buf[cur][t];
}

constexpr int MT_NT = 256;
constexpr int MT_IPT = 16;
constexpr int MT_TILE = MT_NT * MT_IPT;

__global__ __launch_bounds__(MT_NT) void k_mt_count(const uint32_t* __restrict__ w, int64_t n, uint32_t* __restrict__ tiles) {
    __shared__ uint32_t lds[MT_NT / 64 + 1];
    const int64_t base = (int64_t)blockIdx.x * MT_TILE;
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < MT_IPT; j++) {
        int64_t i = base + (int64_t)j * MT_NT + threadIdx.x;
        if (i < n) c += (w[i] >> 25) < 100u;
    }
    uint32_t tot;
    block_excl_scan<MT_NT>(c, lds, &tot);
    if (threadIdx.x == 0) tiles[blockIdx.x] = tot;
}

__global__ __launch_bounds__(MT_NT) void k_mt_write(const uint32_t* __restrict__ w, int64_t n,
                                                     const uint32_t* __restrict__ tiles, uint8_t* __restrict__ ring,
                                                     uint64_t ring_mask, uint64_t produced) {
    __shared__ uint32_t lds[MT_NT / 64 + 1];
    const int64_t base = (int64_t)blockIdx.x * MT_TILE + (int64_t)threadIdx.x * MT_IPT;   // blocked order
    uint32_t v[MT_IPT];
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < MT_IPT; j++) {
        int64_t i = base + j;
        v[j] = i < n ? (w[i] >> 25) : 200u;
        c += v[j] < 100u;
    }
    uint32_t tot;
    uint64_t pos = produced + tiles[blockIdx.x] + block_excl_scan<MT_NT>(c, lds, &tot);
#pragma unroll
    for (int j = 0; j < MT_IPT; j++) {
        if (v[j] < 100u) {
            ring[pos & ring_mask] = (uint8_t)(v[j] + 1);
            pos++;
        }
    }
}

void noise_init(NoiseStream& ns, const uint32_t* state625, uint64_t ring_cap_pow2, hipStream_t st) {
    memcpy(ns.initial.mt, state625, 624 * 4);
    ns.initial.idx = (int)state625[624];
    ns.replay = ns.initial;
    ns.replay_draws = 0;
    ns.produced = 0;
    ns.consumed = 0;
    ns.ring.ensure(ring_cap_pow2);
    ns.ring_mask = ring_cap_pow2 - 1;
    SB_HIP(hipMalloc((void**)&ns.d_state, 624 * 4));
    SB_HIP(hipMalloc((void**)&ns.d_total, 16));
    SB_HIP(hipHostMalloc((void**)&ns.h_total, 16, hipHostMallocDefault));
    SB_HIP(hipEventCreateWithFlags(&ns.ev_ready, hipEventDisableTiming));
    // the host emits the partially consumed block (words idx..623) so the device always starts
    // with a twist; those words go through the same compaction
    HostMT h = ns.initial;
    uint32_t lead[624];
    int nlead = 0;
    while (h.idx < 624) lead[nlead++] = h.next();
    SB_HIP(hipMemcpyAsync(ns.d_state, h.mt, 624 * 4, hipMemcpyHostToDevice, st));
    if (nlead) {
        ns.raw.ensure(624);
        SB_HIP(hipMemcpyAsync(ns.raw.p, lead, nlead * 4, hipMemcpyHostToDevice, st));
        int64_t nt = (nlead + MT_TILE - 1) / MT_TILE;
        ns.scan.tiles.ensure(nt);
        hipLaunchKernelGGL(k_mt_count, dim3((unsigned)nt), dim3(MT_NT), 0, st, ns.raw.p, (int64_t)nlead, ns.scan.tiles.p);
        scan_tiles_inplace(ns.scan.tiles.p, nt, ns.d_total, st);
        hipLaunchKernelGGL(k_mt_write, dim3((unsigned)nt), dim3(MT_NT), 0, st, ns.raw.p, (int64_t)nlead, ns.scan.tiles.p,
                           ns.ring.p, ns.ring_mask, (uint64_t)0);
        SB_HIP(hipMemcpyAsync(ns.h_total, ns.d_total, 4, hipMemcpyDeviceToHost, st));
        SB_HIP(hipStreamSynchronize(st));
        ns.produced += *ns.h_total;
    }
}

void noise_generate_async(NoiseStream& ns, uint64_t words, hipStream_t st) {
    if (ns.pending) return;
    uint64_t room = ns.ring_mask + 1 - (ns.produced - ns.consumed);
    // never let unconsumed values overrun the ring: accepted draws <= words generated
    if (words > room) words = room;
    int64_t ntw = (int64_t)(words / 624);
    if (ntw <= 0) return;
    int64_t n = ntw * 624;
    ns.raw.ensure((size_t)n);
    hipLaunchKernelGGL(k_mt_gen, dim3(1), dim3(640), 0, st, ns.d_state, ns.raw.p, ntw);
    int64_t nt = (n + MT_TILE - 1) / MT_TILE;
    ns.scan.tiles.ensure(nt);
    hipLaunchKernelGGL(k_mt_count, dim3((unsigned)nt), dim3(MT_NT), 0, st, ns.raw.p, n, ns.scan.tiles.p);
    scan_tiles_inplace(ns.scan.tiles.p, nt, ns.d_total, st);
    hipLaunchKernelGGL(k_mt_write, dim3((unsigned)nt), dim3(MT_NT), 0, st, ns.raw.p, n, ns.scan.tiles.p, ns.ring.p,
                       ns.ring_mask, ns.produced);
    SB_HIP(hipMemcpyAsync(ns.h_total, ns.d_total, 4, hipMemcpyDeviceToHost, st));
    SB_HIP(hipEventRecord(ns.ev_ready, st));
    SB_HIP(hipGetLastError());
    ns.pending = true;
    ns.pending_words = (uint64_t)n;
}

static void noise_collect(NoiseStream& ns) {
    if (!ns.pending) return;
    SB_HIP(hipEventSynchronize(ns.ev_ready));
    ns.produced += *ns.h_total;
    ns.pending = false;
}

void noise_ensure(NoiseStream& ns, uint64_t need, hipStream_t st) {
    noise_collect(ns);
    while (ns.produced - ns.consumed < need) {
        uint64_t deficit = need - (ns.produced - ns.consumed);
        if (deficit > ns.ring_mask + 1) throw HipError{hipErrorOutOfMemory, "noise ring too small for one step"};
        uint64_t words = deficit * 128 / 100 + 8192;
        noise_generate_async(ns, words, st);
        if (!ns.pending) throw HipError{hipErrorOutOfMemory, "noise ring full"};
        noise_collect(ns);
    }
}

void noise_mt_state(NoiseStream& ns, uint32_t* out625) {
    // replay on the host from the last cursor: draws consumed so far
    while (ns.replay_draws < ns.consumed) {
        while ((ns.replay.next() >> 25) >= 100u) {
        }
        ns.replay_draws++;
    }
    memcpy(out625, ns.replay.mt, 624 * 4);
    out625[624] = (uint32_t)ns.replay.idx;
}

void noise_free(NoiseStream& ns) {
    if (ns.d_state) (void)hipFree(ns.d_state);
    if (ns.d_total) (void)hipFree(ns.d_total);
    if (ns.h_total) (void)hipHostFree(ns.h_total);
    if (ns.ev_ready) (void)hipEventDestroy(ns.ev_ready);
    ns.raw.release();
    ns.ring.release();
    ns.scan.tiles.release();
    ns.d_state = nullptr;
    ns.d_total = nullptr;
    ns.h_total = nullptr;
    ns.ev_ready = nullptr;
}

void mt_debug_words(const uint32_t* state625, int64_t n, uint32_t* out) {
    HostMT h;
    memcpy(h.mt, state625, 624 * 4);
    h.idx = (int)state625[624];
    int64_t k = 0;
    while (h.idx < 624 && k < n) out[k++] = h.next();
    if (k == n) return;
    int64_t ntw = (n - k + 623) / 624;
    uint32_t* ds = nullptr;
    uint32_t* dout = nullptr;
    SB_HIP(hipMalloc((void**)&ds, 624 * 4));
    SB_HIP(hipMalloc((void**)&dout, (size_t)ntw * 624 * 4));
    SB_HIP(hipMemcpy(ds, h.mt, 624 * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_mt_gen, dim3(1), dim3(640), 0, 0, ds, dout, ntw);
    SB_HIP(hipGetLastError());
    SB_HIP(hipMemcpy(out + k, dout, (size_t)(n - k) * 4, hipMemcpyDeviceToHost));
    (void)hipFree(ds);
    (void)hipFree(dout);
}

}  // namespace sb
