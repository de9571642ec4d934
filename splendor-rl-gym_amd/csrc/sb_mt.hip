// sb_mt.hip — the randint(1,100) noise stream of the heuristics, on the device.
//
// The reference draws one `randint(1, 100)` per scored state (src/solver.py:215,247,260,284),
// in next_queue order (the order sorted() calls its key).  CPython implements it as MT19937
// words w with rejection: value = 1 + (w >> 25), redrawing while (w >> 25) >= 100.  The stream is
// data-independent, so the engine produces it ahead of use, in chunks of P*L words:
//   k_mt_gen_par  P producers (one workgroup each, one per CU) run the MT19937 twist (3 dependent
//                 phases of <= 227 words) from their own start window; producer p writes words
//                 [p*L, (p+1)*L) of the chunk;
//   k_mt_jump     advances producer windows by J words: w(n+J)[j] = XOR_{g_i=1} y_{n+1+i+j} with
//                 g = x^(J-1) mod phi (sb_gf2.hip); the sequence y is extended in LDS, the
//                 correlation runs one wave per (64 outputs x poly slice), uniform over poly bits;
//   compaction  each producer writes only its accepted draws (in order) to a staging segment
//               (ballot + wave-count scan per twist); k_mt_place copies the segments into a ring of u8
//               values, so next_queue element k reads ring[(consumed + k) & mask].
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include <vector>

#include "sb_block.h"
#include "sb_gf2.h"
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

// P producers, one workgroup each; producer b runs `twists` twists from window b.  MODE 0 (raw) writes
// the tempered words (debug); MODE 1 (compact) writes only the accepted randint values (1..100) of
// the segment, in order, to stage[b * L ..] and their count to counts[b] (fused accept compaction);
// MODE 2 (count) only counts them; MODE 3 (checkpoint) counts per sub-segment of ck twists and saves
// the window at the start of each sub-segment to out (sharded streams, see noise_shard_chunk).
#ifndef SB_MT_GEN_NT
#define SB_MT_GEN_NT 256   // threads per producer: 4 waves (640: one lane per word; more waves beside k_expand)
#endif
constexpr int MG_NT = SB_MT_GEN_NT;
constexpr int MG_NW = MG_NT / 64;
constexpr int MG_R = (624 + MG_NT - 1) / MG_NT;   // words per thread in the temper / accept phase
static_assert(MG_NT >= 227 && MG_NT % 64 == 0, "one mix phase per pass");
template <int MODE>
__global__ __launch_bounds__(MG_NT) void k_mt_gen_par(const uint32_t* __restrict__ wins, uint32_t* __restrict__ out,
                                                       uint8_t* __restrict__ stage, uint32_t* __restrict__ counts,
                                                       int64_t twists, int ck = 1) {
    constexpr bool RAW = MODE == 0;
    __shared__ uint32_t buf[2][624];
    __shared__ uint32_t wc[MG_R][MG_NW];
    const int t = threadIdx.x, wv = t >> 6, lane = t & 63;
    const int64_t b = blockIdx.x;
    for (int i = t; i < 624; i += MG_NT) buf[0][i] = wins[b * 624 + i];
    __syncthreads();
    uint32_t* o = RAW ? out + b * twists * 624 : nullptr;
    uint8_t* sg = RAW ? nullptr : stage + b * twists * 624;
    uint32_t run = 0;
    int cur = 0;
    const int64_t nsub = MODE == 3 ? twists / ck : 0;
    for (int64_t w = 0; w < twists; w++) {
        uint32_t* A = buf[cur];
        uint32_t* B = buf[cur ^ 1];
        if (MODE == 3 && w % ck == 0) {   // sub-segment boundary: its window, the previous one's count
            for (int i = t; i < 624; i += MG_NT) out[(b * nsub + w / ck) * 624 + i] = A[i];
            if (t == 0 && w > 0) counts[b * nsub + w / ck - 1] = run;
            run = 0;
        }
        if (t < 227) B[t] = mt_mix(A[t], A[t + 1], A[t + 397]);
        __syncthreads();
        if (t < 227) B[227 + t] = mt_mix(A[227 + t], A[228 + t], B[t]);
        __syncthreads();
        if (t < 169) B[454 + t] = mt_mix(A[454 + t], A[455 + t], B[227 + t]);
        else if (t == 169) B[623] = mt_mix(A[623], B[0], B[396]);
        __syncthreads();
        uint32_t y[MG_R];
#pragma unroll
        for (int r = 0; r < MG_R; r++) y[r] = r * MG_NT + t < 624 ? mt_temper(B[r * MG_NT + t]) : 0u;
        if (RAW) {
#pragma unroll
            for (int r = 0; r < MG_R; r++)
                if (r * MG_NT + t < 624) o[w * 624 + r * MG_NT + t] = y[r];
        } else {
            // accepted words in word order: round r (words r*NT + t), then wave, then lane
            uint64_t m[MG_R];
#pragma unroll
            for (int r = 0; r < MG_R; r++) {
                m[r] = __ballot(r * MG_NT + t < 624 && (y[r] >> 25) < 100u);
                if (lane == 0) wc[r][wv] = (uint32_t)__popcll(m[r]);
            }
            __syncthreads();
            uint32_t before = 0;
#pragma unroll
            for (int r = 0; r < MG_R; r++) {
                uint32_t rb = 0, rt = 0;
#pragma unroll
                for (int x = 0; x < MG_NW; x++) {
                    const uint32_t c = wc[r][x];
                    rb += x < wv ? c : 0u;
                    rt += c;
                }
                const bool acc = (m[r] >> lane) & 1;
                if (MODE == 1 && acc) sg[run + before + rb + __popcll(m[r] & lanemask_lt())] = (uint8_t)((y[r] >> 25) + 1);
                before += rt;
            }
            run += before;
        }
        cur ^= 1;
    }
    if (!RAW && t == 0) counts[MODE == 3 ? b * nsub + nsub - 1 : b] = run;
}

// copy each producer's accepted values to the ring at produced + exclusive offset
// grid (P, MT_PLACE_SPLIT): block (b, y) copies slice y of producer b's segment
constexpr int MT_PLACE_SPLIT = 32;
__global__ __launch_bounds__(256) void k_mt_place(const uint8_t* __restrict__ stage, int64_t seg,
                                                  const uint32_t* __restrict__ counts, const uint32_t* __restrict__ offs,
                                                  uint8_t* __restrict__ ring, uint64_t ring_mask, uint64_t produced) {
    const int64_t b = blockIdx.x;
    const uint32_t n = counts[b];
    const uint32_t per = (n + MT_PLACE_SPLIT - 1) / MT_PLACE_SPLIT;
    const uint32_t j0 = blockIdx.y * per, j1 = j0 + per < n ? j0 + per : n;
    const uint64_t base = produced + offs[b];
    const uint8_t* src = stage + b * seg;
    for (uint32_t j = j0 + threadIdx.x; j < j1; j += blockDim.x) ring[(base + j) & ring_mask] = src[j];
}

// Sharded streams: block j regenerates one sub-segment (twists twists) from window j of wins (624
// words each); its first accepted draw has global index seg_acc0[j].  Accepted values with global
// index in [a, b) go to ring[index & ring_mask]; the block stops once past b.
// ranges of accepted-draw indices [a[k], b[k]) this rank emits with, each placed at ring position dst[k] + (idx - a[k])
// (one range at its own index for contiguous slices; block-cyclic slices: a range per block, placed in local order)
__global__ __launch_bounds__(640) void k_mt_fill(const uint32_t* __restrict__ wins, const uint64_t* __restrict__ seg_acc0,
                                                  int64_t twists, const NoiseRanges R, uint8_t* __restrict__ ring,
                                                  uint64_t ring_mask) {
    uint64_t b = 0;
    for (int k = 0; k < R.n; k++) b = R.b[k] > b ? R.b[k] : b;
    __shared__ uint32_t buf[2][624];
    __shared__ uint32_t wc[10];
    const int t = threadIdx.x, wv = t >> 6;
    const uint32_t* win = wins + (int64_t)blockIdx.x * 624;
    if (t < 624) buf[0][t] = win[t];
    __syncthreads();
    uint64_t run = seg_acc0[blockIdx.x];
    int cur = 0;
    for (int64_t w = 0; w < twists && run < b; w++) {
        uint32_t* A = buf[cur];
        uint32_t* B = buf[cur ^ 1];
        if (t < 227) B[t] = mt_mix(A[t], A[t + 1], A[t + 397]);
        __syncthreads();
        if (t < 227) B[227 + t] = mt_mix(A[227 + t], A[228 + t], B[t]);
        __syncthreads();
        if (t < 169) B[454 + t] = mt_mix(A[454 + t], A[455 + t], B[227 + t]);
        else if (t == 169) B[623] = mt_mix(A[623], B[0], B[396]);
        __syncthreads();
        const uint32_t y = t < 624 ? mt_temper(B[t]) : 0u;
        const bool acc = t < 624 && (y >> 25) < 100u;
        const uint64_t m = __ballot(acc);
        if ((t & 63) == 0) wc[wv] = __popcll(m);
        __syncthreads();
        uint32_t before = 0, total = 0;
#pragma unroll
        for (int x = 0; x < 10; x++) {
            const uint32_t c = wc[x];
            before += x < wv ? c : 0u;
            total += c;
        }
        const uint64_t idx = run + before + __popcll(m & lanemask_lt());
        if (acc)
            for (int k = 0; k < R.n; k++)
                if (idx >= R.a[k] && idx < R.b[k]) ring[(R.dst[k] + (idx - R.a[k])) & ring_mask] = (uint8_t)((y >> 25) + 1);
        run += total;
        cur ^= 1;
        __syncthreads();   // wc is rewritten by the next twist
    }
}

[[maybe_unused]] constexpr int JMP_SEQ = 1 + 19937 + 624;   // y_0 .. y_{19937+623}
[[maybe_unused]] constexpr int JMP_NT = 1024;
[[maybe_unused]] constexpr int JMP_PARTS = 8;               // poly split: 8 x 78 words
constexpr int JMP_JG = 10;                 // 624 outputs in groups of 64

#ifndef SB_MT_JUMP_ROLL
#define SB_MT_JUMP_ROLL 1   // rolling-window jump: 19 KB of LDS (0: the whole sequence in 87 KB)
#endif
#if SB_MT_JUMP_ROLL
// window src0+b -> window dst0+b advanced by J (gp = x^(J-1) mod phi as 624 u32).  In place is safe.
// The sequence y is generated in a ring of JR_RING words, JR_S polynomial bits at a time: each block of
// bits needs y over [i0 + 1, i0 + JR_S + 624]; wave w accumulates the outputs of groups w, w+4, w+8 in
// registers.  Runs beside the step's kernels on the side stream: 87 KB of LDS per CU had held the
// expansion and the select to fewer resident blocks while it ran.
#ifndef SB_JR_WIDE
#define SB_JR_WIDE 1   // 0: one LDS read per set poly bit (the round-2 loop)
#endif
#ifndef SB_JR_NT
#define SB_JR_NT 1024   // A/B profiles/r2_ab_mt_nt.txt: 256 / 640 / 1024 threads
#endif
constexpr int JR_NT = SB_JR_NT, JR_RING = 4096, JR_S = 1024;
constexpr int JR_NW = JR_NT / 64, JR_Q = (JMP_JG + JR_NW - 1) / JR_NW;   // output groups per wave
static_assert(JR_RING >= 2 * JR_S + 624 + 227 + 1, "ring holds the block being read and the next one");
__global__ __launch_bounds__(JR_NT) void k_mt_jump(const uint32_t* win_in, uint32_t* win_out, int src0, int dst0,
                                                    const uint32_t* __restrict__ gpoly) {
    __shared__ uint32_t ring[JR_RING + 32];   // + a mirror of slots 0..31: a word's 32 reads never wrap
    __shared__ uint32_t gp[624];
    constexpr int M = JR_RING - 1;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const int64_t src = src0 + blockIdx.x, dst = dst0 + blockIdx.x;
    for (int i = t; i < 624; i += JR_NT) {
        const uint32_t v = win_in[src * 624 + i];
        ring[i] = v;
        if (SB_JR_WIDE && i < 32) ring[JR_RING + i] = v;
        gp[i] = gpoly[i];
    }
    __syncthreads();
    int have = 624;   // y[0, have) generated
    uint32_t acc[JR_Q];
#pragma unroll
    for (int q = 0; q < JR_Q; q++) acc[q] = 0u;
    for (int i0 = 0; i0 < 19937; i0 += JR_S) {
        const int need = i0 + JR_S + 625;   // y indices read by this block: [i0 + 1, i0 + JR_S + 624]
        while (have < need) {   // y_{k+624} = f(y_k, y_{k+1}, y_{k+397}), 227 at a time
            const int k = have - 624 + t;
            if (t < 227) {
                const int d = (k + 624) & M;
                const uint32_t v = mt_mix(ring[k & M], ring[(k + 1) & M], ring[(k + 397) & M]);
                ring[d] = v;
                if (SB_JR_WIDE && d < 32) ring[JR_RING + d] = v;
            }
            have += 227;
            __syncthreads();
        }
        const int wend = (i0 + JR_S) / 32 < 624 ? (i0 + JR_S) / 32 : 624;
#pragma unroll
        for (int q = 0; q < JR_Q; q++) {
            const int jg = w + JR_NW * q;
            if (jg >= JMP_JG) break;
            const int j = jg * 64 + lane;
            const int jj = j < 624 ? j : 623;
            uint32_t a = acc[q];
            for (int wi = i0 / 32; wi < wend; wi++) {
#if SB_JR_WIDE
                // all 32 words of the slice read at once (immediate offsets from one masked base, no wrap
                // thanks to the mirror), the poly bits applied as wave-uniform masks: the loads pipeline
                // instead of one LDS round trip per set bit
                const uint32_t bits = __builtin_amdgcn_readfirstlane(gp[wi]);
                if (!bits) continue;
                const uint32_t* r = ring + ((1 + wi * 32 + jj) & M);
                uint32_t v[32];
#pragma unroll
                for (int b = 0; b < 32; b++) v[b] = r[b];
#pragma unroll
                for (int b = 0; b < 32; b++) a ^= v[b] & (0u - ((bits >> b) & 1u));
#else
                uint32_t bits = gp[wi];   // wave-uniform
                while (bits) {
                    const int b = __builtin_ctz(bits);
                    bits &= bits - 1;
                    a ^= ring[(1 + wi * 32 + b + jj) & M];
                }
#endif
            }
            acc[q] = a;
        }
        __syncthreads();   // the next block's generation overwrites slots read here
    }
#pragma unroll
    for (int q = 0; q < JR_Q; q++) {
        const int j = (w + JR_NW * q) * 64 + lane;
        if (w + JR_NW * q < JMP_JG && j < 624) win_out[dst * 624 + j] = acc[q];
    }
}
constexpr int JMP_LAUNCH_NT = JR_NT;
#else
constexpr int JMP_LAUNCH_NT = JMP_NT;
// window src0+b -> window dst0+b advanced by J (gp = x^(J-1) mod phi as 624 u32).  In place is safe.
__global__ __launch_bounds__(JMP_NT) void k_mt_jump(const uint32_t* win_in, uint32_t* win_out, int src0, int dst0,
                                                     const uint32_t* __restrict__ gpoly) {
    __shared__ uint32_t seq[JMP_SEQ + 64];
    __shared__ uint32_t res[624];
    __shared__ uint32_t gp[624];
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const int64_t src = src0 + blockIdx.x, dst = dst0 + blockIdx.x;
    for (int i = t; i < 624; i += JMP_NT) {
        seq[i] = win_in[src * 624 + i];
        res[i] = 0;
        gp[i] = gpoly[i];
    }
    __syncthreads();
    for (int k0 = 0; k0 < JMP_SEQ - 624; k0 += 227) {   // y_{k+624} = f(y_k, y_{k+1}, y_{k+397})
        const int k = k0 + t;
        if (t < 227 && k < JMP_SEQ - 624) seq[k + 624] = mt_mix(seq[k], seq[k + 1], seq[k + 397]);
        __syncthreads();
    }
    for (int task = w; task < JMP_JG * JMP_PARTS; task += JMP_NT / 64) {
        const int jg = task % JMP_JG, part = task / JMP_JG;
        const int j = jg * 64 + lane;
        const int jj = j < 624 ? j : 623;
        uint32_t acc = 0;
        const int w0 = part * (624 / JMP_PARTS), w1 = w0 + 624 / JMP_PARTS;
        for (int wi = w0; wi < w1; wi++) {
            uint32_t bits = gp[wi];   // wave-uniform
            while (bits) {
                const int b = __builtin_ctz(bits);
                bits &= bits - 1;
                acc ^= seq[1 + wi * 32 + b + jj];
            }
        }
        if (j < 624) atomicXor(&res[j], acc);
    }
    __syncthreads();
    for (int i = t; i < 624; i += JMP_NT) win_out[dst * 624 + i] = res[i];
}
#endif

void MTProducers::init(const uint32_t origin[624], int P_, int64_t twists_, hipStream_t st) {
    if (P_ < 1 || (P_ & (P_ - 1))) throw HipError{hipErrorInvalidValue, "MT producers must be a power of two"};
    if (!gf2::self_test()) throw HipError{hipErrorInvalidValue, "MT19937 jump-ahead self-test failed"};
    P = P_;
    twists = twists_;
    chunk = 0;
    const uint64_t L = (uint64_t)twists * 624;
    int levels = 0;
    while ((1 << levels) < P) levels++;
    std::vector<uint32_t> polys((size_t)(levels + 1) * 624);
    for (int k = 0; k < levels; k++) gf2::to_words(gf2::jump_poly(L << k), &polys[(size_t)k * 624]);
    gf2::to_words(gf2::jump_poly(L * (uint64_t)P), &polys[(size_t)levels * 624]);
    SB_HIP(hipMalloc((void**)&d_win, (size_t)P * 624 * 4));
    SB_HIP(hipMalloc((void**)&d_poly, polys.size() * 4));
    SB_HIP(hipMemcpyAsync(d_poly, polys.data(), polys.size() * 4, hipMemcpyHostToDevice, st));
    SB_HIP(hipMemcpyAsync(d_win, origin, 624 * 4, hipMemcpyHostToDevice, st));
    for (int k = 0; k < levels; k++)   // doubling tree: windows [2^k, 2^(k+1)) from [0, 2^k)
        hipLaunchKernelGGL(k_mt_jump, dim3(1u << k), dim3(JMP_LAUNCH_NT), 0, st, d_win, d_win, 0, 1 << k,
                           d_poly + (size_t)k * 624);
    chunk_poly = d_poly + (size_t)levels * 624;
    SB_HIP(hipGetLastError());
}

void MTProducers::gen_chunk(uint32_t* out, hipStream_t st) {
    if (chunk > 0)   // every producer jumps P*L ahead of its previous segment start
        hipLaunchKernelGGL(k_mt_jump, dim3(P), dim3(JMP_LAUNCH_NT), 0, st, d_win, d_win, 0, 0, chunk_poly);
    hipLaunchKernelGGL(k_mt_gen_par<0>, dim3(P), dim3(MG_NT), 0, st, d_win, out, (uint8_t*)nullptr,
                       (uint32_t*)nullptr, twists);
    SB_HIP(hipGetLastError());
    chunk++;
}

void MTProducers::gen_chunk_accepted(uint8_t* stage, uint32_t* counts, hipStream_t st) {
    if (chunk > 0)
        hipLaunchKernelGGL(k_mt_jump, dim3(P), dim3(JMP_LAUNCH_NT), 0, st, d_win, d_win, 0, 0, chunk_poly);
    hipLaunchKernelGGL(k_mt_gen_par<1>, dim3(P), dim3(MG_NT), 0, st, d_win, (uint32_t*)nullptr, stage, counts,
                       twists);
    SB_HIP(hipGetLastError());
    chunk++;
}

void MTProducers::release() {
    if (d_win) (void)hipFree(d_win);
    if (d_poly) (void)hipFree(d_poly);
    if (stride_poly) (void)hipFree(stride_poly);
    d_win = d_poly = stride_poly = nullptr;
}

static void compact_accepted(NoiseStream& ns, const uint32_t* raw, int64_t n, hipStream_t st) {
    int64_t nt = (n + MT_TILE - 1) / MT_TILE;
    ns.scan.tiles.ensure(nt);
    hipLaunchKernelGGL(k_mt_count, dim3((unsigned)nt), dim3(MT_NT), 0, st, raw, n, ns.scan.tiles.p);
    scan_tiles_inplace(ns.scan.tiles.p, nt, ns.d_total, st);
    hipLaunchKernelGGL(k_mt_write, dim3((unsigned)nt), dim3(MT_NT), 0, st, raw, n, ns.scan.tiles.p, ns.ring.p,
                       ns.ring_mask, ns.produced);
    SB_HIP(hipMemcpyAsync(ns.h_total, ns.d_total, 4, hipMemcpyDeviceToHost, st));
}

void noise_init(NoiseStream& ns, const uint32_t* state625, uint64_t ring_cap_pow2, int64_t twists, hipStream_t st) {
    memcpy(ns.initial.mt, state625, 624 * 4);
    ns.initial.idx = (int)state625[624];
    ns.replay = ns.initial;
    ns.replay_draws = 0;
    ns.produced = 0;
    ns.consumed = 0;
    ns.ring.ensure(ring_cap_pow2);
    ns.ring_mask = ring_cap_pow2 - 1;
    SB_HIP(hipMalloc((void**)&ns.d_total, 16));
    SB_HIP(hipHostMalloc((void**)&ns.h_total, 16, hipHostMallocDefault));
    SB_HIP(hipEventCreateWithFlags(&ns.ev_ready, hipEventDisableTiming));
    // the host emits the partially consumed block (words idx..623); the device producers start at
    // the next twist of the remaining window
    HostMT h = ns.initial;
    uint32_t lead[624];
    int nlead = 0;
    while (h.idx < 624) lead[nlead++] = h.next();
    ns.prod.init(h.mt, 256, twists, st);
    if (nlead) {
        ns.raw.ensure(624);
        SB_HIP(hipMemcpyAsync(ns.raw.p, lead, nlead * 4, hipMemcpyHostToDevice, st));
        compact_accepted(ns, ns.raw.p, nlead, st);
        SB_HIP(hipStreamSynchronize(st));
        ns.produced += *ns.h_total;
    }
}

uint64_t noise_chunk_words(const NoiseStream& ns) { return (uint64_t)ns.prod.P * ns.prod.twists * 624; }

void noise_generate_async(NoiseStream& ns, hipStream_t st) {
    if (ns.pending) return;
    const uint64_t n = noise_chunk_words(ns);
    const uint64_t room = ns.ring_mask + 1 - (ns.produced - ns.consumed);
    if (n > room) return;   // accepted draws <= words: never overrun unconsumed values
    const int P = ns.prod.P;
    ns.stage.ensure((size_t)n);
    ns.scan.tiles.ensure((size_t)2 * P);
    uint32_t* counts = ns.scan.tiles.p;
    uint32_t* offs = ns.scan.tiles.p + P;
    ns.prod.gen_chunk_accepted(ns.stage.p, counts, st);
    SB_HIP(hipMemcpyAsync(offs, counts, (size_t)P * 4, hipMemcpyDeviceToDevice, st));
    scan_tiles_inplace(offs, P, ns.d_total, st);
    hipLaunchKernelGGL(k_mt_place, dim3(P, MT_PLACE_SPLIT), dim3(256), 0, st, ns.stage.p, (int64_t)ns.prod.twists * 624, counts, offs,
                       ns.ring.p, ns.ring_mask, ns.produced);
    SB_HIP(hipMemcpyAsync(ns.h_total, ns.d_total, 4, hipMemcpyDeviceToHost, st));
    SB_HIP(hipEventRecord(ns.ev_ready, st));
    SB_HIP(hipGetLastError());
    ns.pending = true;
}

static void noise_collect(NoiseStream& ns) {
    if (!ns.pending) return;
    SB_HIP(hipEventSynchronize(ns.ev_ready));
    ns.produced += *ns.h_total;
    ns.pending = false;
}

void noise_ensure(NoiseStream& ns, uint64_t need, hipStream_t st) {
    // wait for an in-flight chunk only when its draws are needed now
    if (ns.pending && (ns.produced - ns.consumed < need || hipEventQuery(ns.ev_ready) == hipSuccess)) noise_collect(ns);
    if (need > ns.ring_mask + 1 - noise_chunk_words(ns))
        throw HipError{hipErrorOutOfMemory, "noise ring too small for one step"};
    while (ns.produced - ns.consumed < need) {
        noise_generate_async(ns, st);
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

// ---- sharded stream (world > 1): this rank owns chunks c = rank, rank + world, ...
void noise_shard_setup(NoiseStream& ns, int rank, int world, hipStream_t st) {
    MTProducers& pr = ns.prod;
    for (int k = 0; k < rank; k++)   // producers to chunk `rank`
        hipLaunchKernelGGL(k_mt_jump, dim3(pr.P), dim3(JMP_LAUNCH_NT), 0, st, pr.d_win, pr.d_win, 0, 0, pr.chunk_poly);
    const uint64_t L = (uint64_t)pr.twists * 624;
    std::vector<uint32_t> w(624);
    gf2::to_words(gf2::jump_poly(L * (uint64_t)pr.P * (uint64_t)world), w.data());
    SB_HIP(hipMalloc((void**)&pr.stride_poly, 624 * 4));
    SB_HIP(hipMemcpyAsync(pr.stride_poly, w.data(), 624 * 4, hipMemcpyHostToDevice, st));
    SB_HIP(hipStreamSynchronize(st));
    pr.chunk = 0;
    ns.ck = (int)std::min<int64_t>(pr.twists, 64);   // fill granularity: 64 twists (~31k draws)
    if (const char* e = getenv("SB_NOISE_CK")) {      // test knob: finer checkpoints (power of two)
        const int v = atoi(e);
        if (v >= 1 && v <= ns.ck && !(v & (v - 1))) ns.ck = v;
    }
    ns.sharded = true;
}

void noise_shard_chunk(NoiseStream& ns, int slot, uint32_t* d_counts, hipStream_t st_main, hipStream_t st_mt) {
    MTProducers& pr = ns.prod;
    if (slot < 0 || slot >= ns.nslots) throw HipError{hipErrorInvalidValue, "noise chunk slot out of range"};
    const int64_t S = pr.twists / ns.ck;
    ns.ckpt.ensure((size_t)ns.nslots * pr.P * S * 624);
    if (!ns.ev_main) SB_HIP(hipEventCreateWithFlags(&ns.ev_main, hipEventDisableTiming));
    SB_HIP(hipEventRecord(ns.ev_main, st_main));   // earlier packs may still read the slot
    SB_HIP(hipStreamWaitEvent(st_mt, ns.ev_main, 0));
    if (pr.chunk > 0)
        hipLaunchKernelGGL(k_mt_jump, dim3(pr.P), dim3(JMP_LAUNCH_NT), 0, st_mt, pr.d_win, pr.d_win, 0, 0, pr.stride_poly);
    hipLaunchKernelGGL(k_mt_gen_par<3>, dim3(pr.P), dim3(MG_NT), 0, st_mt, pr.d_win,
                       ns.ckpt.p + (size_t)slot * pr.P * S * 624, (uint8_t*)nullptr, d_counts, pr.twists, ns.ck);
    SB_HIP(hipGetLastError());
    pr.chunk++;   // asynchronous: the caller synchronises st_mt before using d_counts or the slot
}

__global__ void k_mt_pack(const uint32_t* __restrict__ ckpt, const int64_t* __restrict__ idx, uint32_t* __restrict__ out) {
    const int64_t j = blockIdx.x;
    const uint32_t* src = ckpt + idx[j] * 624;
    for (int t = threadIdx.x; t < 624; t += blockDim.x) out[j * 624 + t] = src[t];
}

void noise_shard_pack(NoiseStream& ns, int m, const int64_t* h_idx, uint32_t* d_out, hipStream_t st) {
    if (m <= 0) return;
    const int64_t lim = (int64_t)ns.nslots * ns.prod.P * (ns.prod.twists / ns.ck);
    for (int j = 0; j < m; j++)
        if (h_idx[j] < 0 || h_idx[j] >= lim) throw HipError{hipErrorInvalidValue, "noise window index out of range"};
    ns.segtab.ensure((size_t)m);
    SB_HIP(hipMemcpyAsync(ns.segtab.p, h_idx, (size_t)m * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_mt_pack, dim3(m), dim3(256), 0, st, ns.ckpt.p, (const int64_t*)ns.segtab.p, d_out);
    SB_HIP(hipGetLastError());   // (pageable-source copy above completes before returning)
}

void noise_shard_fill(NoiseStream& ns, int m, const uint32_t* d_wins, const uint64_t* h_acc0, const NoiseRanges& R,
                      hipStream_t st) {
    if (m <= 0 || R.n <= 0) return;
    ns.segtab.ensure((size_t)m);
    SB_HIP(hipMemcpyAsync(ns.segtab.p, h_acc0, (size_t)m * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_mt_fill, dim3(m), dim3(640), 0, st, d_wins, ns.segtab.p, (int64_t)ns.ck, R, ns.ring.p,
                       ns.ring_mask);
    SB_HIP(hipGetLastError());
}

void noise_free(NoiseStream& ns) {
    if (ns.d_total) (void)hipFree(ns.d_total);
    if (ns.h_total) (void)hipHostFree(ns.h_total);
    if (ns.ev_ready) (void)hipEventDestroy(ns.ev_ready);
    if (ns.ev_main) (void)hipEventDestroy(ns.ev_main);
    ns.ev_main = nullptr;
    ns.ckpt.release();
    ns.prod.release();
    ns.segtab.release();
    ns.raw.release();
    ns.stage.release();
    ns.ring.release();
    ns.scan.tiles.release();
    ns.d_total = nullptr;
    ns.h_total = nullptr;
    ns.ev_ready = nullptr;
}

void mt_debug_words(const uint32_t* state625, int64_t n, int P, int64_t twists, uint32_t* out) {
    HostMT h;
    memcpy(h.mt, state625, 624 * 4);
    h.idx = (int)state625[624];
    int64_t k = 0;
    while (h.idx < 624 && k < n) out[k++] = h.next();
    if (k == n) return;
    MTProducers prod;
    prod.init(h.mt, P, twists, 0);
    const int64_t cw = (int64_t)P * twists * 624;
    uint32_t* dout = nullptr;
    SB_HIP(hipMalloc((void**)&dout, (size_t)cw * 4));
    while (k < n) {
        prod.gen_chunk(dout, 0);
        const int64_t take = n - k < cw ? n - k : cw;
        SB_HIP(hipMemcpy(out + k, dout, (size_t)take * 4, hipMemcpyDeviceToHost));
        k += take;
    }
    (void)hipFree(dout);
    prod.release();
}

}  // namespace sb
