// sb_sort.hip — stable descending top-k of u64 keys: the device form of
//   queue = sorted(next_queue, key=heuristic, reverse=True)[:beam_width]   (src/solver.py:452-456)
// sorted() is stable, so ties keep next_queue order (element index).  Keys are order-preserving u64
// images of the float64 scores (positive scores: the IEEE bits themselves).
//
// Everything runs on the stream without a host round trip:
//   1. min/max of the keys: bits above the highest differing bit are common to all keys and skipped;
//   2. one 11-bit MSB radix-select pass over all n keys finds the bucket holding the keep-th key;
//   3. an order-preserving partition writes the keys above that bucket (all kept) to the output and
//      the bucket's elements to a candidate buffer — later passes read only the candidates;
//   4. further 11-bit passes on the candidates resolve the threshold key T and how many of its ties
//      (first in index order) are kept; a final partition appends the candidates above T, then those
//      ties.  The three output groups have disjoint key sets, so a stable sort of the concatenation
//      orders ties by index exactly as sorted() does;
//   5. a stable LSD radix sort (8-bit digits) orders the kept set by the top 40 of the bits that vary
//      inside [lowest kept key, max] (at most 5 passes, one kernel per digit with decoupled look-back;
//      about 50 us per pass on 4M keys).  Keys are f64 score images: on C3 the kept 4M hold ~115k
//      distinct values over 53 varying bits, and no two of them share a 40-bit prefix (814 pairs do at
//      32 bits, 59 at 36: profiles/analysis/keystats.c, turn 12); 6. an exact fix-up re-orders any run
//      of equal prefixes that still holds different keys, stably by the full key.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "sb_block.h"
#include "sb_internal.h"

namespace sb {

constexpr int TK_NT = 256;
constexpr int TK_IPT = 16;
constexpr int TK_TILE = TK_NT * TK_IPT;   // 4096
constexpr int SEL_D = 11;                 // select digit bits
constexpr int SEL_BINS = 1 << SEL_D;
#ifndef SB_SEL_PREPASS
#define SB_SEL_PREPASS 1   // select digits resolved over all keys before the partition (after the first)
#endif
constexpr int SEL_PREPASS = SB_SEL_PREPASS;
constexpr int SEL_PASSES_C = (64 - SEL_D * (1 + SEL_PREPASS) + SEL_D - 1) / SEL_D;   // candidate passes, at most
#ifndef SB_TKH_GRID
#define SB_TKH_GRID 512    // select histogram blocks (fewer flushes of the 2048 bins; 2048: +30 us)
#endif
#ifndef SB_TKH_U
#define SB_TKH_U 16        // select histogram loads in flight per thread
#endif
#ifndef SB_TK_COUNT_GRID
#define SB_TK_COUNT_GRID 2048   // persistent count blocks (8 per CU)
#endif
constexpr int64_t TK_COUNT_GRID = SB_TK_COUNT_GRID;
#ifndef SB_TK_WRITE_GRID
#define SB_TK_WRITE_GRID 1 << 20   // partition blocks at most (tiles beyond are taken in grid strides)
#endif
constexpr int64_t TK_WRITE_GRID = SB_TK_WRITE_GRID;           // candidate passes: ceil(64 / 11) upper bound
#ifndef SB_SORT_PREFIX_BITS
#define SB_SORT_PREFIX_BITS 38   // 64: the plain full-key LSD sort (A/B knob).  38 = an 8-bit first digit + three
                                 // 10-bit ones: the first pass scatters the prefix's lowest, uniformly spread bits,
                                 // and 256 destinations per tile write longer runs than 1024 (that pass took 83-88 us
                                 // against 48-54 for the others at 40 bits; profiles/r4/s2/sort_d0_ab.txt)
#endif
constexpr int OS_PREFIX_BITS = SB_SORT_PREFIX_BITS;
#ifndef SB_OS_D
#define SB_OS_D 10       // digit bits per LSD pass (see k_os_pass below)
#endif
#ifndef SB_OS_EPOCH
#define SB_OS_EPOCH 1            // look-back granules stamped with a per-call epoch (no clearing memset per call)
#endif
#ifndef SB_TK_STAGE
#define SB_TK_STAGE 1            // first partition: one read, staged per tile (0: count + write, two reads)
#endif
constexpr bool TK_STAGE = SB_TK_STAGE;


// device state (u64 words)
enum : int {
    ST_MIN = 0, ST_MAX, ST_PREFIX, ST_SH, ST_NEED, ST_DONE,
    ST_A,       // keys above the first bucket (kept, output group 1)
    ST_NC,      // candidates (first bucket)
    ST_G2,      // candidates above T (output group 2)
    ST_E2,      // candidates equal to the resolved prefix (before the tie limit)
    ST_BASE2,   // output offset of group 2 (= A)
    ST_BASE3,   // output offset of group 3 (= A + G2)
    ST_TOPK,    // sort: bits [0, TOPK) vary among the kept keys
    ST_FBASE,   // fused first pass: histogram bin b counts keys with key >> SB_SEL_FSH == FBASE + b (edges clamped)
    ST_FALLBACK,  // fused first pass unusable (threshold in a clamped bin): run the generic first pass
    ST_SLO,     // sort: lowest possible kept key; digits are taken from (key - SLO) >> SH32
    ST_SH32,    // sort: low bits below the sorted 40-bit prefix
    ST_FXN,     // fix-up: flagged positions (prefix equal to the predecessor's, key not)
    ST_FXI,     // fix-up: work counter over the flagged positions
    ST_HARR,    // select histogram: blocks arrived (the last one picks: SB_TK_PICK_FUSED)
    ST_T2,      // fused first pass: the lowest kept key two selects back (kept across selects)
    ST_FX2N,    // fix-up: runs deferred by k_fx_wave to k_fx_fix
    ST_FX2I,    // fix-up: work counter over them
    ST_D0,      // sort: bits of the first LSD digit (the prefix bits beyond whole OS_D digits)
    ST_HIST = 24,
    ST_WORDS = ST_HIST + SEL_BINS
};

__device__ __forceinline__ uint64_t hi_bits(uint64_t k, uint64_t sh) { return sh >= 64 ? 0ull : k >> sh; }

__device__ __forceinline__ void tk_init_body(uint64_t* st, int64_t keep, int keep_range, int fused) {
    const int t = threadIdx.x;
    if (t < ST_HIST && t != ST_T2 && (t > ST_MAX || !keep_range) && !(fused && t == ST_FBASE)) st[t] = 0;
    __syncthreads();
    if (t == 0) {
        if (!keep_range) st[ST_MIN] = ~0ull;
        st[ST_NEED] = (uint64_t)keep;
    }
    if (!fused)
        for (int i = t; i < SEL_BINS; i += blockDim.x) st[ST_HIST + i] = 0;
}
__global__ void k_tk_init(uint64_t* st, int64_t keep, int keep_range, int fused) { tk_init_body(st, keep, keep_range, fused); }

#ifndef SB_MINMAX_GRID
#define SB_MINMAX_GRID 256   // blocks: each ends with two atomics on the same two words (they serialise)
#endif
__global__ __launch_bounds__(TK_NT) void k_tk_minmax(const uint64_t* __restrict__ keys, int64_t n, uint64_t* st) {
    __shared__ unsigned long long wmin[TK_NT / 64], wmax[TK_NT / 64];
    uint64_t lo = ~0ull, hi = 0;
    constexpr int U = 8;   // independent loads in flight per thread
    const int64_t stride = (int64_t)gridDim.x * TK_NT;
    for (int64_t i0 = (int64_t)blockIdx.x * TK_NT + threadIdx.x; i0 < n; i0 += stride * U) {
        uint64_t kk[U];
#pragma unroll
        for (int u = 0; u < U; u++) kk[u] = i0 + u * stride < n ? keys[i0 + u * stride] : 0ull;
#pragma unroll
        for (int u = 0; u < U; u++)
            if (i0 + u * stride < n) {
                lo = kk[u] < lo ? kk[u] : lo;
                hi = kk[u] > hi ? kk[u] : hi;
            }
    }
#pragma unroll
    for (int o = 32; o; o >>= 1) {   // wave reduction, then one value per wave
        const uint64_t a = __shfl_xor(lo, o, 64), b = __shfl_xor(hi, o, 64);
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    }
    if ((threadIdx.x & 63) == 0) {
        wmin[threadIdx.x >> 6] = lo;
        wmax[threadIdx.x >> 6] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < TK_NT / 64; w++) {
            lo = wmin[w] < lo ? wmin[w] : lo;
            hi = wmax[w] > hi ? wmax[w] : hi;
        }
        if (hi >= lo) {   // the block saw keys
            atomicMin((unsigned long long*)&st[ST_MIN], (unsigned long long)lo);
            atomicMax((unsigned long long*)&st[ST_MAX], (unsigned long long)hi);
        }
    }
}

// common high bits of all keys: SH = position above the highest differing bit
__device__ __forceinline__ void tk_setup_body(uint64_t* st) {
    const uint64_t x = st[ST_MIN] ^ st[ST_MAX];
    const uint64_t top = x ? 64 - (uint64_t)__clzll((long long)x) : 0;
    st[ST_SH] = top;
    st[ST_PREFIX] = hi_bits(st[ST_MIN], top);
    st[ST_DONE] = top == 0;   // all keys equal: the first `keep` in index order
}
__global__ void k_tk_setup(uint64_t* st) { tk_setup_body(st); }

// pick the bucket holding the need-th largest matching element; clears the histogram.  NT threads;
// AT: read the histogram with agent-scope loads (the last block of k_tk_hist, whose flushes came from
// other blocks of the same launch)
template <int NT, bool AT>
__device__ __forceinline__ void tk_pick_body(uint64_t* st) {
    __shared__ uint32_t lds[NT / 64 + 1];
    const int t = threadIdx.x;
    const uint64_t sh = st[ST_SH];
    const uint64_t d = sh < SEL_D ? sh : SEL_D;
    const int nb = 1 << d;
    constexpr int PER = SEL_BINS / NT;   // bins per thread, descending
    uint64_t c[PER];
    uint64_t loc = 0;
#pragma unroll
    for (int j = 0; j < PER; j++) {
        const int b = nb - 1 - (t * PER + j);
        c[j] = b < 0 ? 0ull
                     : AT ? (uint64_t)__hip_atomic_load((unsigned long long*)&st[ST_HIST + b], __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT)
                          : st[ST_HIST + b];
        loc += c[j];
    }
    // counts fit in u32 (n < 2^32)
    uint32_t tot;
    uint64_t cum = block_excl_scan<NT>((uint32_t)loc, lds, &tot);
    const uint64_t need = st[ST_NEED];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; j++) {
        const int b = nb - 1 - (t * PER + j);
        if (b >= 0 && c[j] && cum < need && cum + c[j] >= need) {
            const uint64_t nneed = need - cum;
            st[ST_NEED] = nneed;
            st[ST_PREFIX] = (st[ST_PREFIX] << d) | (uint64_t)b;
            st[ST_SH] = sh - d;
            st[ST_DONE] = (c[j] == nneed) || (sh - d == 0);
        }
        cum += c[j];
    }
    for (int b = t; b < SEL_BINS; b += NT) st[ST_HIST + b] = 0;
}

#ifndef SB_TK_CAND_PICK
#define SB_TK_CAND_PICK 0   // 1: candidate passes on SB_TK_CAND_GRID blocks, the last one picks (one launch per pass).
                           // A/B (profiles/r4/s2/topk_cand_pick_ab.txt): slower on 64-512 blocks (select +20-220 us)
#endif
#ifndef SB_TK_CAND_GRID
#define SB_TK_CAND_GRID 512
#endif
#ifndef SB_TK_PICK_FUSED
#define SB_TK_PICK_FUSED 0   // 1: the select histogram's last block picks (no k_tk_pick launch per pass).  A/B
                             // (profiles/r3/s5/ab_topk.txt): every block's agent-scope release fence writes its
                             // XCD's L2 back: k_tk_hist 109 -> 421 us per step, select 0.61 -> 0.90 ms
#endif

// histogram of the next digit over the elements matching the resolved prefix; n from n_dev if given
// part != nullptr: the block stores its row of SEL_BINS counts there (k_tk_hsum adds the rows up)
#ifndef SB_TKH_NT
#define SB_TKH_NT 1024     // threads per select-histogram block: 4x the resident waves of 256 at the same flush
                           // count (prepass 89 -> 77 us, profiles/r3/s5/ab_topk.txt)
#endif
constexpr int TKH_NT = SB_TKH_NT;
#ifndef SB_TKH_NH
#define SB_TKH_NH 4   // LDS sub-histograms per select-histogram block (waves share them beyond this many)
#endif
constexpr int TKH_NH = TKH_NT / 64 < SB_TKH_NH ? TKH_NT / 64 : SB_TKH_NH;
__global__ __launch_bounds__(TKH_NT) void k_tk_hist(const uint64_t* __restrict__ keys, int64_t n_host,
                                                   const uint64_t* __restrict__ n_dev, uint64_t* st, int only_fallback,
                                                   uint32_t* __restrict__ part, int pick) {
    if (st[ST_DONE] || (only_fallback && !st[ST_FALLBACK])) return;
    __shared__ uint32_t h[TKH_NH][SEL_BINS];
    __shared__ int s_last;
    const int w = (threadIdx.x >> 6) % TKH_NH;
    for (int i = threadIdx.x; i < TKH_NH * SEL_BINS; i += TKH_NT) (&h[0][0])[i] = 0;
    __syncthreads();
    const int64_t n = n_dev ? (int64_t)*n_dev : n_host;
    const uint64_t sh = st[ST_SH], prefix = st[ST_PREFIX];
    const uint64_t d = sh < SEL_D ? sh : SEL_D;
    const uint64_t dmask = (1ull << d) - 1;
    const uint64_t lt = lanemask_lt();
    constexpr int U = SB_TKH_U;   // loads in flight per thread
    const int64_t stride = (int64_t)gridDim.x * TKH_NT;
    for (int64_t i0 = (int64_t)blockIdx.x * TKH_NT + threadIdx.x; i0 < n; i0 += stride * U) {
        uint64_t kk[U];
#pragma unroll
        for (int u = 0; u < U; u++) kk[u] = i0 + u * stride < n ? keys[i0 + u * stride] : 0ull;
#pragma unroll
        for (int u = 0; u < U; u++) {
            int b = -1;
            if (i0 + u * stride < n && hi_bits(kk[u], sh) == prefix) b = (int)((kk[u] >> (sh - d)) & dmask);
            // scores cluster: lanes sharing the first active lane's bin add once (wave-aggregated)
            const uint64_t act = __ballot(b >= 0);
            if (act) {
                const int b0 = __shfl(b, __builtin_ctzll(act), 64);
                const uint64_t same = __ballot(b == b0);
                if (b == b0) {
                    if ((same & lt) == 0) atomicAdd(&h[w][b0], (uint32_t)__popcll(same));
                } else if (b >= 0) {
                    atomicAdd(&h[w][b], 1u);
                }
            }
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < SEL_BINS; b += TKH_NT) {
        uint32_t c = 0;
#pragma unroll
        for (int x = 0; x < TKH_NH; x++) c += h[x][b];
        if (part) part[(size_t)blockIdx.x * SEL_BINS + b] = c;
        else if (c) atomicAdd((unsigned long long*)&st[ST_HIST + b], (unsigned long long)c);
    }
    if (pick) {   // the last block to arrive picks: every block's flush is performed before its arrival
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads();
        if (threadIdx.x == 0)
            s_last = atomicAdd((unsigned long long*)&st[ST_HARR], 1ull) == (unsigned long long)gridDim.x - 1;
        __syncthreads();
        if (s_last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            tk_pick_body<TKH_NT, true>(st);
            if (threadIdx.x == 0) st[ST_HARR] = 0;
        }
    }
}
// column sums of k_tk_hist's rows: grid (SEL_BINS / 256, ceil(rows / 32)), thread = bin; one atomic
// per (bin, 32 rows) instead of one per (block, bin).  A/B (SB_TKH_2STAGE): the extra launch costs more
// than the flush atomics it removes (select +40 us), so the default flushes with atomics
__global__ __launch_bounds__(256) void k_tk_hsum(const uint32_t* __restrict__ part, int rows, uint64_t* st,
                                                 int only_fallback) {
    if (st[ST_DONE] || (only_fallback && !st[ST_FALLBACK])) return;
    const int b = blockIdx.x * 256 + threadIdx.x, r0 = blockIdx.y * 32;
    uint32_t c = 0;
#pragma unroll
    for (int r = 0; r < 32; r++)
        if (r0 + r < rows) c += part[(size_t)(r0 + r) * SEL_BINS + b];
    if (c) atomicAdd((unsigned long long*)&st[ST_HIST + b], (unsigned long long)c);
}
#ifndef SB_TKH_2STAGE
#define SB_TKH_2STAGE 0   // A/B: select +40 us (profiles/r2_ab_hist_flush.txt)
#endif
__global__ __launch_bounds__(TK_NT) void k_tk_pick(uint64_t* st, int only_fallback);
// one select pass: the histogram of the next digit, then the pick (in the histogram's last block, or a launch)
static void tk_hist_pick(TopkScratch& s, hipStream_t st, const uint64_t* keys, int64_t n, const uint64_t* n_dev,
                         uint64_t* stv, int only_fallback, unsigned grid, bool small = false) {
    uint32_t* part = nullptr;
    if (SB_TKH_2STAGE) {
        s.tkh_part.ensure((size_t)grid * SEL_BINS);
        part = s.tkh_part.p;
    }
    // small: a candidate pass (about 0.1M keys on C3) on a small grid whose last block picks — few blocks, so
    // few of the agent-scope fences that made this slow on the 512-block passes over all keys
    const int fused_pick = (SB_TK_PICK_FUSED || (small && SB_TK_CAND_PICK)) && !part;
    hipLaunchKernelGGL(k_tk_hist, dim3(grid), dim3(TKH_NT), 0, st, keys, n, n_dev, stv, only_fallback, part, fused_pick);
    if (part)
        hipLaunchKernelGGL(k_tk_hsum, dim3(SEL_BINS / 256, (grid + 31) / 32), dim3(256), 0, st, part, (int)grid, stv,
                           only_fallback);
    if (!fused_pick) hipLaunchKernelGGL(k_tk_pick, dim3(1), dim3(TK_NT), 0, st, stv, only_fallback);
}

__global__ __launch_bounds__(TK_NT) void k_tk_pick(uint64_t* st, int only_fallback) {
    if (st[ST_DONE] || (only_fallback && !st[ST_FALLBACK])) return;
    tk_pick_body<TK_NT, false>(st);
}

// First pass from the histogram the emission folded (bins of key >> SB_SEL_FSH in [FBASE, FBASE + 2048), the
// edge bins clamped): pick the bin holding the keep-th largest key.  An edge bin mixes prefixes, so a
// threshold there (or a count that is not n) sets FALLBACK and the generic first pass runs instead.
__device__ __forceinline__ void tk_pick_fused_body(uint64_t* st, int64_t n) {
    __shared__ uint32_t lds[TK_NT / 64 + 1];
    const int t = threadIdx.x;
    constexpr int PER = SEL_BINS / TK_NT;
    uint64_t c[PER];
    uint64_t loc = 0;
#pragma unroll
    for (int j = 0; j < PER; j++) {
        c[j] = st[ST_HIST + SEL_BINS - 1 - (t * PER + j)];
        loc += c[j];
    }
    uint32_t tot;
    uint64_t cum = block_excl_scan<TK_NT>((uint32_t)loc, lds, &tot);
    const uint64_t need = st[ST_NEED];
    if (t == 0) st[ST_FALLBACK] = 1;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; j++) {
        const int b = SEL_BINS - 1 - (t * PER + j);
        if (c[j] && cum < need && cum + c[j] >= need && (int64_t)tot == n && b > 0 && b < SEL_BINS - 1) {
            const uint64_t nneed = need - cum;
            st[ST_NEED] = nneed;
            st[ST_PREFIX] = st[ST_FBASE] + (uint64_t)b;
            st[ST_SH] = SB_SEL_FSH;
            st[ST_DONE] = c[j] == nneed;
            st[ST_FALLBACK] = 0;
        }
        cum += c[j];
    }
    __syncthreads();
    for (int b = t; b < SEL_BINS; b += TK_NT) st[ST_HIST + b] = 0;
}

// the fused select's first kernel: state reset, the pick from the folded histogram and, when that is
// unusable, the generic first pass's setup
__global__ __launch_bounds__(TK_NT) void k_tk_begin_fused(uint64_t* st, int64_t keep, int64_t n) {
    tk_init_body(st, keep, 1, 1);
    __syncthreads();
    tk_pick_fused_body(st, n);
    __syncthreads();
    if (threadIdx.x == 0 && st[ST_FALLBACK]) tk_setup_body(st);
}

// per-tile counts of elements above / equal to the resolved prefix.  A block takes tiles
// blockIdx.x, + gridDim.x, ... (16 loads in flight per thread); a wave counts with ballots and the four
// wave counts meet in LDS (double-buffered: one barrier per tile).
__global__ __launch_bounds__(TK_NT) void k_tk_count(const uint64_t* __restrict__ keys, int64_t n_host,
                                                    const uint64_t* __restrict__ n_dev, const uint64_t* __restrict__ st,
                                                    uint32_t* __restrict__ gt, uint32_t* __restrict__ eq) {
    constexpr int NW = TK_NT / 64;
    __shared__ uint32_t wc[2][2][NW];
    const int64_t n = n_dev ? (int64_t)*n_dev : n_host;
    const uint64_t sh = st[ST_SH], prefix = st[ST_PREFIX];
    const int t = threadIdx.x, w = t >> 6;
    const int64_t ntiles = (n + TK_TILE - 1) / TK_TILE;
    int buf = 0;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x, buf ^= 1) {
        const int64_t base = tile * TK_TILE;
        uint64_t kk[TK_IPT];
#pragma unroll
        for (int j = 0; j < TK_IPT; j++) {
            const int64_t i = base + (int64_t)j * TK_NT + t;
            kk[j] = i < n ? keys[i] : 0ull;
        }
        uint32_t a = 0, b = 0;
#pragma unroll
        for (int j = 0; j < TK_IPT; j++) {
            const int64_t i = base + (int64_t)j * TK_NT + t;
            const uint64_t hb = hi_bits(kk[j], sh);
            a += (uint32_t)__popcll(__ballot(i < n && hb > prefix));
            b += (uint32_t)__popcll(__ballot(i < n && hb == prefix));
        }
        if ((t & 63) == 0) {
            wc[buf][0][w] = a;
            wc[buf][1][w] = b;
        }
        __syncthreads();
        if (t == 0) {
            uint32_t sa = 0, sb = 0;
#pragma unroll
            for (int x = 0; x < NW; x++) {
                sa += wc[buf][0][x];
                sb += wc[buf][1][x];
            }
            gt[tile] = sa;
            eq[tile] = sb;
        }
    }
}

// single workgroup: exclusive tile offsets for both classes; totals into st[slot_gt], st[slot_eq].
// phase 2 also sets the output bases of groups 2 and 3.  Thread t scans SC_PER consecutive tiles in
// registers; one workgroup scan per SC_PER * 1024 tiles.
constexpr int SC_PER = 16;
__device__ __forceinline__ void tk_sortsetup_body(uint64_t* st, int selected, int prefix_bits);
// lb (the final partition's scan, SB_OS_EPOCH): the select's state is final here, so this one workgroup also
// does the sort's setup and clears the look-back buffer's hdr_words header words (no k_os_begin launch)
__global__ __launch_bounds__(1024) void k_tk_scan(uint32_t* __restrict__ gt, uint32_t* __restrict__ eq, int64_t n_host,
                                                   const uint64_t* __restrict__ n_dev, uint64_t* st, int slot_gt,
                                                   int slot_eq, int phase2, uint64_t* __restrict__ lb = nullptr,
                                                   int hdr_words = 0, int prefix_bits = 0) {
    __shared__ uint32_t lds[1024 / 64 + 1];
    // the chunk's counts and offsets staged through LDS so that loads and stores are coalesced (a thread's SC_PER
    // consecutive tiles straight from global touched a line per lane: 17-22 us for C3's 9.2k tiles), padded rows
    // against bank conflicts
    __shared__ uint32_t sg_l[1024 * (SC_PER + 1)], se_l[1024 * (SC_PER + 1)];
    const int64_t ntiles = ((n_dev ? (int64_t)*n_dev : n_host) + TK_TILE - 1) / TK_TILE;
    uint32_t cg = 0, ce = 0;
    for (int64_t b = 0; b < ntiles; b += 1024 * SC_PER) {
        if (b > 0) __syncthreads();   // the previous chunk's LDS reads are done
#pragma unroll
        for (int j = 0; j < SC_PER; j++) {
            const int64_t k = (int64_t)j * 1024 + threadIdx.x;   // chunk-relative tile, coalesced over threads
            const uint32_t row = (uint32_t)(k / SC_PER), col = (uint32_t)(k % SC_PER);
            sg_l[row * (SC_PER + 1) + col] = b + k < ntiles ? gt[b + k] : 0u;
            se_l[row * (SC_PER + 1) + col] = b + k < ntiles ? eq[b + k] : 0u;
        }
        __syncthreads();
        uint32_t g[SC_PER], e[SC_PER], sg = 0, se = 0;
#pragma unroll
        for (int j = 0; j < SC_PER; j++) {
            g[j] = sg_l[threadIdx.x * (SC_PER + 1) + j];
            e[j] = se_l[threadIdx.x * (SC_PER + 1) + j];
            sg += g[j];
            se += e[j];
        }
        uint32_t tg, te;
        uint32_t xg = block_excl_scan<1024>(sg, lds, &tg) + cg;
        uint32_t xe = block_excl_scan<1024>(se, lds, &te) + ce;
#pragma unroll
        for (int j = 0; j < SC_PER; j++) {   // the offsets back through LDS: coalesced stores
            sg_l[threadIdx.x * (SC_PER + 1) + j] = xg;
            se_l[threadIdx.x * (SC_PER + 1) + j] = xe;
            xg += g[j];
            xe += e[j];
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < SC_PER; j++) {
            const int64_t k = (int64_t)j * 1024 + threadIdx.x;
            const uint32_t row = (uint32_t)(k / SC_PER), col = (uint32_t)(k % SC_PER);
            if (b + k < ntiles) {
                gt[b + k] = sg_l[row * (SC_PER + 1) + col];
                eq[b + k] = se_l[row * (SC_PER + 1) + col];
            }
        }
        cg += tg;
        ce += te;
    }
    if (threadIdx.x == 0) {
        st[slot_gt] = cg;
        st[slot_eq] = ce;
        if (phase2) {
            st[ST_BASE2] = st[ST_A];
            st[ST_BASE3] = st[ST_A] + cg;
        }
    }
    if (lb) {
        if (threadIdx.x == 0) tk_sortsetup_body(st, 1, prefix_bits);
        for (int i = threadIdx.x; i < hdr_words; i += blockDim.x) lb[i] = 0;
    }
}

// The select's tail in one workgroup (small candidate sets: C4's hold a few thousand keys): every remaining
// digit over the candidates (LDS histogram, in-block pick), then the stable partition of the candidates above T
// (group 2) and the first NEED ties (group 3), the totals and bases, and the sort's setup — in place of up to four
// histogram + pick launch pairs and the count / scan / write launches, each ≈4.5 us even when it has nothing to do.
// Correct for any candidate count; the host picks it from the previous select's count (a large jump only costs time).
constexpr int TT_NT = 1024;
constexpr int TT_U = 8;   // candidate loads in flight per thread
__global__ __launch_bounds__(TT_NT) void k_tk_tail(const uint64_t* __restrict__ ck, const uint32_t* __restrict__ ci,
                                                   uint64_t* st, uint64_t* __restrict__ gk, uint32_t* __restrict__ gi,
                                                   uint64_t* __restrict__ lb, int hdr_words, int prefix_bits) {
    __shared__ uint32_t h[SEL_BINS];
    __shared__ uint32_t lds[TT_NT / 64 + 1];
    __shared__ uint64_t s_prefix, s_sh, s_need;
    __shared__ int s_done;
    const int t = threadIdx.x;
    const int64_t nc = (int64_t)st[ST_NC];
    if (t == 0) {
        s_prefix = st[ST_PREFIX];
        s_sh = st[ST_SH];
        s_need = st[ST_NEED];
        s_done = (int)st[ST_DONE];
    }
    __syncthreads();
    for (int it = 0; it < 8 && !s_done && s_sh > 0; it++) {   // at most ceil(64 / SEL_D) digits
        const uint64_t sh = s_sh, prefix = s_prefix, need = s_need;
        const uint64_t d = sh < SEL_D ? sh : SEL_D;
        const uint64_t dmask = (1ull << d) - 1;
        for (int i = t; i < SEL_BINS; i += TT_NT) h[i] = 0;
        __syncthreads();
        for (int64_t i0 = t; i0 < nc; i0 += (int64_t)TT_NT * TT_U) {
            uint64_t kk[TT_U];
#pragma unroll
            for (int u = 0; u < TT_U; u++) kk[u] = i0 + u * TT_NT < nc ? ck[i0 + u * TT_NT] : 0ull;
#pragma unroll
            for (int u = 0; u < TT_U; u++)
                if (i0 + u * TT_NT < nc && hi_bits(kk[u], sh) == prefix) atomicAdd(&h[(kk[u] >> (sh - d)) & dmask], 1u);
        }
        __syncthreads();
        const int nb = 1 << d;
        constexpr int PER = SEL_BINS / TT_NT;
        uint32_t c[PER], loc = 0;
#pragma unroll
        for (int j = 0; j < PER; j++) {
            const int b = nb - 1 - (t * PER + j);
            c[j] = b >= 0 ? h[b] : 0u;
            loc += c[j];
        }
        uint32_t tot;
        uint64_t cum = block_excl_scan<TT_NT>(loc, lds, &tot);
#pragma unroll
        for (int j = 0; j < PER; j++) {
            const int b = nb - 1 - (t * PER + j);
            if (b >= 0 && c[j] && cum < need && cum + c[j] >= need) {
                s_need = need - cum;
                s_prefix = (prefix << d) | (uint64_t)b;
                s_sh = sh - d;
                s_done = (c[j] == need - cum) || (sh - d == 0);
            }
            cum += c[j];
        }
        __syncthreads();
    }
    const uint64_t sh = s_sh, prefix = s_prefix, need = s_need;
    // group 2's size first (group 3 starts after it), then both groups in index order, 1024 candidates a round
    uint32_t above = 0;
    for (int64_t i = t; i < nc; i += TT_NT) above += hi_bits(ck[i], sh) > prefix;
    uint32_t g2;
    (void)block_excl_scan<TT_NT>(above, lds, &g2);
    const uint64_t base2 = st[ST_A], base3 = base2 + g2;
    uint64_t run_g = 0, run_e = 0;
    for (int64_t b0 = 0; b0 < nc; b0 += TT_NT) {
        const int64_t i = b0 + t;
        uint64_t k = 0;
        bool g = false, e = false;
        if (i < nc) {
            k = ck[i];
            const uint64_t hb = hi_bits(k, sh);
            g = hb > prefix;
            e = hb == prefix;
        }
        uint32_t totv;
        const uint32_t x = block_excl_scan<TT_NT>((uint32_t)g | ((uint32_t)e << 16), lds, &totv);
        if (g) {
            const uint64_t o = base2 + run_g + (x & 0xFFFFu);
            gk[o] = k;
            gi[o] = ci[i];
        } else if (e) {
            const uint64_t re = run_e + (x >> 16);
            if (re < need) {
                gk[base3 + re] = k;
                gi[base3 + re] = ci[i];
            }
        }
        run_g += totv & 0xFFFFu;
        run_e += totv >> 16;
    }
    __syncthreads();
    if (t == 0) {
        st[ST_PREFIX] = prefix;
        st[ST_SH] = sh;
        st[ST_NEED] = need;
        st[ST_DONE] = 1;
        st[ST_G2] = g2;
        st[ST_E2] = run_e;
        st[ST_BASE2] = base2;
        st[ST_BASE3] = base3;
        if (lb) tk_sortsetup_body(st, 1, prefix_bits);
    }
    if (lb)
        for (int i = t; i < hdr_words; i += TT_NT) lb[i] = 0;
}

// Order-preserving partition of a tile (4096 elements, striped: element r*256 + t is thread t's r-th):
// all 16 keys of a thread are loaded up front; per round and wave a ballot per class; one scan over
// the tile's 16 x 4 (round, wave) counts orders everything.  A block takes tiles in grid strides.
// Elements above the prefix -> (gk, gi) at *gbase + rank; equal ones -> (ek, ei) at *ebase + rank,
// only the first *limit of them if limit is given.
__global__ __launch_bounds__(TK_NT) void k_tk_write(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ idx,
                                                    int64_t n_host, const uint64_t* __restrict__ n_dev,
                                                    const uint64_t* __restrict__ st, const uint32_t* __restrict__ gt_off,
                                                    const uint32_t* __restrict__ eq_off, uint64_t* __restrict__ gk,
                                                    uint32_t* __restrict__ gi, const uint64_t* __restrict__ gbase,
                                                    uint64_t* __restrict__ ek, uint32_t* __restrict__ ei,
                                                    const uint64_t* __restrict__ ebase, const uint64_t* __restrict__ limit,
                                                    const uint32_t* __restrict__ pay) {
    constexpr int NW = TK_NT / 64;
    __shared__ uint32_t cnt[TK_IPT * NW];   // (round, wave): above | equal << 16, then exclusive offsets
    const int64_t n = n_dev ? (int64_t)*n_dev : n_host;
    const int64_t ntiles = (n + TK_TILE - 1) / TK_TILE;
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const uint64_t sh = st[ST_SH], prefix = st[ST_PREFIX];
    const uint64_t lim = limit ? *limit : ~0ull;
    const uint64_t eb = ebase ? *ebase : 0;
    const uint64_t gb = gbase ? *gbase : 0;
    const uint64_t lt = lanemask_lt();
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t base = tile * TK_TILE;
        uint64_t kk[TK_IPT];
#pragma unroll
        for (int r = 0; r < TK_IPT; r++) {
            const int64_t i = base + (int64_t)r * TK_NT + t;
            kk[r] = i < n ? keys[i] : 0ull;
        }
        uint32_t fg = 0, fe = 0;   // bit r: this thread's r-th element is above / equal
#pragma unroll
        for (int r = 0; r < TK_IPT; r++) {
            const int64_t i = base + (int64_t)r * TK_NT + t;
            const uint64_t hb = hi_bits(kk[r], sh);
            const bool g = i < n && hb > prefix, e = i < n && hb == prefix;
            fg |= (uint32_t)g << r;
            fe |= (uint32_t)e << r;
            const uint64_t bg = __ballot(g), be = __ballot(e);
            if (l == 0) cnt[r * NW + w] = (uint32_t)__popcll(bg) | ((uint32_t)__popcll(be) << 16);
        }
        // the written elements' payloads, all loads in flight across the barriers (loaded in the write loop,
        // each round waited for its own load: up to 16 latencies per tile)
        uint32_t pv[TK_IPT];
#pragma unroll
        for (int r = 0; r < TK_IPT; r++) {
            const int64_t i = base + (int64_t)r * TK_NT + t;
            pv[r] = ((fg | fe) >> r) & 1 ? (idx ? idx[i] : (pay ? pay[i] : (uint32_t)i)) : 0u;
        }
        __syncthreads();
        if (t < 64) {   // exclusive scan of the 64 packed counts (round-major = index order)
            const uint32_t v = t < TK_IPT * NW ? cnt[t] : 0u;
            const uint32_t inc = wave_incl_scan(v);
            if (t < TK_IPT * NW) cnt[t] = inc - v;
        }
        __syncthreads();
        if (fg | fe) {
            const uint64_t og = gb + gt_off[tile];
            const uint64_t oe = eq_off[tile];   // rank among equal elements before this tile
#pragma unroll
            for (int r = 0; r < TK_IPT; r++) {
                const uint64_t bg = __ballot((fg >> r) & 1), be = __ballot((fe >> r) & 1);
                const uint32_t c = cnt[r * NW + w];
                if ((fg >> r) & 1) {
                    const uint64_t o = og + (c & 0xFFFFu) + __popcll(bg & lt);
                    gk[o] = kk[r];
                    gi[o] = pv[r];
                } else if ((fe >> r) & 1) {
                    const uint64_t re = oe + (c >> 16) + __popcll(be & lt);
                    if (re < lim) {
                        ek[eb + re] = kk[r];
                        ei[eb + re] = pv[r];
                    }
                }
            }
        }
        __syncthreads();   // the next tile rewrites cnt
    }
}

// The first partition over all n keys in one read (SB_TK_STAGE): a tile ranks its elements as k_tk_write
// does and stages them in its own TK_TILE-slot region of (sk, si) — elements above the prefix from the
// region's front, equal ones from its back (reversed) — and stores its two counts; k_tk_scan then gives
// every tile its offsets and k_tk_unstage copies the staged elements to their places.  k_tk_count +
// k_tk_write read the n keys twice; this reads them once and moves only the staged ~10%.
__global__ __launch_bounds__(TK_NT) void k_tk_stage(const uint64_t* __restrict__ keys, int64_t n,
                                                    const uint64_t* __restrict__ st, uint32_t* __restrict__ gt,
                                                    uint32_t* __restrict__ eq, uint64_t* __restrict__ sk,
                                                    uint32_t* __restrict__ si, const uint32_t* __restrict__ pay) {
    constexpr int NW = TK_NT / 64;
    __shared__ uint32_t cnt[TK_IPT * NW];   // (round, wave): above | equal << 16, then exclusive offsets
    __shared__ uint32_t tot;
    const int64_t ntiles = (n + TK_TILE - 1) / TK_TILE;
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const uint64_t sh = st[ST_SH], prefix = st[ST_PREFIX];
    const uint64_t lt = lanemask_lt();
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t base = tile * TK_TILE;
        uint64_t kk[TK_IPT];
#pragma unroll
        for (int r = 0; r < TK_IPT; r++) {
            const int64_t i = base + (int64_t)r * TK_NT + t;
            kk[r] = i < n ? keys[i] : 0ull;
        }
        uint32_t fg = 0, fe = 0;
#pragma unroll
        for (int r = 0; r < TK_IPT; r++) {
            const int64_t i = base + (int64_t)r * TK_NT + t;
            const uint64_t hb = hi_bits(kk[r], sh);
            const bool g = i < n && hb > prefix, e = i < n && hb == prefix;
            fg |= (uint32_t)g << r;
            fe |= (uint32_t)e << r;
            const uint64_t bg = __ballot(g), be = __ballot(e);
            if (l == 0) cnt[r * NW + w] = (uint32_t)__popcll(bg) | ((uint32_t)__popcll(be) << 16);
        }
        uint32_t pv[TK_IPT];   // payloads of the staged elements, loads in flight across the barriers
#pragma unroll
        for (int r = 0; r < TK_IPT; r++) {
            const int64_t i = base + (int64_t)r * TK_NT + t;
            pv[r] = ((fg | fe) >> r) & 1 ? (pay ? pay[i] : (uint32_t)i) : 0u;
        }
        __syncthreads();
        if (t < 64) {
            const uint32_t v = t < TK_IPT * NW ? cnt[t] : 0u;
            const uint32_t inc = wave_incl_scan(v);
            if (t < TK_IPT * NW) cnt[t] = inc - v;
            if (t == 63) tot = inc;
        }
        __syncthreads();
        if (t == 0) {
            gt[tile] = tot & 0xFFFFu;
            eq[tile] = tot >> 16;
        }
        if (fg | fe) {
#pragma unroll
            for (int r = 0; r < TK_IPT; r++) {
                const uint64_t bg = __ballot((fg >> r) & 1), be = __ballot((fe >> r) & 1);
                const uint32_t c = cnt[r * NW + w];
                int64_t o = -1;
                if ((fg >> r) & 1) o = base + (c & 0xFFFFu) + __popcll(bg & lt);
                else if ((fe >> r) & 1) o = base + TK_TILE - 1 - ((c >> 16) + __popcll(be & lt));
                if (o >= 0) {
                    sk[o] = kk[r];
                    si[o] = pv[r];
                }
            }
        }
        __syncthreads();   // the next tile rewrites cnt
    }
}

// staged elements to their places: tile t's above ones to (gk, gi)[gt_off[t] ..), its equal ones (in index
// order) to (ek, ei)[eq_off[t] ..); counts from consecutive offsets (the last tile's from the totals).  A
// wave per tile.
__global__ __launch_bounds__(256) void k_tk_unstage(const uint64_t* __restrict__ sk, const uint32_t* __restrict__ si,
                                                    int64_t n, const uint64_t* __restrict__ st,
                                                    const uint32_t* __restrict__ gt_off, const uint32_t* __restrict__ eq_off,
                                                    uint64_t* __restrict__ gk, uint32_t* __restrict__ gi,
                                                    uint64_t* __restrict__ ek, uint32_t* __restrict__ ei) {
    const int64_t ntiles = (n + TK_TILE - 1) / TK_TILE;
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    const uint32_t ta = (uint32_t)st[ST_A], te = (uint32_t)st[ST_NC];
    for (int64_t tile = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); tile < ntiles; tile += nw) {
        const uint32_t og = gt_off[tile], oe = eq_off[tile];
        const uint32_t a = (tile + 1 < ntiles ? gt_off[tile + 1] : ta) - og;
        const uint32_t e = (tile + 1 < ntiles ? eq_off[tile + 1] : te) - oe;
        const int64_t base = tile * TK_TILE;
        constexpr int U = 8;   // loads in flight per lane before the stores
        for (uint32_t j0 = 0; j0 < a; j0 += 64 * U) {
            uint64_t kv[U];
            uint32_t iv[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t j = j0 + u * 64 + lane;
                if (j < a) {
                    kv[u] = sk[base + j];
                    iv[u] = si[base + j];
                }
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t j = j0 + u * 64 + lane;
                if (j < a) {
                    gk[og + j] = kv[u];
                    gi[og + j] = iv[u];
                }
            }
        }
        for (uint32_t j = lane; j < e; j += 64) {
            ek[oe + j] = sk[base + TK_TILE - 1 - j];
            ei[oe + j] = si[base + TK_TILE - 1 - j];
        }
    }
}

__global__ void k_iota(uint32_t* v, const uint64_t* keys, uint64_t* okeys, int64_t n, const uint32_t* pay) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        v[i] = pay ? pay[i] : (uint32_t)i;
        okeys[i] = keys[i];
    }
}

// bits that vary among the kept keys: [lowest kept, max]; lowest kept >= prefix << sh
// The kept keys lie in [lo, max]: sorting key - lo (same order) needs only the bits of max - lo,
// one digit fewer than the bits in which lo and max differ when the range crosses a power of two.
__device__ __forceinline__ void tk_sortsetup_body(uint64_t* st, int selected, int prefix_bits) {
    uint64_t lo = st[ST_MIN];
    if (selected) lo = st[ST_SH] >= 64 ? 0ull : (st[ST_PREFIX] << st[ST_SH]);
    const uint64_t x = st[ST_MAX] - lo;
    const uint64_t topk = x ? 64 - (uint64_t)__clzll((long long)x) : 0;
    st[ST_SLO] = lo;
    st[ST_TOPK] = topk;
    st[ST_SH32] = topk > (uint64_t)prefix_bits ? topk - prefix_bits : 0;   // the sort orders the top varying bits
    st[ST_D0] = (uint64_t)(prefix_bits % SB_OS_D ? prefix_bits % SB_OS_D : SB_OS_D);   // first digit: the bits beyond whole digits
    st[ST_FXN] = 0;
    st[ST_FXI] = 0;
    st[ST_FX2N] = 0;
    st[ST_FX2I] = 0;
}
__global__ void k_tk_sortsetup(uint64_t* st, int selected, int prefix_bits) { tk_sortsetup_body(st, selected, prefix_bits); }

// ---- stable LSD radix sort of the kept set, one kernel per OS_D-bit digit (decoupled look-back)
// Digit p of key k is (~(k - SLO) >> OS_D p) & (OS_B - 1) (ascending digits = descending keys).  k_os_hist builds the
// global histograms of every needed digit in one read.  Pass p: tiles of OS_TILE elements take
// tickets in launch order; a tile ranks its elements stably ((round, wave) counts per digit + the
// lane rank from a wave match), publishes its per-digit counts, looks back over its predecessors'
// published counts for its exclusive offsets and scatters.  The look-back words are 8-byte granules
// {epoch = pass + 1, flag, count} stored and polled with agent-scope atomics (sc1): the data is the
// flag, so no fence is needed.  The granules are zeroed once per sort call (memset); a predecessor
// always holds an earlier ticket, so it is resident and the wait ends.
constexpr int OS_NT = 256;
#ifndef SB_OS_IPT
#define SB_OS_IPT 8      // elements per thread: 8 x 1024 threads = 8192-element tiles (16 spills 45 VGPRs at 1024)
#endif
constexpr int OS_IPT = SB_OS_IPT;
#ifndef SB_OS_PNT
#define SB_OS_PNT 1024   // threads per sort-pass workgroup (one tile of OS_PNT * OS_IPT elements): with 10-bit
                         // digits each thread owns one digit's look-back (OS_DPT = 1)
#endif
constexpr int OS_PNT = SB_OS_PNT;
constexpr int OS_TILE = OS_PNT * OS_IPT;
constexpr int OS_NW = OS_PNT / 64;   // waves per pass workgroup
#ifndef SB_OS_LB
#define SB_OS_LB 8       // predecessors polled together per look-back round (16: 123 VGPRs, select +20-30 us on C3,
                         // +10 on C4; 32 spills: profiles/r4/s2/fsh_ab.txt)
#endif
constexpr int OS_LB = SB_OS_LB;
#ifndef SB_OS_DBG
#define SB_OS_DBG 0      // timing diagnostics only (wrong order): 1 no look-back, 2 unscattered writes
#endif
#ifndef SB_OS_D
#define SB_OS_D 10       // digit bits per LSD pass: four passes for the 40-bit prefix.  Round 4: 10-bit digits on
                         // 1024-thread, 8192-element tiles (one digit per thread in the look-back, 107 VGPRs) against
                         // round 3's 8-bit digits on 256 x 16: select 0.608-0.611 -> 0.583-0.584 ms on C3, 0.293 ->
                         // 0.271-0.273 on C4 (profiles/r4/s2/sort_ab.txt).  Round 3 measured 10-bit digits on the
                         // 256-thread tiles at 132 us per pass (four digits per thread, 229 VGPRs, 2 waves per SIMD)
#endif
constexpr int OS_D = SB_OS_D;
constexpr int OS_B = 1 << OS_D;                     // bins per digit
constexpr int OS_MAXP = (64 + OS_D - 1) / OS_D;     // passes over a full 64-bit key
constexpr int OS_DPT = OS_B / OS_PNT;               // digits owned per pass thread (consecutive)
static_assert(OS_B % OS_PNT == 0 && OS_MAXP <= 8, "digit width vs pass workgroup");
constexpr uint64_t OS_AGG = 1ull << 32, OS_INC = 2ull << 32;
constexpr uint32_t OS_SPIN_MAX = 1u << 26;
// control words at the start of the look-back buffer (u64): the digit histograms (u32 pairs), tickets
constexpr int OS_HIST_WORDS = OS_MAXP * OS_B / 2;
constexpr int OS_TICKET = OS_HIST_WORDS;          // 8 u32 tickets in 4 words
constexpr int OS_ERR = OS_TICKET + 4;             // spin-limit flag
constexpr int OS_HDR = OS_ERR + 4;                // 16-B aligned

typedef __attribute__((address_space(1))) unsigned long long gu64_t;

// sort setup + the look-back buffer's header (digit histograms, tickets, error word) cleared: one launch
__global__ void k_os_begin(uint64_t* st, int selected, int prefix_bits, uint64_t* __restrict__ lb) {
    if (threadIdx.x == 0) tk_sortsetup_body(st, selected, prefix_bits);
    for (int i = threadIdx.x; i < OS_HDR; i += blockDim.x) lb[i] = 0;
}

__device__ __forceinline__ void os_publish(uint64_t* p, uint64_t v) {
    __hip_atomic_store((gu64_t*)p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t os_poll(const uint64_t* p) {
    return __hip_atomic_load((gu64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// digit p covers bits [os_shift(p), os_shift(p) + os_width(p)) of the prefix: the first is ST_D0 bits wide, the rest OS_D
__device__ __forceinline__ int sort_passes(const uint64_t* st) {
    const int64_t v = (int64_t)(st[ST_TOPK] - st[ST_SH32]), d0 = (int64_t)st[ST_D0];
    return v <= 0 ? 0 : (v <= d0 ? 1 : 1 + (int)((v - d0 + OS_D - 1) / OS_D));
}
__device__ __forceinline__ int os_shift(const uint64_t* st, int p) { return p == 0 ? 0 : (int)st[ST_D0] + OS_D * (p - 1); }
__device__ __forceinline__ uint32_t os_mask(const uint64_t* st, int p) {
    return p == 0 ? (1u << (int)st[ST_D0]) - 1u : (uint32_t)(OS_B - 1);
}
__device__ __forceinline__ uint64_t sort_prefix(uint64_t k, uint64_t slo, uint64_t sh) { return (k - slo) >> sh; }

// histograms of every needed digit over the m keys (first lane's bin wave-aggregated: high digits
// cluster); 16 loads in flight per thread
#ifndef SB_OSH_GRID
#define SB_OSH_GRID 256      // 1024-thread blocks, one per CU (a quarter of the 256-thread grid's flush atomics:
                             // 39 -> 29 us, profiles/r3/s5/ab_topk.txt)
#endif
#ifndef SB_OSH_NT
#define SB_OSH_NT 1024       // threads per k_os_hist block
#endif
constexpr int OSH_NT = SB_OSH_NT;
#ifndef SB_OSH_WH
#define SB_OSH_WH 1          // per-wave sub-histograms (less LDS atomic contention between waves)
#endif
constexpr int OSH_NHMAX = 65536 / (OS_MAXP * OS_B * 4) < 1 ? 1 : 65536 / (OS_MAXP * OS_B * 4);   // 64 KB of LDS
constexpr int OSH_NH = SB_OSH_WH ? (OSH_NT / 64 < OSH_NHMAX ? OSH_NT / 64 : OSH_NHMAX) : 1;
// Flush of the blocks' histograms: one atomic per (block, bin).  The two-stage flush (SB_OSH_2STAGE:
// each block stores its row of P*256 counts, k_os_hsum adds 32 rows per thread with one atomic per
// (column, 32 rows)) was measured no faster: the same-address atomics are not what bounds k_os_hist.
#ifndef SB_OSH_2STAGE
#define SB_OSH_2STAGE 0   // A/B: no faster (profiles/r2_ab_hist_flush.txt)
#endif
constexpr int OSH_ROW = OS_MAXP * OS_B;   // u32 per block row (every digit)
constexpr int OSH_RCHUNK = 32;       // rows per k_os_hsum thread
// first_dev (optional): count only keys[*first_dev ..) (the rest were counted where they were written)
__global__ __launch_bounds__(OSH_NT) void k_os_hist(const uint64_t* __restrict__ keys, int64_t n,
                                                    const uint64_t* __restrict__ st, uint64_t* __restrict__ lb,
                                                    uint32_t* __restrict__ part, const uint64_t* __restrict__ first_dev) {
    __shared__ uint32_t hh[OSH_NH][OS_MAXP][OS_B];
    const int P = sort_passes(st);
    const uint64_t slo = st[ST_SLO], sh = st[ST_SH32];
    for (int i = threadIdx.x; i < OSH_NH * OS_MAXP * OS_B; i += OSH_NT) (&hh[0][0][0])[i] = 0;
    __syncthreads();
    uint32_t (*h)[OS_B] = hh[SB_OSH_WH ? ((threadIdx.x >> 6) % OSH_NH) : 0];
    const uint64_t lt = lanemask_lt();
    const int64_t stride = (int64_t)gridDim.x * OSH_NT;
    const int64_t i_lo = first_dev ? (int64_t)*first_dev : 0;
    for (int64_t i0 = i_lo + (int64_t)blockIdx.x * OSH_NT + threadIdx.x; i0 - threadIdx.x < n; i0 += stride * OS_IPT) {
        uint64_t kk[OS_IPT];
#pragma unroll
        for (int r = 0; r < OS_IPT; r++) kk[r] = i0 + r * stride < n ? ~sort_prefix(keys[i0 + r * stride], slo, sh) : 0ull;
#pragma unroll
        for (int r = 0; r < OS_IPT; r++) {
            const bool valid = i0 + r * stride < n;
            if (!__ballot(valid)) break;
            for (int p = 0; p < P; p++) {
                const int b = valid ? (int)((kk[r] >> os_shift(st, p)) & os_mask(st, p)) : -1;
                const uint64_t act = __ballot(b >= 0);
                const int b0 = __shfl(b, __builtin_ctzll(act), 64);
                const uint64_t same = __ballot(b == b0);
                if (b == b0) {
                    if ((same & lt) == 0) atomicAdd(&h[p][b0], (uint32_t)__popcll(same));
                } else if (b >= 0) {
                    atomicAdd(&h[p][b], 1u);
                }
            }
        }
    }
    __syncthreads();
    uint32_t* gh = reinterpret_cast<uint32_t*>(lb);
    for (int i = threadIdx.x; i < P * OS_B; i += OSH_NT) {
        uint32_t c = 0;
#pragma unroll
        for (int v = 0; v < OSH_NH; v++) c += (&hh[v][0][0])[i];
        if (SB_OSH_2STAGE) part[(size_t)blockIdx.x * OSH_ROW + i] = c;
        else if (c) atomicAdd(&gh[i], c);
    }
}
// column sums of the k_os_hist rows: grid (8, ceil(rows / OSH_RCHUNK)), thread = column
__global__ __launch_bounds__(256) void k_os_hsum(const uint32_t* __restrict__ part, int rows,
                                                 const uint64_t* __restrict__ st, uint64_t* __restrict__ lb) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    if (col >= sort_passes(st) * OS_B) return;
    const int r0 = blockIdx.y * OSH_RCHUNK;
    uint32_t c = 0;
#pragma unroll
    for (int r = 0; r < OSH_RCHUNK; r++)
        if (r0 + r < rows) c += part[(size_t)(r0 + r) * OSH_ROW + col];
    if (c) atomicAdd(reinterpret_cast<uint32_t*>(lb) + col, c);
}

// the tile's global offsets per digit: exclusive scan over the earlier tiles' published counts (look
// back over the predecessors, OS_LB granules polled together: add counts until the first inclusive one;
// wait where a predecessor has not published yet) plus the global start of the digit
// The granules' epoch (bits 34..63) is ebase + pass + 1: ebase advances by 8 every sort call, so granules left
// by earlier calls never match and the look-back buffer needs no clearing per call (SB_OS_EPOCH)
// The thread owns OS_DPT consecutive digits d0 ..: their look-backs run together (every poll of a round issued
// before any is used).
__device__ __forceinline__ void os_lookback(uint64_t* lb, int64_t tile, int p, const uint32_t* agg, int d0,
                                            uint32_t ebase, uint32_t* excl) {
    const uint64_t epv = (uint64_t)ebase + (uint64_t)(p + 1);
    const uint64_t ep = epv << 34;
    uint64_t* mine = lb + OS_HDR + tile * OS_B + d0;
#pragma unroll
    for (int k = 0; k < OS_DPT; k++) excl[k] = 0;
    if (tile == 0 || (SB_OS_DBG & 1)) {   // DBG 1 (timing only): no look-back
#pragma unroll
        for (int k = 0; k < OS_DPT; k++) os_publish(mine + k, ep | OS_INC | agg[k]);
        return;
    }
#pragma unroll
    for (int k = 0; k < OS_DPT; k++) os_publish(mine + k, ep | OS_AGG | agg[k]);
    int64_t j[OS_DPT];
    bool done[OS_DPT];
#pragma unroll
    for (int k = 0; k < OS_DPT; k++) {
        j[k] = tile - 1;
        done[k] = false;
    }
    int left = OS_DPT;
    uint32_t spins = 0;
    while (left > 0) {
        uint64_t v[OS_DPT][OS_LB];
#pragma unroll
        for (int k = 0; k < OS_DPT; k++)
#pragma unroll
            for (int u = 0; u < OS_LB; u++)
                v[k][u] = !done[k] && j[k] - u >= 0 ? os_poll(lb + OS_HDR + (j[k] - u) * OS_B + d0 + k) : (ep | OS_INC);
        bool stalled = false;
#pragma unroll
        for (int k = 0; k < OS_DPT; k++) {
            if (done[k]) continue;
            int u = 0;
            for (; u < OS_LB; u++) {
                if ((v[k][u] >> 34) != epv) break;
                excl[k] += (uint32_t)v[k][u];
                if (v[k][u] & OS_INC) {
                    done[k] = true;
                    left--;
                    break;
                }
            }
            if (!done[k]) {
                j[k] -= u;
                stalled |= u < OS_LB;
            }
        }
        if (stalled && ++spins > OS_SPIN_MAX) {   // bounded: a lost predecessor shows up as an error, not a hang
            atomicOr(reinterpret_cast<uint32_t*>(lb + OS_ERR), 1u);
            break;
        }
    }
#pragma unroll
    for (int k = 0; k < OS_DPT; k++) os_publish(mine + k, ep | OS_INC | (uint64_t)(excl[k] + agg[k]));
}

// Wave-sequential ranking: wave w owns the contiguous sub-tile [w * 64 * OS_IPT, (w + 1) * 64 * OS_IPT) of
// the tile and walks it 64 elements per round (coalesced loads); per round a wave match (8 ballots) groups
// equal digits, the group leader adds the group size to the wave's running count of that digit (an LDS
// atomic that returns the count before) and the group shares it — the element's rank among the wave's
// equal digits in index order.  A digit's offset in the tile is the sum of the earlier waves' counts.
#ifndef SB_OS_WAVES
#define SB_OS_WAVES 0   // 0: the compiler's register choice (155 VGPRs: 3 waves per SIMD).  4 (128 VGPRs, a 104 B
                        // spill) measured slower: 257 -> 341 us per step (profiles/r3/s5/ab_sort_digits.txt)
#endif
// M (the pass's way to its tiles' offsets): 0 the decoupled look-back (default); 1 count only (each tile's per-digit
// counts to tcnt[digit][tile], no scatter); 2 scatter with tcnt scanned over the tiles (k_os_tscan) — the
// two-level variant (SB_OS_TWOLEVEL), measured slower: profiles/r4/s2/sort_twolevel_ab.txt
template <int M>
__global__ __launch_bounds__(OS_PNT, SB_OS_WAVES) void k_os_pass(uint64_t* k0, uint32_t* v0, uint64_t* k1, uint32_t* v1, int64_t n,
                                                   int p, const uint64_t* __restrict__ st, uint64_t* __restrict__ lb,
                                                   uint32_t ebase, uint32_t* __restrict__ tcnt) {
    if (p >= sort_passes(st)) return;
    const uint64_t* kin = (p & 1) ? k1 : k0;
    const uint32_t* vin = (p & 1) ? v1 : v0;
    uint64_t* kout = (p & 1) ? k0 : k1;
    uint32_t* vout = (p & 1) ? v0 : v1;
    __shared__ uint32_t wcnt[OS_NW][OS_B];   // running digit counts per wave, then exclusive offsets in the tile
    __shared__ uint32_t sbase[OS_B];
    __shared__ uint32_t lds[OS_NW + 1];
    __shared__ uint32_t s_tile;
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    uint32_t* ticket = reinterpret_cast<uint32_t*>(lb + OS_TICKET);
    const int64_t ntiles = (n + OS_TILE - 1) / OS_TILE;
    const int shift = os_shift(st, p);
    const uint32_t dmask = os_mask(st, p);
    const uint64_t slo = st[ST_SLO], psh = st[ST_SH32];
    const uint64_t lt = lanemask_lt();
    const uint32_t* gh = reinterpret_cast<const uint32_t*>(lb) + p * OS_B;
    for (int it = 0;; it++) {
        if (M == 0 && t == 0)
            s_tile = (SB_OS_DBG & 4) ? (it ? 0xFFFFFFFFu : blockIdx.x) : atomicAdd(&ticket[p], 1u);   // DBG 4: block order
        for (int i = t; i < OS_NW * OS_B; i += OS_PNT) (&wcnt[0][0])[i] = 0;
        __syncthreads();
        const int64_t tile = M == 0 ? (int64_t)s_tile : (int64_t)blockIdx.x + (int64_t)it * gridDim.x;
        if (tile >= ntiles) return;
        const int64_t base = tile * OS_TILE + (int64_t)w * (64 * OS_IPT) + l;
        uint64_t kk[OS_IPT];
        uint32_t vv[OS_IPT];
        uint32_t rk[OS_IPT];   // digit | rank among the wave's equal digits << OS_D
#pragma unroll
        for (int r = 0; r < OS_IPT; r++) {
            const int64_t i = base + (int64_t)r * 64;
            kk[r] = i < n ? kin[i] : 0ull;
            vv[r] = M != 1 && i < n ? vin[i] : 0u;
        }
#pragma unroll
        for (int r = 0; r < OS_IPT; r++) {
            const bool valid = base + (int64_t)r * 64 < n;
            const uint32_t d = (uint32_t)(((~sort_prefix(kk[r], slo, psh)) >> shift) & dmask);
            uint64_t peers = __ballot(valid);
#pragma unroll
            for (int b = 0; b < OS_D; b++) {
                const uint64_t bb = __ballot((d >> b) & 1);
                peers &= ((d >> b) & 1) ? bb : ~bb;
            }
            const int leader = valid ? __builtin_ctzll(peers) : l;
            uint32_t before = 0;
            if (valid && leader == l) before = atomicAdd(&wcnt[w][d], (uint32_t)__popcll(peers));
            before = __shfl(before, leader, 64);
            rk[r] = d | ((before + (uint32_t)__popcll(peers & lt)) << OS_D);
        }
        __syncthreads();
        // thread t owns digits t * OS_DPT ..: the waves' exclusive offsets and the tile aggregates
        const int d0 = t * OS_DPT;
        uint32_t agg[OS_DPT], excl[OS_DPT], gv[OS_DPT], gsum = 0;
#pragma unroll
        for (int k = 0; k < OS_DPT; k++) {
            uint32_t a = 0;
#pragma unroll
            for (int x = 0; x < OS_NW; x++) {
                const uint32_t c = wcnt[x][d0 + k];
                wcnt[x][d0 + k] = a;
                a += c;
            }
            agg[k] = a;
            gv[k] = gh[d0 + k];
            gsum += gv[k];
        }
        if constexpr (M == 1) {   // count only: the tile's per-digit counts, digit-major for the scan over tiles
#pragma unroll
            for (int k = 0; k < OS_DPT; k++) tcnt[(int64_t)(d0 + k) * ntiles + tile] = agg[k];
            __syncthreads();   // the next tile rewrites wcnt
            continue;
        }
        if constexpr (M == 2) {
#pragma unroll
            for (int k = 0; k < OS_DPT; k++) excl[k] = tcnt[(int64_t)(d0 + k) * ntiles + tile];
        } else {
            os_lookback(lb, tile, p, agg, d0, ebase, excl);
        }
        uint32_t tot;
        uint32_t run = block_excl_scan<OS_PNT>(gsum, lds, &tot);   // global start of each digit
#pragma unroll
        for (int k = 0; k < OS_DPT; k++) {
            sbase[d0 + k] = run + excl[k];
            run += gv[k];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < OS_IPT; r++) {
            const int64_t i = base + (int64_t)r * 64;
            if (i < n) {
                const uint32_t d = rk[r] & (OS_B - 1);
                const uint32_t o = (SB_OS_DBG & 2) ? (uint32_t)i : sbase[d] + wcnt[w][d] + (rk[r] >> OS_D);
                kout[o] = kk[r];
                vout[o] = vv[r];
            }
        }
        __syncthreads();   // the next tile rewrites wcnt / sbase
    }
}

// the per-digit counts of k_os_pass<1> scanned over the tiles in place (exclusive): a wave per digit, each lane
// a contiguous run of tiles
__global__ __launch_bounds__(256) void k_os_tscan(uint32_t* __restrict__ tcnt, int64_t ntiles, int p,
                                                  const uint64_t* __restrict__ st) {
    if (p >= sort_passes(st)) return;
    const int lane = threadIdx.x & 63;
    const int d = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (d >= OS_B) return;
    uint32_t* c = tcnt + (int64_t)d * ntiles;
    const int64_t per = (ntiles + 63) / 64, a = lane * per, b = a + per < ntiles ? a + per : ntiles;
    uint32_t sum = 0;
    for (int64_t i = a; i < b; i++) sum += c[i];
    uint32_t run = wave_incl_scan(sum) - sum;
    for (int64_t i = a; i < b; i++) {
        const uint32_t v = c[i];
        c[i] = run;
        run += v;
    }
}

// ---- exact fix-up of the 40-bit-prefix sort.  Sorted output = (prefix desc, input order); the required
// order is (key desc, input order) — input order is next_queue order among equal keys (the select writes
// each key set in index order).  k_fx_mark lists the positions whose prefix equals the predecessor's but
// whose key does not; k_fx_fix claims each such position's run of equal prefixes once (epoch-stamped run
// marks), counts its distinct keys (an LDS set; a run holds a handful), and places every element at
// start(its key, in descending key order) + its rank among equal keys in run order — one wave, 64
// elements per round, so the placement is stable — through the other ping-pong buffer.
constexpr int FX_NT = 256;
constexpr int FX_SET = 1024;   // distinct keys per run (more sets error bit 32: never expected)
constexpr int FX_LIST = 256;   // distinct keys placed by the compact start computation

// out (SB_FX_COPY): the sorted payloads are copied to out here (k_fx_fix rewrites the runs it re-places), and
// the look-back's spin-limit flag is reported — k_copy_idx's work without its launch
__global__ __launch_bounds__(256) void k_fx_mark(const uint64_t* k0, const uint64_t* k1, int64_t m, uint64_t* st,
                                                 uint32_t* __restrict__ list, const uint32_t* v0, const uint32_t* v1,
                                                 uint32_t* __restrict__ out, const uint64_t* lb, uint32_t* err) {
    const int P = sort_passes(st);
    const uint64_t* kf = (P & 1) ? k1 : k0;
    const uint64_t slo = st[ST_SLO], sh = st[ST_SH32];
    if (out) {
        if (err && blockIdx.x == 0 && threadIdx.x == 0 && lb[OS_ERR]) atomicOr(err, 4u);
        const uint32_t* vf = (P & 1) ? v1 : v0;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
            out[i] = vf[i];
    }
    if (sh == 0) return;   // the prefix is the whole key: nothing to fix
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + 1; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t a = kf[i - 1], b = kf[i];
        if (a != b && sort_prefix(a, slo, sh) == sort_prefix(b, slo, sh)) {
            const uint64_t j = atomicAdd((unsigned long long*)&st[ST_FXN], 1ull);
            list[j] = (uint32_t)i;
        }
    }
}

// deferred (k_fx_wave ran first): list = the starts of the runs it claimed but left (too many distinct keys),
// counted in ST_FX2N — no claim here
__global__ __launch_bounds__(FX_NT) void k_fx_fix(uint64_t* k0, uint32_t* v0, uint64_t* k1, uint32_t* v1, uint32_t* out, int64_t m,
                                                  uint64_t* st, const uint32_t* __restrict__ list,
                                                  uint32_t* __restrict__ runmark, uint32_t epoch, uint32_t* err,
                                                  int deferred = 0) {
    const int P = sort_passes(st);
    uint64_t* kf = (P & 1) ? k1 : k0;
    uint32_t* vf = (P & 1) ? v1 : v0;
    uint64_t* ka = (P & 1) ? k0 : k1;   // the other buffer: scratch for the run
    uint32_t* va = (P & 1) ? v0 : v1;
    const uint64_t slo = st[ST_SLO], sh = st[ST_SH32], nflag = st[deferred ? ST_FX2N : ST_FXN];
    const int ticket = deferred ? ST_FX2I : ST_FXI;
    __shared__ uint64_t skey[FX_SET];
    __shared__ uint32_t scnt[FX_SET], sstart[FX_SET];
    __shared__ uint64_t lkey[FX_LIST];
    __shared__ uint32_t lslot[FX_LIST];
    __shared__ uint64_t sa, sb, sj;
    __shared__ uint32_t go, nd;
    const int t = threadIdx.x;
    for (;;) {
        if (t == 0) sj = atomicAdd((unsigned long long*)&st[ticket], 1ull);
        __syncthreads();
        const uint64_t j = sj;
        if (j >= nflag) return;
        const int64_t i = list[j];
        const uint64_t pre = sort_prefix(kf[i], slo, sh);
        // the run [a, b) of equal prefixes around i: the block walks out 256 positions at a time
        if (t == 0) {
            sa = (uint64_t)i;
            sb = (uint64_t)i + 1;
        }
        __syncthreads();
        for (int64_t base = i - 1;; base -= FX_NT) {
            const int64_t q = base - t;
            const bool same = q >= 0 && sort_prefix(kf[q], slo, sh) == pre;
            if (same) atomicMin((unsigned long long*)&sa, (unsigned long long)q);
            const int any_out = __syncthreads_or(!same);
            if (any_out) break;
        }
        for (int64_t base = i + 1;; base += FX_NT) {
            const int64_t q = base + t;
            const bool same = q < m && sort_prefix(kf[q], slo, sh) == pre;
            if (same) atomicMax((unsigned long long*)&sb, (unsigned long long)(q + 1));
            const int any_out = __syncthreads_or(!same);
            if (any_out) break;
        }
        // claim the run once per sort call (several flagged positions can share it)
        if (t == 0) {
            uint32_t old = runmark[sa];
            go = deferred;   // a deferred run was claimed by the wave that listed it
            while (!deferred && old != epoch) {
                const uint32_t got = atomicCAS(&runmark[sa], old, epoch);
                if (got == old) {
                    go = 1;
                    break;
                }
                old = got;
            }
            nd = 0;
        }
        __syncthreads();
        if (!go) continue;
        const int64_t a = (int64_t)sa, b = (int64_t)sb;
        const uint64_t none = kf[a] ^ (1ull << 63);   // no key of the run: they lie within 2^32 of each other
        for (int x = t; x < FX_SET; x += FX_NT) {
            skey[x] = none;
            scnt[x] = 0;
        }
        __syncthreads();
        // distinct keys of the run and their counts (an LDS set, linear probing on the key)
        for (int64_t q = a + t; q < b; q += FX_NT) {
            const uint64_t k = kf[q];
            uint32_t h = (uint32_t)(k ^ (k >> 29)) & (FX_SET - 1);
            for (int probe = 0;; probe++) {
                if (probe == FX_SET) {
                    if (err) atomicOr(err, 32u);
                    break;
                }
                const unsigned long long prev = atomicCAS((unsigned long long*)&skey[h], (unsigned long long)none,
                                                          (unsigned long long)k);
                if (prev == none || prev == k) {
                    atomicAdd(&scnt[h], 1u);
                    break;
                }
                h = (h + 1) & (FX_SET - 1);
            }
        }
        __syncthreads();
        // start of each distinct key in the run: elements with a larger key come first
        for (int x = t; x < FX_SET; x += FX_NT)   // the distinct keys, compacted
            if (scnt[x]) {
                const uint32_t e = atomicAdd(&nd, 1u);
                if (e < FX_LIST) {
                    lkey[e] = skey[x];
                    lslot[e] = (uint32_t)x;
                } else if (err) {
                    atomicOr(err, 32u);
                }
            }
        __syncthreads();
        const uint32_t nl = nd < FX_LIST ? nd : FX_LIST;
        for (uint32_t e = t; e < nl; e += FX_NT) {   // elements with a larger key come first
            uint32_t before = 0;
            for (uint32_t f = 0; f < nl; f++)
                if (lkey[f] > lkey[e]) before += scnt[lslot[f]];
            sstart[lslot[e]] = before;
        }
        __syncthreads();
        for (uint32_t e = t; e < nl; e += FX_NT) scnt[lslot[e]] = 0;   // the running count of placed elements
        __syncthreads();
        if (t < 64) {   // one wave places the run in order, 64 elements per round: stable
            const uint64_t lt = (t ? (1ull << t) - 1 : 0ull);
            for (int64_t q0 = a; q0 < b; q0 += 64) {
                const int64_t q = q0 + t;
                const bool valid = q < b;
                uint64_t k = 0;
                int slot = -1;
                if (valid) {
                    k = kf[q];
                    uint32_t h = (uint32_t)(k ^ (k >> 29)) & (FX_SET - 1);
                    while (skey[h] != k) h = (h + 1) & (FX_SET - 1);
                    slot = (int)h;
                }
                uint64_t peers = __ballot(valid);
#pragma unroll
                for (int bit = 0; bit < 10; bit++) {
                    const uint64_t bb = __ballot((slot >> bit) & 1);
                    peers &= ((slot >> bit) & 1) ? bb : ~bb;
                }
                if (valid) {
                    const uint32_t rank = (uint32_t)__popcll(peers & lt);
                    const int64_t dst = a + sstart[slot] + scnt[slot] + rank;
                    ka[dst] = k;
                    va[dst] = vf[q];
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                if (valid && (peers & lt) == 0) scnt[slot] += (uint32_t)__popcll(peers);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            }
        }
        __syncthreads();
        for (int64_t q = a + t; q < b; q += FX_NT) {
            kf[q] = ka[q];
            vf[q] = va[q];
            if (out) out[q] = va[q];
        }
        __syncthreads();
    }
}

// Fix-up, a wave per flagged position (ahead of k_fx_fix): the wave finds the run of equal prefixes around it
// (64 positions per step), claims it, lists its distinct keys with their counts (ballots: a run holds a
// handful), and places every element at start(its key, descending) + its rank among equal keys in run order,
// writing the payloads to out.  A run with more than FXW_MAXD distinct keys goes to k_fx_fix (deferred).
// Every run is worked on by one wave, in parallel: a workgroup per run in turn (k_fx_fix alone) made prefixes
// shorter than 40 bits cost more than the LSD pass they save.
constexpr int FXW_MAXD = 32;
__global__ __launch_bounds__(256) void k_fx_wave(const uint64_t* __restrict__ k0, const uint32_t* __restrict__ v0,
                                                 const uint64_t* __restrict__ k1, const uint32_t* __restrict__ v1,
                                                 uint32_t* __restrict__ out, int64_t m, uint64_t* st,
                                                 const uint32_t* __restrict__ list, uint32_t* __restrict__ list2,
                                                 uint32_t* __restrict__ runmark, uint32_t epoch) {
    const int P = sort_passes(st);
    const uint64_t* kf = (P & 1) ? k1 : k0;
    const uint32_t* vf = (P & 1) ? v1 : v0;
    const uint64_t slo = st[ST_SLO], sh = st[ST_SH32], nflag = st[ST_FXN];
    const int lane = threadIdx.x & 63;
    const uint64_t lt = lanemask_lt();
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t j = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); j < (int64_t)nflag; j += nw) {
        const int64_t i = list[j];
        const uint64_t pre = sort_prefix(kf[i], slo, sh);
        int64_t a = -1, b = -1;
        for (int64_t base = i - 1; a < 0; base -= 64) {   // lane l looks at base - l
            const int64_t q = base - lane;
            const bool same = q >= 0 && sort_prefix(kf[q], slo, sh) == pre;
            const uint64_t ns = __ballot(!same);
            if (ns) a = base - __builtin_ctzll(ns) + 1;
        }
        for (int64_t base = i + 1; b < 0; base += 64) {
            const int64_t q = base + lane;
            const bool same = q < m && sort_prefix(kf[q], slo, sh) == pre;
            const uint64_t ns = __ballot(!same);
            if (ns) b = base + __builtin_ctzll(ns);
        }
        int go = 0;
        if (lane == 0) {
            uint32_t old = runmark[a];
            while (old != epoch) {
                const uint32_t got = atomicCAS(&runmark[a], old, epoch);
                if (got == old) {
                    go = 1;
                    break;
                }
                old = got;
            }
        }
        if (!__builtin_amdgcn_readfirstlane(go)) continue;
        // distinct keys: lane d holds the d-th one found and its count
        uint64_t dk = 0;
        uint32_t dc = 0;
        int nd = 0;
        bool over = false;
        for (int64_t q0 = a; q0 < b && !over; q0 += 64) {
            const int64_t q = q0 + lane;
            const bool valid = q < b;
            const uint64_t k = valid ? kf[q] : 0ull;
            uint64_t left = __ballot(valid);
            for (int d = 0; d < nd; d++) {
                const uint64_t kd = __shfl(dk, d, 64);
                const uint64_t mm = __ballot(valid && k == kd);
                if (lane == d) dc += (uint32_t)__popcll(mm);
                left &= ~mm;
            }
            while (left) {
                if (nd == FXW_MAXD) {
                    over = true;
                    break;
                }
                const uint64_t kd = __shfl(k, __builtin_ctzll(left), 64);
                const uint64_t mm = __ballot(valid && k == kd);
                if (lane == nd) {
                    dk = kd;
                    dc = (uint32_t)__popcll(mm);
                }
                nd++;
                left &= ~mm;
            }
        }
        if (over) {   // claimed: k_fx_fix places it without claiming
            if (lane == 0) list2[atomicAdd((unsigned long long*)&st[ST_FX2N], 1ull)] = (uint32_t)a;
            continue;
        }
        uint32_t start = 0, run = 0;   // lane d: elements with a larger key; elements of key d placed so far
        for (int d = 0; d < nd; d++) {
            const uint64_t kd = __shfl(dk, d, 64);
            const uint32_t cd = (uint32_t)__shfl((int)dc, d, 64);
            if (lane < nd && kd > dk) start += cd;
        }
        for (int64_t q0 = a; q0 < b; q0 += 64) {
            const int64_t q = q0 + lane;
            const bool valid = q < b;
            const uint64_t k = valid ? kf[q] : 0ull;
            const uint32_t v = valid ? vf[q] : 0u;
            int64_t dst = -1;
            for (int d = 0; d < nd; d++) {
                const uint64_t kd = __shfl(dk, d, 64);
                const uint64_t mm = __ballot(valid && k == kd);
                const uint32_t sd = (uint32_t)__shfl((int)start, d, 64), rd = (uint32_t)__shfl((int)run, d, 64);
                if (valid && k == kd) dst = a + sd + rd + __popcll(mm & lt);
                if (lane == d) run += (uint32_t)__popcll(mm);
            }
            if (valid) out[dst] = v;
        }
    }
}

__global__ void k_copy_idx(const uint32_t* v0, const uint32_t* v1, const uint64_t* st, uint32_t* out, int64_t n,
                           const uint64_t* lb, uint32_t* err) {
    if (err && blockIdx.x == 0 && threadIdx.x == 0 && lb[OS_ERR]) atomicOr(err, 4u);
    const uint32_t* in = (sort_passes(st) & 1) ? v1 : v0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

static unsigned grid_for(int64_t n, int nt, unsigned cap = 8192) {
    int64_t g = (n + nt - 1) / nt;
    if (g < 1) g = 1;
    return (unsigned)(g < cap ? g : cap);
}

void TopkScratch::release() {
    k0.release();
    k1.release();
    v0.release();
    v1.release();
    ck.release();
    ci.release();
    os.release();
    tile_a.release();
    tile_b.release();
    small.release();
    fx_list.release();
    fx_mark.release();
    fx_list2.release();
    os_tcnt.release();
    if (h_nc) (void)hipHostFree(h_nc);
    if (nc_ev) (void)hipEventDestroy(nc_ev);
    h_nc = nullptr;
    nc_ev = nullptr;
    nc_pending = false;
    osh_part.release();
    tkh_part.release();
    sk.release();
    si.release();
}

// before the producer of a turn's keys runs: reset the key range; with fused = 1 also place the fused
// first-pass window (from the previous turn's maximum: its top bin sits 64 bins (two binades) above
// it) and zero the histogram the producer adds to
__global__ void k_tk_range_reset(uint64_t* st, int fused, int off_window, uint32_t* fill_ff, int fill_n) {
    if (fill_ff)   // the caller's fill_n-word table (the gather's first ranks)
        for (int i = threadIdx.x; i < fill_n; i += blockDim.x) fill_ff[i] = 0xFFFFFFFFu;
    if (threadIdx.x == 0) {
        if (fused) {
            int64_t b0;
            if (SB_SEL_FSH == 47) {   // 64 binades centred on the threshold two selects back (ST_T2).  Round 3 hung the
                                      // window two binades above the previous maximum; C4's players alternate, so its
                                      // threshold flips sign every turn (order keys 2^63 apart) and that, or the
                                      // previous threshold, left C4 in fallback
                b0 = st[ST_T2] ? (int64_t)(st[ST_T2] >> 47) - SEL_BINS / 2
                               : (int64_t)(st[ST_MAX] >> 47) + 64 - (SEL_BINS - 1);
                st[ST_T2] = st[ST_SLO];   // the previous select's lowest kept key: two selects back at the next reset
            } else {   // half a binade below the previous threshold (ST_SLO: the lowest kept key) to 1.5 above
                const uint64_t ref = st[ST_SLO] ? st[ST_SLO] : st[ST_MAX];
                b0 = (int64_t)(ref >> SB_SEL_FSH) - (int64_t)((1ull << 52) >> SB_SEL_FSH) / 2;
            }
            st[ST_FBASE] = off_window ? 0 : (b0 < 0 ? 0 : (uint64_t)b0);
        }
        st[ST_MIN] = ~0ull;
        st[ST_MAX] = 0;
    }
    if (fused)
        for (int i = threadIdx.x; i < SEL_BINS; i += blockDim.x) st[ST_HIST + i] = 0;
}

void topk_reserve(TopkScratch& s, int64_t n, int64_t keep) {
    const int64_t m = n < keep ? n : keep;
    s.k0.ensure(m);
    s.k1.ensure(m);
    s.v0.ensure(m);
    s.v1.ensure(m);
    s.ck.ensure(n);
    s.ci.ensure(n);
    s.tile_a.ensure(n / TK_TILE + 1);
    s.tile_b.ensure(n / TK_TILE + 1);
    if (TK_STAGE && n > keep) {
        s.sk.ensure((size_t)(n / TK_TILE + 1) * TK_TILE);
        s.si.ensure((size_t)(n / TK_TILE + 1) * TK_TILE);
    }
    s.os.ensure((size_t)OS_HDR + (size_t)(m / OS_TILE + 1) * OS_B);
    s.small.ensure(ST_WORDS);
    s.fx_list.ensure((size_t)m);
    if (SB_OSH_2STAGE) s.osh_part.ensure((size_t)grid_for(m, OS_NT * OS_IPT, SB_OSH_GRID) * OSH_ROW);
    if (SB_TKH_2STAGE) s.tkh_part.ensure((size_t)grid_for(n, TK_NT * 16, SB_TKH_GRID) * SEL_BINS);
    if (s.fx_mark.cap < (size_t)m) {   // run marks start at epoch 0 (see topk_stable_desc)
        s.fx_mark.ensure((size_t)m);
        SB_HIP(hipMemset(s.fx_mark.p, 0, s.fx_mark.cap * 4));
        s.fx_epoch = 0;
    }
}

unsigned long long* topk_range_reset(TopkScratch& s, hipStream_t st, bool fused, bool off_window, uint32_t* fill_ff,
                                     int fill_n) {
    s.small.ensure(ST_WORDS);
    hipLaunchKernelGGL(k_tk_range_reset, dim3(1), dim3(256), 0, st, s.small.p, (int)fused, (int)off_window, fill_ff, fill_n);
    return (unsigned long long*)(s.small.p + ST_MIN);
}

unsigned long long* topk_fused_hist(TopkScratch& s) { return (unsigned long long*)(s.small.p + ST_HIST); }
const uint64_t* topk_fused_base(TopkScratch& s) { return s.small.p + ST_FBASE; }

int64_t topk_stable_desc(const uint64_t* keys, int64_t n, int64_t keep, uint32_t* out_idx, TopkScratch& s,
                         hipStream_t st, bool range_ready, uint32_t* err, bool fused, const uint32_t* payload,
                         bool full_key) {
    if (n <= 0 || keep <= 0) return 0;
    const int64_t m = n < keep ? n : keep;
    // up to 2^21 kept keys a 30-bit prefix (three LSD passes): prefix collisions fall with the square of the count —
    // C4's 1M kept keys flag none at 30 bits, C3's 4M flag 40-90k and their fix-up costs more than the fourth pass
    // saves (profiles/r4/s2/sort_prefix_ab.txt)
#ifndef SB_SORT_SMALL_M
#define SB_SORT_SMALL_M (1 << 21)
#endif
    const int prefix_bits = full_key ? 64 : (m <= SB_SORT_SMALL_M && OS_PREFIX_BITS > 30 ? 30 : OS_PREFIX_BITS);
    s.k0.ensure(m);
    s.k1.ensure(m);
    s.v0.ensure(m);
    s.v1.ensure(m);
    s.small.ensure(ST_WORDS);
    uint64_t* stv = s.small.p;
    const bool selected = n > keep;
    // the sort's look-back buffer: granules of earlier calls carry older epochs (SB_OS_EPOCH), so it is cleared
    // only when (re)allocated or when the epochs wrap; its header is cleared with the sort's setup below
    const int64_t ntiles_s = (m + OS_TILE - 1) / OS_TILE;
    const size_t lb_words = (size_t)OS_HDR + (size_t)ntiles_s * OS_B;
    const size_t lb_cap = s.os.cap;
    s.os.ensure(lb_words);
    uint32_t ebase = 0;
    if (SB_OS_EPOCH) {
        if (s.os.cap != lb_cap || s.os_epoch >= (1u << 26)) {
            SB_HIP(hipMemsetAsync(s.os.p, 0, s.os.cap * 8, st));
            s.os_epoch = 0;
        }
        ebase = ++s.os_epoch * 8;
    }
    bool sort_begun = false;   // the setup + header clear rode on the final partition's scan
    if (fused && selected) {
        hipLaunchKernelGGL(k_tk_begin_fused, dim3(1), dim3(TK_NT), 0, st, stv, (int64_t)m, n);
    } else {
        hipLaunchKernelGGL(k_tk_init, dim3(1), dim3(TK_NT), 0, st, stv, (int64_t)m, (int)range_ready, (int)fused);
        if (!range_ready)
            hipLaunchKernelGGL(k_tk_minmax, dim3(grid_for(n, TK_NT * 8, SB_MINMAX_GRID)), dim3(TK_NT), 0, st, keys, n, stv);
        if (selected) hipLaunchKernelGGL(k_tk_setup, dim3(1), dim3(1), 0, st, stv);
    }
    if (selected) {
        const int64_t ntiles = (n + TK_TILE - 1) / TK_TILE;
        s.tile_a.ensure(ntiles);
        s.tile_b.ensure(ntiles);
        s.ck.ensure(n);
        s.ci.ensure(n);
        const unsigned hg = grid_for(n, TK_NT * 16, SB_TKH_GRID);
        // first digit over all keys (folded into the producer when fused, generic pass as fallback),
        // then partition: above -> output group 1, bucket -> candidates
        tk_hist_pick(s, st, keys, n, nullptr, stv, (int)fused, hg);
        // more digits over all keys before the partition: the scores crowd into few first-pass bins (about
        // half of C3's keys share the threshold's), so the partition would copy most keys as candidates
        // (with the fine fused bins, SB_SEL_FSH < 47, only after a fallback to the generic first pass)
        for (int e = 0; e < SEL_PREPASS; e++) {
            tk_hist_pick(s, st, keys, n, nullptr, stv, (fused && SB_SEL_FSH < 47) ? 1 : 0, hg);
        }
        const unsigned cg = (unsigned)std::min<int64_t>(ntiles, TK_COUNT_GRID);
        const unsigned wg = (unsigned)std::min<int64_t>(ntiles, TK_WRITE_GRID);
        if (TK_STAGE) {   // one read of the keys: staged per tile, then moved (k_tk_stage)
            s.sk.ensure((size_t)ntiles * TK_TILE);
            s.si.ensure((size_t)ntiles * TK_TILE);
            hipLaunchKernelGGL(k_tk_stage, dim3(cg), dim3(TK_NT), 0, st, keys, n, stv, s.tile_a.p, s.tile_b.p, s.sk.p,
                               s.si.p, payload);
            hipLaunchKernelGGL(k_tk_scan, dim3(1), dim3(1024), 0, st, s.tile_a.p, s.tile_b.p, n, (const uint64_t*)nullptr,
                               stv, (int)ST_A, (int)ST_NC, 0);
            hipLaunchKernelGGL(k_tk_unstage, dim3((unsigned)std::min<int64_t>((ntiles + 3) / 4, 8192)), dim3(256), 0, st,
                               s.sk.p, s.si.p, n, stv, s.tile_a.p, s.tile_b.p, s.k0.p, s.v0.p, s.ck.p, s.ci.p);
        } else {
            hipLaunchKernelGGL(k_tk_count, dim3(cg), dim3(TK_NT), 0, st, keys, n, (const uint64_t*)nullptr,
                               stv, s.tile_a.p, s.tile_b.p);
            hipLaunchKernelGGL(k_tk_scan, dim3(1), dim3(1024), 0, st, s.tile_a.p, s.tile_b.p, n, (const uint64_t*)nullptr,
                               stv, (int)ST_A, (int)ST_NC, 0);
            hipLaunchKernelGGL(k_tk_write, dim3(wg), dim3(TK_NT), 0, st, keys, (const uint32_t*)nullptr, n,
                               (const uint64_t*)nullptr, stv, s.tile_a.p, s.tile_b.p, s.k0.p, s.v0.p,
                               (const uint64_t*)nullptr, s.ck.p, s.ci.p, (const uint64_t*)nullptr,
                               (const uint64_t*)nullptr, payload);
        }
        // remaining digits on the candidates (device-side count; passes after DONE exit at once) — or the whole tail
        // in one workgroup when the previous select's candidates were few (the pinned count, read without a wait)
#ifndef SB_TK_TAIL_MAX
#define SB_TK_TAIL_MAX 4096
#endif
        bool tail = false;
        if (s.nc_pending && hipEventQuery(s.nc_ev) == hipSuccess) tail = *s.h_nc <= (uint64_t)SB_TK_TAIL_MAX;
        const uint64_t* nc = stv + ST_NC;
        if (tail) {
            hipLaunchKernelGGL(k_tk_tail, dim3(1), dim3(TT_NT), 0, st, s.ck.p, s.ci.p, stv, s.k0.p, s.v0.p,
                               SB_OS_EPOCH ? s.os.p : (uint64_t*)nullptr, (int)OS_HDR, prefix_bits);
            sort_begun = SB_OS_EPOCH;
        } else {
            for (int pass = 0; pass < SEL_PASSES_C; pass++) {
                tk_hist_pick(s, st, s.ck.p, n, nc, stv, 0, std::min(hg, (unsigned)SB_TK_CAND_GRID), true);
            }
            // candidates above T -> group 2, the first NEED ties -> group 3
            hipLaunchKernelGGL(k_tk_count, dim3(cg), dim3(TK_NT), 0, st, s.ck.p, n, nc, stv, s.tile_a.p, s.tile_b.p);
            hipLaunchKernelGGL(k_tk_scan, dim3(1), dim3(1024), 0, st, s.tile_a.p, s.tile_b.p, n, nc, stv, (int)ST_G2,
                               (int)ST_E2, 1, SB_OS_EPOCH ? s.os.p : (uint64_t*)nullptr, (int)OS_HDR, prefix_bits);
            sort_begun = SB_OS_EPOCH;
            hipLaunchKernelGGL(k_tk_write, dim3(wg), dim3(TK_NT), 0, st, s.ck.p, s.ci.p, n, nc, stv,
                               s.tile_a.p, s.tile_b.p, s.k0.p, s.v0.p, stv + ST_BASE2, s.k0.p, s.v0.p, stv + ST_BASE3,
                               stv + ST_NEED, (const uint32_t*)nullptr);
        }
        if (!s.h_nc) {
            SB_HIP(hipHostMalloc((void**)&s.h_nc, 8, hipHostMallocDefault));
            SB_HIP(hipEventCreateWithFlags(&s.nc_ev, hipEventDisableTiming));
        }
        SB_HIP(hipMemcpyAsync(s.h_nc, stv + ST_NC, 8, hipMemcpyDeviceToHost, st));
        SB_HIP(hipEventRecord(s.nc_ev, st));
        s.nc_pending = true;
    } else {
        hipLaunchKernelGGL(k_iota, dim3(grid_for(m, 256)), dim3(256), 0, st, s.v0.p, keys, s.k0.p, m, payload);
    }
#ifdef SB_DBG_EMPTY   // diagnostic: extra empty launches (kernel boundary cost)
    for (int e = 0; e < SB_DBG_EMPTY; e++) hipLaunchKernelGGL(k_tk_sortsetup, dim3(1), dim3(1), 0, st, stv, (int)selected, prefix_bits);
#endif
    const int64_t ntiles = ntiles_s;
    if (SB_OS_EPOCH) {
        if (!sort_begun) hipLaunchKernelGGL(k_os_begin, dim3(1), dim3(256), 0, st, stv, (int)selected, prefix_bits, s.os.p);
    } else {
        hipLaunchKernelGGL(k_tk_sortsetup, dim3(1), dim3(1), 0, st, stv, (int)selected, prefix_bits);
        SB_HIP(hipMemsetAsync(s.os.p, 0, lb_words * 8, st));
    }
    const unsigned ohg = grid_for(m, OSH_NT * OS_IPT, SB_OSH_GRID);
    if (SB_OSH_2STAGE) s.osh_part.ensure((size_t)ohg * OSH_ROW);
    hipLaunchKernelGGL(k_os_hist, dim3(ohg), dim3(OSH_NT), 0, st, s.k0.p, m, stv, s.os.p, s.osh_part.p,
                       (const uint64_t*)nullptr);
    if (SB_OSH_2STAGE)
        hipLaunchKernelGGL(k_os_hsum, dim3(OS_MAXP * OS_B / 256, (ohg + OSH_RCHUNK - 1) / OSH_RCHUNK), dim3(256), 0, st, s.osh_part.p,
                           (int)ohg, stv, s.os.p);
#ifndef SB_OS_GRID
#define SB_OS_GRID 1u << 20   // blocks per pass at most (tiles beyond are taken by ticket)
#endif
    const unsigned osg = (unsigned)std::min<int64_t>(ntiles, (int64_t)(SB_OS_GRID));
#ifndef SB_OS_TWOLEVEL
#define SB_OS_TWOLEVEL 0   // tiles from which a pass counts, scans and scatters (three launches, no look-back).  A/B at
                           // 256 (C3): count 19 + scan 5-7 + scatter 31-35 us per pass against ≈50 with the look-back,
                           // and the first pass's scatter alone 75-78 (select 0.585 -> 0.62 ms): the look-back is not
                           // what makes a pass slow, the scatter of 1024 digits is (profiles/r4/s2/sort_twolevel_ab.txt)
#endif
    const bool twolevel = SB_OS_TWOLEVEL > 0 && ntiles >= SB_OS_TWOLEVEL;
    if (twolevel) s.os_tcnt.ensure((size_t)OS_B * (size_t)ntiles);
    for (int p = 0; p < (prefix_bits + OS_D - 1) / OS_D; p++) {   // passes beyond the varying bits exit at once
        if (twolevel) {
            hipLaunchKernelGGL(k_os_pass<1>, dim3(osg), dim3(OS_PNT), 0, st, s.k0.p, s.v0.p, s.k1.p, s.v1.p, m, p,
                               stv, s.os.p, ebase, s.os_tcnt.p);
            hipLaunchKernelGGL(k_os_tscan, dim3(OS_B / 4), dim3(256), 0, st, s.os_tcnt.p, ntiles, p, stv);
            hipLaunchKernelGGL(k_os_pass<2>, dim3(osg), dim3(OS_PNT), 0, st, s.k0.p, s.v0.p, s.k1.p, s.v1.p, m, p,
                               stv, s.os.p, ebase, s.os_tcnt.p);
        } else {
            hipLaunchKernelGGL(k_os_pass<0>, dim3(osg), dim3(OS_PNT), 0, st, s.k0.p, s.v0.p, s.k1.p, s.v1.p, m, p,
                               stv, s.os.p, ebase, (uint32_t*)nullptr);
        }
    }
    // exact order among keys that share their 32-bit prefix
    if (s.fx_mark.cap < (size_t)m) {   // run claims carry this call's epoch: zeroed only when (re)allocated
        s.fx_mark.ensure((size_t)m);
        SB_HIP(hipMemsetAsync(s.fx_mark.p, 0, s.fx_mark.cap * 4, st));
        s.fx_epoch = 0;
    }
    const uint32_t epoch = ++s.fx_epoch;
    s.fx_list.ensure((size_t)m);
#ifndef SB_FX_COPY
#define SB_FX_COPY 1   // the payload copy to out_idx in k_fx_mark / k_fx_fix instead of a k_copy_idx launch
#endif
    uint32_t* fxo = SB_FX_COPY ? out_idx : nullptr;
    hipLaunchKernelGGL(k_fx_mark, dim3(grid_for(m, 256, 2048)), dim3(256), 0, st, s.k0.p, s.k1.p, m, stv, s.fx_list.p,
                       s.v0.p, s.v1.p, fxo, s.os.p, err);
#ifndef SB_FX_GRID
#define SB_FX_GRID 64   // fix-up workgroups (each takes flagged positions until none are left)
#endif
#ifndef SB_FX_WAVE
#define SB_FX_WAVE 1   // a wave per run first (k_fx_wave), k_fx_fix only for runs it defers
#endif
    if (SB_FX_WAVE && fxo) {
        s.fx_list2.ensure((size_t)m);
        hipLaunchKernelGGL(k_fx_wave, dim3(1024), dim3(256), 0, st, s.k0.p, s.v0.p, s.k1.p, s.v1.p, fxo, m, stv, s.fx_list.p,
                           s.fx_list2.p, s.fx_mark.p, epoch);
        hipLaunchKernelGGL(k_fx_fix, dim3(SB_FX_GRID), dim3(FX_NT), 0, st, s.k0.p, s.v0.p, s.k1.p, s.v1.p, fxo, m, stv,
                           s.fx_list2.p, s.fx_mark.p, epoch, err, 1);
    } else {
        hipLaunchKernelGGL(k_fx_fix, dim3(SB_FX_GRID), dim3(FX_NT), 0, st, s.k0.p, s.v0.p, s.k1.p, s.v1.p, fxo, m, stv,
                           s.fx_list.p, s.fx_mark.p, epoch, err, 0);
    }
    if (!fxo)
        hipLaunchKernelGGL(k_copy_idx, dim3(grid_for(m, 256)), dim3(256), 0, st, s.v0.p, s.v1.p, stv, out_idx, m, s.os.p, err);
    SB_HIP(hipGetLastError());
    static const bool stats = getenv("SB_TOPK_STATS") != nullptr;   // diagnostics: the select's counts (a host wait)
    if (stats && selected) {
        uint64_t h[ST_HIST];
        SB_HIP(hipMemcpyAsync(h, stv, sizeof(h), hipMemcpyDeviceToHost, st));
        SB_HIP(hipStreamSynchronize(st));
        fprintf(stderr, "topk n %lld keep %lld: above %llu candidates %llu above-T %llu ties %llu sh %llu fallback %llu "
                "bins: fbase %llu min %llu max %llu T %llu; sort passes %d, fix-up flagged %llu deferred %llu\n",
                (long long)n, (long long)keep, (unsigned long long)h[ST_A], (unsigned long long)h[ST_NC],
                (unsigned long long)h[ST_G2], (unsigned long long)h[ST_E2], (unsigned long long)h[ST_SH],
                (unsigned long long)h[ST_FALLBACK], (unsigned long long)h[ST_FBASE],
                (unsigned long long)(h[ST_MIN] >> 47), (unsigned long long)(h[ST_MAX] >> 47),
                (unsigned long long)(h[ST_SLO] >> 47), (int)((h[ST_TOPK] - h[ST_SH32] + OS_D - 1) / OS_D),
                (unsigned long long)h[ST_FXN], (unsigned long long)h[ST_FX2N]);
    }
    return m;
}

}  // namespace sb
