// sb_sort.hip — stable descending top-k of u64 score keys: the device form of
//   queue = sorted(next_queue, key=heuristic, reverse=True)[:beam_width]   (src/solver.py:452-456)
// sorted() is stable, so ties keep next_queue order (element index).  Scores are positive
// float64, so their IEEE bit patterns order like the values.
//
//   1. radix select (MSB-first 8-bit digits) finds the threshold bucket holding the keep-th key
//      and how many of its elements (first in index order) are kept;
//   2. an order-preserving compaction writes the kept (key, index) pairs in index order;
//   3. a stable LSD radix sort on ~key orders them; passes whose digit is constant are skipped.
#include "sb_block.h"
#include "sb_internal.h"

namespace sb {

constexpr int TK_NT = 256;
constexpr int TK_IPT = 16;
constexpr int TK_TILE = TK_NT * TK_IPT;   // 4096

// select state (device, u64 words): [0] prefix  [1] bits resolved  [2] need  [3] done
//                                  [4..4+256) pass histogram   [260..260+8*256) global digit hists
constexpr int SEL_HIST = 4;
constexpr int GH = 260;

__global__ void k_sel_init(uint64_t* st, int64_t keep) {
    int t = threadIdx.x;
    if (t == 0) {
        st[0] = 0;
        st[1] = 0;
        st[2] = (uint64_t)keep;
        st[3] = 0;
    }
    for (int i = t; i < 256 + 8 * 256; i += blockDim.x) st[SEL_HIST + i] = 0;
}

__global__ __launch_bounds__(TK_NT) void k_sel_hist(const uint64_t* __restrict__ keys, int64_t n, uint64_t* st) {
    if (st[3]) return;
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t prefix = st[0];
    const int bits = (int)st[1];
    for (int64_t i = (int64_t)blockIdx.x * TK_NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * TK_NT) {
        uint64_t k = keys[i];
        bool match = bits == 0 || (k >> (64 - bits)) == prefix;
        if (match) atomicAdd(&h[(k >> (56 - bits)) & 255], 1u);
    }
    __syncthreads();
    uint32_t c = h[threadIdx.x];
    if (c) atomicAdd((unsigned long long*)&st[SEL_HIST + threadIdx.x], (unsigned long long)c);
}

__global__ void k_sel_pick(uint64_t* st) {
    if (st[3] || threadIdx.x != 0) return;
    uint64_t need = st[2], cum = 0;
    int d = 255;
    for (; d > 0; d--) {
        uint64_t c = st[SEL_HIST + d];
        if (cum + c >= need) break;
        cum += c;
    }
    uint64_t c = st[SEL_HIST + d];
    need -= cum;
    st[0] = (st[0] << 8) | (uint64_t)d;
    st[1] += 8;
    st[2] = need;
    if (c == need || st[1] == 64) st[3] = 1;
    for (int i = 0; i < 256; i++) st[SEL_HIST + i] = 0;
}

// tile counts of keys strictly above / equal to the threshold prefix
__global__ __launch_bounds__(TK_NT) void k_sel_count(const uint64_t* __restrict__ keys, int64_t n,
                                                      const uint64_t* __restrict__ st, uint32_t* __restrict__ gt,
                                                      uint32_t* __restrict__ eq) {
    __shared__ uint32_t lds[TK_NT / 64 + 1];
    const uint64_t prefix = st[0];
    const int bits = (int)st[1];
    const int64_t base = (int64_t)blockIdx.x * TK_TILE;
    uint32_t a = 0, b = 0;
#pragma unroll
    for (int j = 0; j < TK_IPT; j++) {
        int64_t i = base + (int64_t)j * TK_NT + threadIdx.x;
        if (i < n) {
            uint64_t top = keys[i] >> (64 - bits);
            a += top > prefix;
            b += top == prefix;
        }
    }
    uint32_t ta, tb;
    block_excl_scan<TK_NT>(a, lds, &ta);
    block_excl_scan<TK_NT>(b, lds, &tb);
    if (threadIdx.x == 0) {
        gt[blockIdx.x] = ta;
        eq[blockIdx.x] = tb;
    }
}

// single workgroup: eq -> exclusive eq offsets; gt -> exclusive kept offsets
__global__ __launch_bounds__(1024) void k_sel_scan(uint32_t* __restrict__ gt, uint32_t* __restrict__ eq, int64_t ntiles,
                                                    const uint64_t* __restrict__ st) {
    __shared__ uint32_t lds[1024 / 64 + 1];
    const uint64_t m = st[2];
    uint32_t ceq = 0, ckept = 0;
    for (int64_t b = 0; b < ntiles; b += 1024) {
        int64_t i = b + threadIdx.x;
        uint32_t g = i < ntiles ? gt[i] : 0, e = i < ntiles ? eq[i] : 0;
        uint32_t te;
        uint32_t ex_e = block_excl_scan<1024>(e, lds, &te) + ceq;
        uint64_t take = ex_e >= m ? 0 : (m - ex_e < e ? m - ex_e : e);
        uint32_t kept = g + (uint32_t)take, tk;
        uint32_t ex_k = block_excl_scan<1024>(kept, lds, &tk) + ckept;
        if (i < ntiles) {
            eq[i] = ex_e;
            gt[i] = ex_k;
        }
        ceq += te;
        ckept += tk;
    }
}

__global__ __launch_bounds__(TK_NT) void k_sel_write(const uint64_t* __restrict__ keys, int64_t n,
                                                      const uint64_t* __restrict__ st, const uint32_t* __restrict__ kept_off,
                                                      const uint32_t* __restrict__ eq_off, uint64_t* __restrict__ okeys,
                                                      uint32_t* __restrict__ oidx) {
    __shared__ uint32_t lds[TK_NT / 64 + 1];
    const uint64_t prefix = st[0];
    const int bits = (int)st[1];
    const uint64_t m = st[2];
    const int64_t base = (int64_t)blockIdx.x * TK_TILE + (int64_t)threadIdx.x * TK_IPT;   // blocked order
    uint64_t k[TK_IPT];
    uint32_t ne = 0;
#pragma unroll
    for (int j = 0; j < TK_IPT; j++) {
        int64_t i = base + j;
        k[j] = i < n ? keys[i] : 0;
        uint64_t top = k[j] >> (64 - bits);
        ne += (i < n) & (top == prefix);
    }
    uint32_t t;
    uint32_t eq_run = block_excl_scan<TK_NT>(ne, lds, &t) + eq_off[blockIdx.x];
    // kept count of this thread depends on eq_run; compute then scan
    uint32_t kc = 0;
    {
        uint32_t er = eq_run;
#pragma unroll
        for (int j = 0; j < TK_IPT; j++) {
            int64_t i = base + j;
            if (i >= n) break;
            uint64_t top = k[j] >> (64 - bits);
            if (top > prefix) kc++;
            else if (top == prefix) { kc += er < m; er++; }
        }
    }
    uint32_t out = block_excl_scan<TK_NT>(kc, lds, &t) + kept_off[blockIdx.x];
#pragma unroll
    for (int j = 0; j < TK_IPT; j++) {
        int64_t i = base + j;
        if (i >= n) break;
        uint64_t top = k[j] >> (64 - bits);
        bool keep = top > prefix;
        if (top == prefix) { keep = eq_run < m; eq_run++; }
        if (keep) {
            okeys[out] = k[j];
            oidx[out] = (uint32_t)i;
            out++;
        }
    }
}

__global__ void k_iota(uint32_t* v, const uint64_t* keys, uint64_t* okeys, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        v[i] = (uint32_t)i;
        okeys[i] = keys[i];
    }
}

// global digit histograms of ~key for all 8 LSD passes (constant-digit detection)
__global__ __launch_bounds__(TK_NT) void k_sort_ghist(const uint64_t* __restrict__ keys, int64_t n, uint64_t* st) {
    __shared__ uint32_t h[8][256];
    for (int i = threadIdx.x; i < 8 * 256; i += TK_NT) (&h[0][0])[i] = 0;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * TK_NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * TK_NT) {
        uint64_t k = ~keys[i];
#pragma unroll
        for (int p = 0; p < 8; p++) atomicAdd(&h[p][(k >> (8 * p)) & 255], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 8 * 256; i += TK_NT) {
        uint32_t c = (&h[0][0])[i];
        if (c) atomicAdd((unsigned long long*)&st[GH + i], (unsigned long long)c);
    }
}

__global__ void k_sort_flags(const uint64_t* st, int64_t n, uint32_t* flags) {
    int p = threadIdx.x;   // 8 threads
    if (p >= 8) return;
    uint32_t constant = 0;
    for (int d = 0; d < 256; d++)
        if (st[GH + p * 256 + d] == (uint64_t)n) constant = 1;
    flags[p] = constant;
}

// per-tile histogram of digit (~key >> shift) & 255, column-major [digit][tile]
__global__ __launch_bounds__(TK_NT) void k_sort_hist(const uint64_t* __restrict__ keys, int64_t n, int shift,
                                                      uint32_t* __restrict__ hist, int64_t ntiles) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * TK_TILE;
#pragma unroll
    for (int j = 0; j < TK_IPT; j++) {
        int64_t i = base + (int64_t)j * TK_NT + threadIdx.x;
        if (i < n) atomicAdd(&h[((~keys[i]) >> shift) & 255], 1u);
    }
    __syncthreads();
    hist[(int64_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// stable scatter: tile elements processed in index order, rank among equal digits by
// wave match (8 ballots) + per-wave LDS counts.
__global__ __launch_bounds__(TK_NT) void k_sort_scatter(const uint64_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                         uint64_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                         int64_t n, int shift, const uint32_t* __restrict__ hist,
                                                         int64_t ntiles) {
    __shared__ uint32_t base_d[256];
    __shared__ uint32_t wcnt[TK_NT / 64][256];
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    base_d[t] = hist[(int64_t)t * ntiles + blockIdx.x];
    const int64_t tile = (int64_t)blockIdx.x * TK_TILE;
    for (int r = 0; r < TK_IPT; r++) {
        for (int x = 0; x < TK_NT / 64; x++) wcnt[x][t] = 0;
        __syncthreads();
        int64_t i = tile + (int64_t)r * TK_NT + t;
        bool valid = i < n;
        uint64_t k = valid ? kin[i] : 0;
        uint32_t v = valid ? vin[i] : 0;
        uint32_t d = (uint32_t)(((~k) >> shift) & 255);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            uint64_t bb = __ballot((d >> b) & 1);
            peers &= ((d >> b) & 1) ? bb : ~bb;
        }
        uint32_t rank = __popcll(peers & ((1ull << l) - 1));
        if (valid && rank == 0) wcnt[w][d] = __popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t off = base_d[d] + rank;
            for (int x = 0; x < w; x++) off += wcnt[x][d];
            kout[off] = k;
            vout[off] = v;
        }
        __syncthreads();
        uint32_t add = 0;
        for (int x = 0; x < TK_NT / 64; x++) add += wcnt[x][t];
        base_d[t] += add;
    }
}

__global__ void k_copy_idx(const uint32_t* in, uint32_t* out, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

static unsigned grid_for(int64_t n, int nt, unsigned cap = 8192) {
    int64_t g = (n + nt - 1) / nt;
    if (g < 1) g = 1;
    return (unsigned)(g < cap ? g : cap);
}

int64_t topk_stable_desc(const uint64_t* keys, int64_t n, int64_t keep, uint32_t* out_idx, TopkScratch& s,
                         hipStream_t st) {
    if (n <= 0 || keep <= 0) return 0;
    const int64_t m = n < keep ? n : keep;
    s.k0.ensure(m);
    s.k1.ensure(m);
    s.v0.ensure(m);
    s.v1.ensure(m);
    s.small.ensure(GH + 8 * 256);
    if (!s.h_flags) SB_HIP(hipHostMalloc((void**)&s.h_flags, 64, hipHostMallocDefault));
    uint64_t* stv = s.small.p;
    hipLaunchKernelGGL(k_sel_init, dim3(1), dim3(256), 0, st, stv, (int64_t)m);
    if (n > keep) {
        for (int pass = 0; pass < 8; pass++) {
            hipLaunchKernelGGL(k_sel_hist, dim3(grid_for(n, TK_NT * 8, 4096)), dim3(TK_NT), 0, st, keys, n, stv);
            hipLaunchKernelGGL(k_sel_pick, dim3(1), dim3(64), 0, st, stv);
        }
        int64_t ntiles = (n + TK_TILE - 1) / TK_TILE;
        s.tile_a.ensure(ntiles);
        s.tile_b.ensure(ntiles);
        hipLaunchKernelGGL(k_sel_count, dim3((unsigned)ntiles), dim3(TK_NT), 0, st, keys, n, stv, s.tile_a.p, s.tile_b.p);
        hipLaunchKernelGGL(k_sel_scan, dim3(1), dim3(1024), 0, st, s.tile_a.p, s.tile_b.p, ntiles, stv);
        hipLaunchKernelGGL(k_sel_write, dim3((unsigned)ntiles), dim3(TK_NT), 0, st, keys, n, stv, s.tile_a.p,
                           s.tile_b.p, s.k0.p, s.v0.p);
    } else {
        hipLaunchKernelGGL(k_iota, dim3(grid_for(m, 256)), dim3(256), 0, st, s.v0.p, keys, s.k0.p, m);
    }
    // constant-digit detection
    hipLaunchKernelGGL(k_sort_ghist, dim3(grid_for(m, TK_NT * 8, 2048)), dim3(TK_NT), 0, st, s.k0.p, m, stv);
    uint32_t* dflags = (uint32_t*)(stv + 3);   // reuse: word 3 (done flag) no longer needed -> 8 u32 in [3..6]
    hipLaunchKernelGGL(k_sort_flags, dim3(1), dim3(64), 0, st, stv, m, dflags);
    SB_HIP(hipMemcpyAsync(s.h_flags, dflags, 32, hipMemcpyDeviceToHost, st));
    SB_HIP(hipStreamSynchronize(st));
    int64_t ntiles = (m + TK_TILE - 1) / TK_TILE;
    s.tile_hist.ensure((size_t)ntiles * 256);
    uint64_t *ka = s.k0.p, *kb = s.k1.p;
    uint32_t *va = s.v0.p, *vb = s.v1.p;
    for (int p = 0; p < 8; p++) {
        if (s.h_flags[p]) continue;
        hipLaunchKernelGGL(k_sort_hist, dim3((unsigned)ntiles), dim3(TK_NT), 0, st, ka, m, 8 * p, s.tile_hist.p, ntiles);
        scan_exclusive_u32(s.tile_hist.p, s.tile_hist.p, ntiles * 256, nullptr, s.scan, st);
        hipLaunchKernelGGL(k_sort_scatter, dim3((unsigned)ntiles), dim3(TK_NT), 0, st, ka, va, kb, vb, m, 8 * p,
                           s.tile_hist.p, ntiles);
        uint64_t* tk = ka; ka = kb; kb = tk;
        uint32_t* tv = va; va = vb; vb = tv;
    }
    hipLaunchKernelGGL(k_copy_idx, dim3(grid_for(m, 256)), dim3(256), 0, st, va, out_idx, m);
    SB_HIP(hipGetLastError());
    return m;
}

}  // namespace sb
