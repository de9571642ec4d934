// sb_device.h — device-side primitives of the MI355X Splendor beam engine (gfx950 only).
//
// Everything here restates one piece of IamJasonBian/Splendor-RL-Gym's speedrun step exactly:
//   * packed state codec                 State (src/solver.py:308-318)
//   * CPython 64-bit tuple hash          hash((cards, gems)) (src/solver.py:318, 332-336)
//   * buy test + buy arithmetic          get_buys key (src/solver.py:360-373, src/buys.py:13-17),
//                                        buy_card / subtract_with_bonus / increase_bonus
//                                        (src/solver.py:338-355, src/gems.py:116-143)
//   * take patterns                      get_takes / take_gems (src/gems.py:14-113)
//   * heuristic scorers                  src/solver.py:210-305, float64, no FMA contraction
// Compiled with -ffp-contract=off so a*b+c stays two IEEE roundings like CPython.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sb {

constexpr int NCARDS = 90;
constexpr int NCOL = 5;
constexpr int MAXG = 7;
constexpr int MAX_CHILDREN = 192;    // >= 90 buys + 100 takes; stride of per-parent raw slots
constexpr int NPAT_MAX = 100;        // patterns in the largest bucket (total == 10)
constexpr int N_POW = 11;
constexpr int POW_BASES = 256;

constexpr uint64_t XXP1 = 11400714785074694791ull;
constexpr uint64_t XXP2 = 14029467366897019727ull;
constexpr uint64_t XXP5 = 2870177450012600261ull;
constexpr uint64_t EMPTY = ~0ull;    // never a tuple hash: CPython maps -1 to 1546275796

// pow-table rows, in the exponent order of sb_init_tables
enum PowRow { P03 = 0, P04, P05, P06, P07, P08, P12, P20, P25, P28, P32 };

// Card word: bits 0..14 cost (3 bits per colour), 15..17 pt, 18..20 colour.
// Pattern word: bits 0..14 (delta + 2) per colour, 15..17 index of the 2 in a take-2 pattern (7 = take-3).
// Enumeration tables (derived on the host from the same deck and patterns):
//   aff_lo/aff_hi[i][v]  cards whose colour-i cost is <= v (90-bit masks): the buy set of a state is
//                        AND_i aff[i][min(g_i + b_i, 7)] minus its own cards, in deck order
//   pdelta[b][p]         pattern p of bucket b as a packed signed gem delta: child gems = gf + pdelta
//   tmask[gf]            valid take patterns (bucket order) of gem field gf, 100-bit mask
struct Tables {
    uint32_t card[NCARDS];
    uint32_t pat[4][NPAT_MAX];
    int32_t npat[4];
    uint64_t colmask_lo[NCOL];
    uint32_t colmask_hi[NCOL];
    double pw[N_POW][POW_BASES];
    double noise[100];
    uint64_t aff_lo[NCOL][8];
    uint32_t aff_hi[NCOL][8];
    int32_t pdelta[4][NPAT_MAX];
    uint64_t tmask[1 << 15][2];
};

// ---------------------------------------------------------------- state codec
__host__ __device__ __forceinline__ int st_gem(uint64_t hi, int i) { return (int)((hi >> (26 + 3 * i)) & 7); }
__host__ __device__ __forceinline__ int st_pts(uint64_t hi) { return (int)((hi >> 41) & 0xFF); }
__host__ __device__ __forceinline__ int st_saved(uint64_t hi) { return (int)(hi >> 49); }
__host__ __device__ __forceinline__ uint32_t st_chi(uint64_t hi) { return (uint32_t)(hi & ((1u << 26) - 1)); }
__host__ __device__ __forceinline__ uint32_t st_gemfield(uint64_t hi) { return (uint32_t)((hi >> 26) & 0x7FFF); }
__host__ __device__ __forceinline__ uint64_t st_with_gems(uint64_t hi, uint32_t gemfield) {
    return (hi & ~(0x7FFFull << 26)) | ((uint64_t)gemfield << 26);
}
__host__ __device__ __forceinline__ bool st_owns(uint64_t lo, uint64_t hi, int c) {
    return c < 64 ? ((lo >> c) & 1) : ((hi >> (c - 64)) & 1);
}

// ---------------------------------------------------------------- CPython tuple hash
__host__ __device__ __forceinline__ uint64_t th_step(uint64_t acc, uint64_t lane) {
    acc += lane * XXP2;
    acc = (acc << 31) | (acc >> 33);
    return acc * XXP1;
}
__host__ __device__ __forceinline__ uint64_t th_fin(uint64_t acc, uint64_t len) {
    acc += len ^ (XXP5 ^ 3527539ull);
    return acc == ~0ull ? 1546275796ull : acc;
}
// hash(tuple(sorted cards)) over the 90-bit mask (lo, chi)
__host__ __device__ __forceinline__ uint64_t hash_cards(uint64_t lo, uint32_t chi) {
    uint64_t acc = XXP5;
    uint64_t n = 0;
    while (lo) {
        int c = __builtin_ctzll(lo);
        lo &= lo - 1;
        acc = th_step(acc, (uint64_t)c);
        n++;
    }
    while (chi) {
        int c = __builtin_ctz(chi);
        chi &= chi - 1;
        acc = th_step(acc, (uint64_t)(64 + c));
        n++;
    }
    return th_fin(acc, n);
}
// hash(gems) for the 15-bit gem field
__host__ __device__ __forceinline__ uint64_t hash_gems(uint32_t gf) {
    uint64_t acc = XXP5;
#pragma unroll
    for (int i = 0; i < NCOL; i++) acc = th_step(acc, (uint64_t)((gf >> (3 * i)) & 7));
    return th_fin(acc, NCOL);
}
__host__ __device__ __forceinline__ uint64_t state_key(uint64_t hcards, uint64_t hgems) {
    uint64_t acc = th_step(XXP5, hcards);
    acc = th_step(acc, hgems);
    return th_fin(acc, 2);
}
__host__ __device__ __forceinline__ uint64_t key_of(uint64_t lo, uint64_t hi) {
    return state_key(hash_cards(lo, st_chi(hi)), hash_gems(st_gemfield(hi)));
}

// slot hash for the open-addressing visited set (the key is already mixed; fmix64 spreads low bits)
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

// ---------------------------------------------------------------- per-state derived values
struct Derived {
    int g[NCOL];
    int b[NCOL];
    int pts, saved;
};

__device__ __forceinline__ void derive(const Tables& T, uint64_t lo, uint64_t hi, Derived& d) {
    uint32_t chi = st_chi(hi);
#pragma unroll
    for (int i = 0; i < NCOL; i++) {
        d.g[i] = st_gem(hi, i);
        d.b[i] = __popcll(lo & T.colmask_lo[i]) + __popc(chi & T.colmask_hi[i]);
    }
    d.pts = st_pts(hi);
    d.saved = st_saved(hi);
}

__device__ __forceinline__ int card_cost(uint32_t cw, int i) { return (int)((cw >> (3 * i)) & 7); }
__device__ __forceinline__ int card_pt(uint32_t cw) { return (int)((cw >> 15) & 7); }
__device__ __forceinline__ int card_color(uint32_t cw) { return (int)((cw >> 18) & 7); }

// card c affordable with min(g+b, 7) (src/solver.py:360-369): cost <= 7, so cost <= g+b suffices
__device__ __forceinline__ bool affordable(uint32_t cw, const Derived& d) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < NCOL; i++) ok &= card_cost(cw, i) <= d.g[i] + d.b[i];
    return ok;
}

// buy_card (src/solver.py:338-355 + src/gems.py:116-129); returns the child's hi word
__device__ __forceinline__ uint64_t buy_child_hi(uint32_t cw, int c, const Derived& d, uint64_t hi, uint64_t* lo) {
    uint32_t gf = 0;
    int sv = 0;
#pragma unroll
    for (int i = 0; i < NCOL; i++) {
        int cost = card_cost(cw, i);
        int cc = cost - d.b[i];
        cc = cc < 0 ? 0 : cc;
        sv += cost - cc;
        int x = d.g[i] - cc;
        x = x < 0 ? 0 : x;
        gf |= (uint32_t)x << (3 * i);
    }
    uint64_t nh = st_with_gems(hi, gf);
    if (c < 64) *lo |= 1ull << c; else nh |= 1ull << (c - 64);
    nh += (uint64_t)card_pt(cw) << 41;       // pts field never overflows (max 140)
    nh += (uint64_t)sv << 49;                // saved field 15 bits
    return nh;
}

// take pattern p applied to gems; valid per src/gems.py:54-66.  Returns false if invalid.
__device__ __forceinline__ bool take_child(uint32_t pw, const Derived& d, uint32_t* gf_out) {
    int two = (int)((pw >> 15) & 7);
    bool ok = true;
    uint32_t gf = 0;
#pragma unroll
    for (int i = 0; i < NCOL; i++) {
        int x = d.g[i] + (int)((pw >> (3 * i)) & 7) - 2;
        ok &= (x >= 0) & (x <= MAXG);
        gf |= (uint32_t)(x & 7) << (3 * i);
        if (two == i) ok &= d.g[i] <= MAXG - 4;
    }
    *gf_out = gf;
    return ok;
}

__device__ __forceinline__ int take_bucket(const Derived& d) {
    int tot = d.g[0] + d.g[1] + d.g[2] + d.g[3] + d.g[4];
    return tot > 10 ? -1 : (tot <= 7 ? 0 : tot - 7);
}

// ---------------------------------------------------------------- scores (src/solver.py:210-286)
// pw is the host-captured float(x) ** e table; evaluation order is Python's, left to right.
// G = total gems, B = total bonus (== len(cards) in speedrun), U = colours with a bonus.
template <int H>
__device__ __forceinline__ double score_vals(const double (*pw)[POW_BASES], int pts, int saved, int G, int B, int U,
                                             double noise) {
    // keeps the table read in bounds only: a state with saved >= 256 sets error bit 2 in the emission
    // (sb_wave.inc) and sb_step fails with "saved >= 256 exceeds the pow tables" (tests: saved_overflow)
    saved = saved < POW_BASES ? saved : POW_BASES - 1;
    if constexpr (H == 0) {   // simple
        return pw[P04][saved] * pw[P25][pts] + noise;
    } else if constexpr (H == 1) {   // balanced
        double r = pw[P28][pts] * 100;
        r = r + pw[P05][saved] * 10;
        r = r + pw[P03][G + B * 2] * 5;
        r = r + pw[P06][B] * 3;       // len(cards) == sum(bonus) in speedrun
        r = r + pw[P04][U] * 2;
        return r + noise;
    } else if constexpr (H == 2) {   // aggressive
        double r = pw[P32][pts] * 200;
        r = r + pw[P03][saved] * 5;
        r = r + pw[P05][B] * 2;
        return r + noise;
    } else {                         // efficiency
        double r = pw[P20][pts] * 50;
        r = r + pw[P07][saved] * 30;
        r = r + pw[P12][B] * 20;
        r = r + pw[P08][U] * 10;
        return r + noise;
    }
}

template <int H>
__device__ __forceinline__ double score_of(const double (*pw)[POW_BASES], const Tables& T, uint64_t lo, uint64_t hi,
                                           double noise) {
    uint32_t chi = st_chi(hi);
    int G = 0, B = 0, U = 0;
#pragma unroll
    for (int i = 0; i < NCOL; i++) {
        int b = __popcll(lo & T.colmask_lo[i]) + __popc(chi & T.colmask_hi[i]);
        G += st_gem(hi, i);
        B += b;
        U += b > 0;
    }
    return score_vals<H>(pw, st_pts(hi), st_saved(hi), G, B, U, noise);
}

// ---------------------------------------------------------------- mask enumeration
// buy set of a state in deck order: (lo 64 cards, hi 26 cards)
__device__ __forceinline__ void buy_set(const uint64_t (*aff_lo)[8], const uint32_t (*aff_hi)[8], const Derived& d,
                                        uint64_t lo, uint64_t hi, uint64_t* blo, uint32_t* bhi) {
    uint64_t ml = ~lo;
    uint32_t mh = ~st_chi(hi) & ((1u << 26) - 1);
#pragma unroll
    for (int i = 0; i < NCOL; i++) {
        int v = d.g[i] + d.b[i];
        v = v < MAXG ? v : MAXG;
        ml &= aff_lo[i][v];
        mh &= aff_hi[i][v];
    }
    *blo = ml;
    *bhi = mh;
}
// 192-bit move space of a parent: bit dsc set for every legal move (buys 0..89, takes NCARDS + bit)
__device__ __forceinline__ void move_space(uint64_t bl, uint32_t bh, uint64_t t0, uint64_t t1, uint64_t* w) {
    w[0] = bl;
    w[1] = (uint64_t)bh | (t0 << (NCARDS - 64));
    w[2] = (t0 >> (128 - NCARDS)) | (t1 << (NCARDS - 64));
}
// per-colour bonus counts packed 5 bits each
__device__ __forceinline__ uint32_t pack_bonus(const Derived& d) {
    uint32_t p = 0;
#pragma unroll
    for (int i = 0; i < NCOL; i++) p |= (uint32_t)d.b[i] << (5 * i);
    return p;
}
__device__ __forceinline__ void derive_packed(uint64_t hi, uint32_t pbon, Derived& d) {
#pragma unroll
    for (int i = 0; i < NCOL; i++) {
        d.g[i] = st_gem(hi, i);
        d.b[i] = (int)((pbon >> (5 * i)) & 31);
    }
    d.pts = st_pts(hi);
    d.saved = st_saved(hi);
}

}  // namespace sb
