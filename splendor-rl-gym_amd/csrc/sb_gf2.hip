// sb_gf2.hip — host-side GF(2) polynomial arithmetic for MT19937 jump-ahead (no device code).
//
// The randint noise (src/solver.py:215 etc.) is CPython's MT19937 stream.  To generate it with one
// producer per CU, each producer needs the generator state p*L words ahead of the origin.  Let
// y_n be the untempered MT words and w(n) = (y_n .. y_{n+623}) the 624-word window; the twist is a
// linear map T with w(n+1) = T w(n) over GF(2).  Its minimal polynomial is x * phi(x), where phi is
// the degree-19937 characteristic polynomial of MT19937 (the extra factor x is the 31 low bits of
// y_n that no later word depends on).  Hence for J >= 1
//     w(n+J) = T g(T) w(n),  g = x^(J-1) mod phi,   i.e.   w(n+J)[j] = XOR_{i: g_i=1} y_{n+1+i+j}.
// phi is recovered with Berlekamp-Massey from 2*19937+ output bits; x^e mod phi by squaring.
#include <stdint.h>
#include <string.h>

#include <map>
#include <mutex>
#include <stdexcept>
#include <vector>

#include "sb_gf2.h"

namespace sb {
namespace gf2 {

static inline uint32_t mt_mix_h(uint32_t a, uint32_t b, uint32_t m) {
    uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return m ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// untempered sequence y_0..y_{n-1} from a window (y_0..y_623)
static void mt_sequence(const uint32_t win[624], std::vector<uint32_t>& y, size_t n) {
    y.assign(n < 624 ? 624 : n, 0);
    memcpy(y.data(), win, 624 * 4);
    for (size_t k = 0; k + 624 < n; k++) y[k + 624] = mt_mix_h(y[k], y[k + 1], y[k + 397]);
}

static inline int getbit(const Poly& p, size_t i) { return (int)((p[i >> 6] >> (i & 63)) & 1); }
static inline void flipbit(Poly& p, size_t i) { p[i >> 6] ^= 1ull << (i & 63); }

// 64 bits of v starting at bit offset `off` (bits past the end read as 0)
static inline uint64_t bits64(const Poly& v, size_t off) {
    size_t q = off >> 6, s = off & 63;
    uint64_t lo = q < v.size() ? v[q] : 0;
    if (s == 0) return lo;
    uint64_t hi = q + 1 < v.size() ? v[q + 1] : 0;
    return (lo >> s) | (hi << (64 - s));
}

// dst ^= src << sh  (bits)
static void xor_shifted(Poly& dst, const Poly& src, size_t src_bits, size_t sh) {
    size_t wq = sh >> 6, ws = sh & 63;
    size_t nw = (src_bits + 63) >> 6;
    for (size_t i = 0; i < nw; i++) {
        uint64_t w = src[i];
        if (!w) continue;
        size_t d = i + wq;
        if (d < dst.size()) dst[d] ^= w << ws;
        if (ws && d + 1 < dst.size()) dst[d + 1] ^= w >> (64 - ws);
    }
}

static Poly compute_charpoly() {
    // bit 31 of y_n from Python's seed-0 state (any non-degenerate window works)
    uint32_t win[624];
    uint32_t x = 5489u;   // MT19937 init_genrand
    win[0] = x;
    for (int i = 1; i < 624; i++) win[i] = x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)i;
    const size_t N = 2 * DEG + 128;
    std::vector<uint32_t> y;
    mt_sequence(win, y, N);
    // reversed bit sequence r[k] = s[N-1-k]
    Poly r((N + 63) / 64 + 2, 0);
    for (size_t k = 0; k < N; k++)
        if ((y[N - 1 - k] >> 31) & 1u) flipbit(r, k);
    Poly C((N + 63) / 64 + 2, 0), B((N + 63) / 64 + 2, 0), T;
    C[0] = 1;
    B[0] = 1;
    size_t L = 0, m = 1;
    for (size_t n = 0; n < N; n++) {
        // d = sum_{i=0..L} C_i s_{n-i} = sum C_i r[N-1-n+i]
        const size_t off = N - 1 - n;
        uint64_t acc = 0;
        const size_t nw = L / 64 + 1;
        for (size_t wi = 0; wi < nw; wi++) {
            uint64_t c = C[wi];
            if (wi == nw - 1) {
                size_t rem = (L % 64) + 1;
                if (rem < 64) c &= (1ull << rem) - 1;
            }
            acc ^= c & bits64(r, off + 64 * wi);
        }
        if (!(__builtin_popcountll(acc) & 1)) {
            m++;
            continue;
        }
        if (2 * L <= n) {
            T = C;
            xor_shifted(C, B, N + 1, m);
            L = n + 1 - L;
            B = T;
            m = 1;
        } else {
            xor_shifted(C, B, N + 1, m);
            m++;
        }
    }
    if (L != DEG) throw std::runtime_error("MT19937 characteristic polynomial: unexpected degree");
    Poly phi(WORDS + 1, 0);   // phi_i = C_{L-i}
    for (size_t i = 0; i <= L; i++)
        if (getbit(C, L - i)) flipbit(phi, i);
    if (!getbit(phi, 0) || !getbit(phi, DEG)) throw std::runtime_error("MT19937 characteristic polynomial: bad ends");
    return phi;
}

const Poly& mt_charpoly() {
    static Poly phi;
    static std::once_flag once;
    std::call_once(once, [] { phi = compute_charpoly(); });
    return phi;
}

// reduce r (degree < 2*DEG) mod phi in place; result has WORDS+1 words
static void reduce(Poly& r) {
    const Poly& phi = mt_charpoly();
    for (size_t i = r.size() * 64; i-- > DEG;) {
        if (i >> 6 >= r.size()) continue;
        if (getbit(r, i)) xor_shifted(r, phi, DEG + 1, i - DEG);
    }
    r.resize(WORDS + 1);
}

Poly sqr_mod(const Poly& a) {
    static uint16_t spread[256];
    static std::once_flag once;
    std::call_once(once, [] {
        for (int v = 0; v < 256; v++) {
            uint16_t s = 0;
            for (int b = 0; b < 8; b++)
                if (v >> b & 1) s |= (uint16_t)(1u << (2 * b));
            spread[v] = s;
        }
    });
    Poly r(2 * (WORDS + 1) + 1, 0);
    for (size_t i = 0; i < a.size() && i <= WORDS; i++) {
        uint64_t w = a[i];
        uint64_t lo = 0, hi = 0;
        for (int b = 0; b < 4; b++) {
            lo |= (uint64_t)spread[(w >> (8 * b)) & 255] << (16 * b);
            hi |= (uint64_t)spread[(w >> (32 + 8 * b)) & 255] << (16 * b);
        }
        r[2 * i] ^= lo;
        r[2 * i + 1] ^= hi;
    }
    reduce(r);
    return r;
}

Poly mulx_mod(const Poly& a) {
    Poly r(WORDS + 2, 0);
    for (size_t i = 0; i <= WORDS && i < a.size(); i++) {
        r[i] |= a[i] << 1;
        r[i + 1] |= a[i] >> 63;
    }
    if (getbit(r, DEG)) xor_shifted(r, mt_charpoly(), DEG + 1, 0);
    r.resize(WORDS + 1);
    return r;
}

Poly divx_mod(const Poly& a) {
    Poly r = a;
    r.resize(WORDS + 1);
    if (getbit(r, 0)) {
        const Poly& phi = mt_charpoly();
        for (size_t i = 0; i <= WORDS; i++) r[i] ^= phi[i];
    }
    for (size_t i = 0; i <= WORDS; i++) r[i] = (r[i] >> 1) | (i + 1 <= WORDS ? r[i + 1] << 63 : 0);
    return r;
}

Poly xpow_mod(uint64_t e) {
    Poly r(WORDS + 1, 0);
    r[0] = 1;
    int top = 63;
    while (top >= 0 && !((e >> top) & 1)) top--;
    for (int b = top; b >= 0; b--) {
        r = sqr_mod(r);
        if ((e >> b) & 1) r = mulx_mod(r);
    }
    return r;
}

void to_words(const Poly& g, uint32_t out[624]) {
    memset(out, 0, 624 * 4);
    for (size_t i = 0; i < DEG; i++)
        if (getbit(g, i)) out[i >> 5] |= 1u << (i & 31);
}

Poly jump_poly(uint64_t J) {
    static std::map<uint64_t, Poly> cache;
    static std::mutex mu;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find(J);
        if (it != cache.end()) return it->second;
    }
    Poly g = divx_mod(xpow_mod(J));   // x^(J-1) mod phi
    std::lock_guard<std::mutex> lk(mu);
    cache[J] = g;
    return g;
}

void jump_window_host(const uint32_t win[624], const Poly& g, uint32_t out[624]) {
    std::vector<uint32_t> y;
    mt_sequence(win, y, 1 + DEG + 624);
    for (int j = 0; j < 624; j++) out[j] = 0;
    for (size_t i = 0; i < DEG; i++)
        if (getbit(g, i))
            for (int j = 0; j < 624; j++) out[j] ^= y[1 + i + j];
}

void advance_window_host(const uint32_t win[624], uint64_t J, uint32_t out[624]) {
    std::vector<uint32_t> y;
    mt_sequence(win, y, (size_t)J + 624);
    memcpy(out, y.data() + J, 624 * 4);
}

bool self_test() {
    uint32_t w[624], a[624], b[624];
    uint32_t x = 12345u;
    for (int i = 0; i < 624; i++) w[i] = x = x * 1664525u + 1013904223u;
    for (uint64_t J : {1ull, 2ull, 397ull, 624ull, 20000ull, 123457ull}) {
        jump_window_host(w, jump_poly(J), a);
        advance_window_host(w, J, b);
        // the low 31 bits of the first word never influence later words; compare all 624 words
        if (memcmp(a, b, sizeof a) != 0) return false;
    }
    return true;
}

}  // namespace gf2
}  // namespace sb
