// sb_gf2.h — GF(2) polynomials for MT19937 jump-ahead (host only; see sb_gf2.hip).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace sb {
namespace gf2 {

constexpr size_t DEG = 19937;                 // degree of the MT19937 characteristic polynomial
constexpr size_t WORDS = (DEG + 63) / 64;     // 312 u64 words hold bits 0..DEG-1
using Poly = std::vector<uint64_t>;           // bit i = coefficient of x^i

const Poly& mt_charpoly();                    // phi(x), computed once by Berlekamp-Massey
Poly sqr_mod(const Poly& a);
Poly mulx_mod(const Poly& a);
Poly divx_mod(const Poly& a);                 // a * x^-1 mod phi (phi(0) = 1)
Poly xpow_mod(uint64_t e);
Poly jump_poly(uint64_t J);                   // g = x^(J-1) mod phi: w(n+J) = T g(T) w(n); cached
void to_words(const Poly& g, uint32_t out[624]);   // 19937 coefficient bits as 624 u32
void jump_window_host(const uint32_t win[624], const Poly& g, uint32_t out[624]);
void advance_window_host(const uint32_t win[624], uint64_t J, uint32_t out[624]);
bool self_test();

}  // namespace gf2
}  // namespace sb
