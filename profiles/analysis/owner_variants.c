// Coarser trail ownership than the whole card set (the k lowest cards) on C3's turn 11 at W=4M: how many buys keep
// their parent's owner and how balanced the owners are.  Input: profiles/analysis/dump_turn_gp.py.
// build: gcc -O2 owner_variants.c -L../../oracle/build -loracle -Wl,-rpath,../../oracle/build -o owner_variants
// card-set ownership variants: fraction of buy children that keep their parent's owner, and load balance
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
int oc_init(const int32_t* deck_rows);
int oc_successors(uint64_t lo, uint64_t hi, uint64_t* out_lo, uint64_t* out_hi, uint64_t* out_key);
static uint64_t mix(uint64_t x) { x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x; }
// feature: the k lowest cards of the 90-bit set (k = 0: the whole set)
static uint64_t feat(uint64_t lo, uint64_t hi, int k) {
    uint32_t chi = (uint32_t)(hi & ((1u << 26) - 1));
    if (k == 0) return mix(lo ^ mix(chi + 0x9e3779b97f4a7c15ull));
    uint64_t a = 0, b = 0; int got = 0;
    uint64_t l = lo; uint32_t h = chi;
    while (got < k && l) { uint64_t bit = l & (~l + 1); a |= bit; l &= l - 1; got++; }
    while (got < k && h) { uint32_t bit = h & (~h + 1); b |= bit; h &= h - 1; got++; }
    return mix(a ^ mix(b + 0x9e3779b97f4a7c15ull + (uint64_t)k));
}
int main(int argc, char** argv) {
    int64_t n; FILE* f = fopen(argv[1], "rb"); if (fread(&n, 8, 1, f) != 1) return 1;
    uint64_t *plo = malloc(n * 8), *phi = malloc(n * 8);
    if (fread(plo, 8, n, f) != (size_t)n || fread(phi, 8, n, f) != (size_t)n) return 1; fclose(f);
    int32_t deck[90 * 8]; FILE* d = fopen("/tmp/deck.bin", "rb"); if (fread(deck, 4, 90 * 8, d) == 0) return 1; fclose(d);
    oc_init(deck);
    const int W = argc > 2 ? atoi(argv[2]) : 8;
    uint64_t tl[256], th[256], tk[256];
    for (int k = 0; k <= 5; k++) {
        uint64_t raw = 0, buys = 0, buys_local = 0, takes = 0;
        uint64_t par[64] = {0}, rawo[64] = {0}, recv[64] = {0};
        for (int64_t r = 0; r < n; r++) {
            const uint64_t fo = feat(plo[r], phi[r], k);
            const int o = (int)((fo >> 40) % W);
            par[o]++;
            int m = oc_successors(plo[r], phi[r], tl, th, tk);
            raw += m; rawo[o] += m;
            for (int c = 0; c < m; c++) {
                const uint32_t pc = (uint32_t)(phi[r] & ((1u << 26) - 1)), cc = (uint32_t)(th[c] & ((1u << 26) - 1));
                if (tl[c] == plo[r] && cc == pc) { takes++; continue; }
                buys++;
                const int oc = (int)((feat(tl[c], th[c], k) >> 40) % W);
                if (oc == o) buys_local++; else recv[oc]++;
            }
        }
        uint64_t pmax = 0, rmax = 0, vmax = 0, vsum = 0;
        for (int o = 0; o < W; o++) { if (par[o] > pmax) pmax = par[o]; if (rawo[o] > rmax) rmax = rawo[o]; if (recv[o] > vmax) vmax = recv[o]; vsum += recv[o]; }
        printf("k=%d%s: takes %.1f%% of raw, buys %.1f%%, buys local %.1f%% -> records %.1f%% of raw; parents max/mean %.3f, raw max/mean %.3f, recv max/mean %.3f\n",
               k, k == 0 ? " (whole card set)" : " lowest cards", 100.0 * takes / raw, 100.0 * buys / raw, 100.0 * buys_local / buys,
               100.0 * (buys - buys_local) / raw, (double)pmax * W / n, (double)rmax * W / raw, vsum ? (double)vmax * W / vsum : 0.0);
    }
    return 0;
}
