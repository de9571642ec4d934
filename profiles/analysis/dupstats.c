// Same-turn duplicate structure of one saturated turn (diagnostic for the k_expand design, round 2).
// Reads a turn's parents (packed lo/hi, rank order), enumerates every raw child with the C oracle
// (oc_successors) and counts how many visited-set probes would remain if the children of a block of
// parents were deduplicated among themselves first (in LDS), for several ways of forming the blocks:
//   rank     consecutive ranks (what k_expand does now)
//   cards    parents sorted by card set, then consecutive (groups that share a card set share takes)
//   cards+g  sorted by card set, then by gem total
//   build: gcc -O2 dupstats.c -L../../oracle/build -loracle -o dupstats ; run: dupstats parents.bin n
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oc_init(const int32_t* deck_rows);
int oc_successors(uint64_t lo, uint64_t hi, uint64_t* out_lo, uint64_t* out_hi, uint64_t* out_key);

static uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
typedef struct { uint64_t* k; uint64_t cap; uint64_t n; } hs_t;
static void hs_init(hs_t* h, uint64_t cap) { h->cap = cap; h->n = 0; h->k = malloc(cap * 8); memset(h->k, 0xFF, cap * 8); }
static int hs_add(hs_t* h, uint64_t k) {   // 1 if new
    uint64_t i = mix(k) & (h->cap - 1);
    while (h->k[i] != ~0ull) { if (h->k[i] == k) return 0; i = (i + 1) & (h->cap - 1); }
    h->k[i] = k; h->n++;
    return 1;
}
static void hs_clear_keys(hs_t* h, const uint64_t* keys, int n) {   // small table reset
    (void)keys; (void)n; memset(h->k, 0xFF, h->cap * 8); h->n = 0;
}

static uint64_t *plo, *phi, **ckeys;
static int* ccnt;
static int* cnb;   // buy children per parent (first cnb[r] of ckeys[r])
static int cmp_cards(const void* a, const void* b) {
    const int i = *(const int*)a, j = *(const int*)b;
    const uint64_t ci = phi[i] & ((1ull << 26) - 1), cj = phi[j] & ((1ull << 26) - 1);
    if (plo[i] != plo[j]) return plo[i] < plo[j] ? -1 : 1;
    if (ci != cj) return ci < cj ? -1 : 1;
    return i - j;
}

// mode 0: dedup every child in the block; 1: takes only (buys always probe)
static uint64_t block_probes(const int* order, int n, int bs, int mode) {
    hs_t h;
    hs_init(&h, 1 << 15);
    uint64_t probes = 0;
    for (int b0 = 0; b0 < n; b0 += bs) {
        hs_clear_keys(&h, 0, 0);
        for (int j = b0; j < b0 + bs && j < n; j++) {
            const int r = order[j];
            for (int c = 0; c < ccnt[r]; c++) probes += (mode == 1 && c < cnb[r]) ? 1 : hs_add(&h, ckeys[r][c]);
        }
    }
    free(h.k);
    return probes;
}

int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "rb");
    const int n = atoi(argv[2]);
    int32_t deck[90 * 7];
    FILE* fd = fopen(argv[3], "rb");
    if (fread(deck, 4, 90 * 7, fd) != 90 * 7) return 1;
    fclose(fd);
    oc_init(deck);
    plo = malloc(n * 8); phi = malloc(n * 8);
    if (fread(plo, 8, n, f) != (size_t)n || fread(phi, 8, n, f) != (size_t)n) return 1;
    fclose(f);
    ckeys = malloc(n * sizeof *ckeys); ccnt = malloc(n * 4); cnb = malloc(n * 4);
    uint64_t raw = 0, nbuy = 0, olo[256], ohi[256], okey[256];
    for (int r = 0; r < n; r++) {
        ccnt[r] = oc_successors(plo[r], phi[r], olo, ohi, okey);
        cnb[r] = 0;
        while (cnb[r] < ccnt[r] && (olo[cnb[r]] != plo[r] || ((ohi[cnb[r]] ^ phi[r]) & ((1ull << 26) - 1)))) cnb[r]++;
        nbuy += cnb[r];
        ckeys[r] = malloc(ccnt[r] * 8 + 8);
        memcpy(ckeys[r], okey, ccnt[r] * 8);
        raw += ccnt[r];
    }
    hs_t g;
    hs_init(&g, 1ull << 29);
    for (int r = 0; r < n; r++) for (int c = 0; c < ccnt[r]; c++) hs_add(&g, ckeys[r][c]);
    printf("buy children %llu (%.1f%% of raw)\n", (unsigned long long)nbuy, 100.0 * nbuy / raw);
    printf("parents %d raw %llu distinct-in-turn %llu (same-turn dups %.1f%% of raw)\n", n, (unsigned long long)raw,
           (unsigned long long)g.n, 100.0 * (raw - g.n) / raw);
    int* order = malloc(n * 4);
    for (int r = 0; r < n; r++) order[r] = r;
    int bss[4] = {32, 64, 128, 256};
    for (int k = 0; k < 4; k++) {
        const uint64_t p = block_probes(order, n, bss[k], 0);
        printf("rank  blocks of %3d: probes %llu (%.1f%% of raw)\n", bss[k], (unsigned long long)p, 100.0 * p / raw);
    }
    qsort(order, n, 4, cmp_cards);
    uint64_t groups = 1;
    for (int j = 1; j < n; j++) groups += cmp_cards(&order[j - 1], &order[j]) != 0 && (plo[order[j]] != plo[order[j-1]] || ((phi[order[j]] ^ phi[order[j-1]]) & ((1ull << 26) - 1)));
    printf("distinct card sets %llu (%.1f parents each)\n", (unsigned long long)groups, (double)n / groups);
    for (int k = 0; k < 4; k++) {
        const uint64_t p = block_probes(order, n, bss[k], 0), q = block_probes(order, n, bss[k], 1);
        printf("cards blocks of %3d: probes %llu (%.1f%% of raw); takes-only dedup %llu (%.1f%%)\n", bss[k],
               (unsigned long long)p, 100.0 * p / raw, (unsigned long long)q, 100.0 * q / raw);
    }
    return 0;
}
