// Reuse distance of same-turn duplicate probes (visited-set lines) under two parent processing orders
// (rank order, grandparent order) and two XCD assignments; input: profiles/analysis/dump_turn_gp.py.
// build: gcc -O2 reuse.c -L../../oracle/build -loracle -Wl,-rpath,../../oracle/build -o reuse
// reuse distance of same-turn duplicate probes under different parent processing orders
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
int oc_init(const int32_t* deck_rows);
int oc_successors(uint64_t lo, uint64_t hi, uint64_t* out_lo, uint64_t* out_hi, uint64_t* out_key);
static uint64_t mix(uint64_t x) { x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x; }
static int64_t n; static uint64_t *plo, *phi; static uint32_t* par;
static uint64_t** ck; static int* cc;
typedef struct { uint64_t k; int64_t pos; int xcd; } ent;
static ent* tab; static uint64_t cap;
static int cmp_gp(const void* a, const void* b) {
    const uint32_t i = *(const uint32_t*)a, j = *(const uint32_t*)b;
    if (par[i] != par[j]) return par[i] < par[j] ? -1 : 1;
    return i < j ? -1 : (i > j);
}
// order: permutation; groups of G parents dealt to 8 XCD streams: mode 0 round robin (hardware-like), 1 contiguous eighths
static void run(const char* name, const uint32_t* order, int G, int mode) {
    memset(tab, 0xFF, cap * sizeof(ent));
    int64_t xpos[8] = {0};
    uint64_t hist[40] = {0}, dup = 0, dup_samex = 0, total = 0;
    int64_t ngroups = (n + G - 1) / G;
    // emulate: streams progress in lockstep by group: group g -> xcd
    for (int64_t g = 0; g < ngroups; g++) {
        int x = mode == 0 ? (int)(g % 8) : (int)(g * 8 / ngroups);
        for (int64_t q = g * G; q < (g + 1) * G && q < n; q++) {
            const uint32_t r = order[q];
            for (int c = 0; c < cc[r]; c++) {
                const uint64_t k = ck[r][c];
                total++;
                uint64_t i = mix(k) & (cap - 1);
                while (tab[i].k != ~0ull && tab[i].k != k) i = (i + 1) & (cap - 1);
                if (tab[i].k == k) {
                    dup++;
                    if (tab[i].xcd == x) {
                        dup_samex++;
                        int64_t d = xpos[x] - tab[i].pos;
                        int b = 0; while ((1ll << b) < d && b < 39) b++;
                        hist[b]++;
                    }
                } else { tab[i].k = k; tab[i].pos = xpos[x]; tab[i].xcd = x; }
                xpos[x]++;
            }
        }
    }
    printf("%-28s G=%d mode=%d: probes %lu dup %lu (%.1f%%) same-XCD dup %.1f%%; same-XCD dup within d probes:", name, G, mode,
           total, dup, 100.0 * dup / total, 100.0 * dup_samex / dup);
    uint64_t acc = 0;
    for (int b = 0; b < 40; b++) { acc += hist[b]; if (b == 10 || b == 12 || b == 14 || b == 15 || b == 16 || b == 18 || b == 20) printf(" <2^%d %.1f%%", b, 100.0 * acc / dup); }
    printf("\n");
}
int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "rb");
    fread(&n, 8, 1, f);
    plo = malloc(n * 8); phi = malloc(n * 8); par = malloc(n * 4);
    fread(plo, 8, n, f); fread(phi, 8, n, f); fread(par, 4, n, f); fclose(f);
    int32_t deck[90 * 8]; FILE* d = fopen("/tmp/deck.bin", "rb"); size_t nd = fread(deck, 4, 90 * 8, d); fclose(d); (void)nd;
    oc_init(deck);
    ck = malloc(n * sizeof(uint64_t*)); cc = malloc(n * sizeof(int));
    uint64_t tl[256], th[256], tk[256];
    for (int64_t r = 0; r < n; r++) {
        int m = oc_successors(plo[r], phi[r], tl, th, tk);
        cc[r] = m; ck[r] = malloc(m * 8); memcpy(ck[r], tk, m * 8);
    }
    cap = 1ull << 28; tab = malloc(cap * sizeof(ent));
    uint32_t* ord = malloc(n * 4);
    for (int64_t i = 0; i < n; i++) ord[i] = (uint32_t)i;
    run("rank order", ord, 32, 0);
    run("rank order", ord, 32, 1);
    qsort(ord, n, 4, cmp_gp);
    run("grandparent order", ord, 32, 0);
    run("grandparent order", ord, 32, 1);
    return 0;
}
