// Score-key structure of one saturated turn's next_queue (diagnostic for the top-k design, round 2).
// Children of the dumped parents, deduplicated within the turn (first occurrence), scored with the
// oracle's heuristic and a pseudo-random noise draw; prints the kept set's key span, distinct values and
// how the kept keys spread over the select bins (key >> 47) and over 16-bit prefixes.
//   build: gcc -O2 keystats.c -L../../oracle/build -loracle -o keystats ; run: keystats parents.bin n deck.bin H W
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oc_init(const int32_t* deck_rows);
int oc_successors(uint64_t lo, uint64_t hi, uint64_t* out_lo, uint64_t* out_hi, uint64_t* out_key);
double oc_score(uint64_t lo, uint64_t hi, int h, int k);

static uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
static int cmp_desc(const void* a, const void* b) {
    const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? 1 : (x > y ? -1 : 0);
}

int main(int argc, char** argv) {
    const int n = atoi(argv[2]), H = atoi(argv[4]);
    const int64_t W = atoll(argv[5]);
    int32_t deck[90 * 7];
    FILE* fd = fopen(argv[3], "rb");
    if (fread(deck, 4, 90 * 7, fd) != 90 * 7) return 1;
    oc_init(deck);
    uint64_t* plo = malloc(n * 8); uint64_t* phi = malloc(n * 8);
    FILE* f = fopen(argv[1], "rb");
    if (fread(plo, 8, n, f) != (size_t)n || fread(phi, 8, n, f) != (size_t)n) return 1;
    const uint64_t cap = 1ull << 28;
    uint64_t* set = malloc(cap * 8);
    memset(set, 0xFF, cap * 8);
    uint64_t* keys = malloc((size_t)n * 40 * 8);
    int64_t m = 0;
    uint64_t olo[256], ohi[256], okey[256], rng = 12345;
    for (int r = 0; r < n; r++) {
        const int c = oc_successors(plo[r], phi[r], olo, ohi, okey);
        for (int j = 0; j < c; j++) {
            uint64_t i = mix(okey[j]) & (cap - 1);
            int dup = 0;
            while (set[i] != ~0ull) { if (set[i] == okey[j]) { dup = 1; break; } i = (i + 1) & (cap - 1); }
            if (dup) continue;
            set[i] = okey[j];
            rng = mix(rng + 1);
            const double s = oc_score(olo[j], ohi[j], H, (int)(rng % 100) + 1);
            uint64_t b;
            memcpy(&b, &s, 8);
            keys[m++] = b;
        }
    }
    qsort(keys, m, 8, cmp_desc);
    const int64_t k = m < W ? m : W;
    const uint64_t T = keys[k - 1], mx = keys[0];
    double dT, dmx;
    memcpy(&dT, &T, 8); memcpy(&dmx, &mx, 8);
    int64_t distinct = 1, tiesT = 0, above_bin = 0;
    for (int64_t i = 1; i < k; i++) distinct += keys[i] != keys[i - 1];
    for (int64_t i = 0; i < m; i++) tiesT += keys[i] == T;
    printf("next_queue %lld kept %lld  max %.4f T %.4f  (max-T bits %d)  distinct kept values %lld  ties of T %lld\n",
           (long long)m, (long long)k, dmx, dT, 64 - __builtin_clzll(mx - T), (long long)distinct, (long long)tiesT);
    // bins of key >> 47 spanned by the kept keys, largest bin
    const uint64_t bT = T >> 47, bM = mx >> 47;
    int64_t big = 0, cur = 0;
    for (int64_t i = 0; i < k; i++) {
        if (i && (keys[i] >> 47) != (keys[i - 1] >> 47)) { big = cur > big ? cur : big; cur = 0; }
        cur++;
        above_bin += (keys[i] >> 47) > bT;
    }
    big = cur > big ? cur : big;
    printf("select bins (key>>47) spanned %llu  largest kept bin %lld  kept above T's bin %lld  all keys in T's bin %lld\n",
           (unsigned long long)(bM - bT + 1), (long long)big, (long long)above_bin,
           (long long)({ int64_t c = 0; for (int64_t i = 0; i < m; i++) c += (keys[i] >> 47) == bT; c; }));
    // the sort's prefix: (key - T) >> sh; pairs of adjacent different keys sharing a prefix = fix-up work
    for (int sh = 29; sh >= 5; sh -= 4) {
        int64_t pairs = 0, runs = 0, runel = 0;
        for (int64_t i = 1; i < k; i++) {
            const int same = ((keys[i] - T) >> sh) == ((keys[i - 1] - T) >> sh);
            if (same && keys[i] != keys[i - 1]) pairs++;
        }
        for (int64_t i = 0; i < k;) {   // runs of equal prefix holding > 1 distinct key
            int64_t j = i + 1, diff = 0;
            while (j < k && ((keys[j] - T) >> sh) == ((keys[i] - T) >> sh)) { diff |= keys[j] != keys[j - 1]; j++; }
            if (diff) { runs++; runel += j - i; }
            i = j;
        }
        printf("prefix (key-T)>>%d (%d bits): %lld flagged pairs, %lld runs to fix, %lld elements in them\n", sh,
               64 - __builtin_clzll(mx - T) - sh, (long long)pairs, (long long)runs, (long long)runel);
    }
    for (int sh = 40; sh >= 24; sh -= 8) {
        int64_t groups = 1, gbig = 0, gcur = 0;
        for (int64_t i = 1; i <= k; i++) {
            if (i == k || (keys[i] >> sh) != (keys[i - 1] >> sh)) { gbig = ++gcur > gbig ? gcur : gbig; gcur = 0; groups += i < k; }
            else gcur++;
        }
        printf("prefix key>>%d: %lld groups among the kept, largest %lld\n", sh, (long long)groups, (long long)gbig);
    }
    return 0;
}
