/*
 * oracle.c — CPU restatement of the reference's speedrun beam step (TEST INFRASTRUCTURE ONLY).
 *
 * This file is the parity checker and the CPU baseline ("kind": "port") for the MI355X beam
 * engine.  It is never linked into, loaded by, or called from the product path
 * (splendor-rl-gym_amd/); only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may use it.  It restates, single-threaded and in plain C, the algorithm of
 * IamJasonBian/Splendor-RL-Gym (snapshot 2025-11-28):
 *
 *   - state identity  hash((cards, gems))                     src/solver.py:318,332-336
 *   - successor order (buys in deck order, then takes)         src/solver.py:357-388
 *   - affordability   get_buys()[min(g+b,7)]                   src/buys.py:13-17,39-41
 *   - buy arithmetic  buy_card/subtract_with_bonus/increase    src/solver.py:338-355, src/gems.py:116-143
 *   - take patterns   distinct_permutations tables             src/gems.py:17-37,54-113
 *   - heuristics      simple/balanced/aggressive/efficiency    src/solver.py:210-305
 *   - turn loop       goal check, trail dedup, stable prune    src/solver.py:425-464
 *   - noise           random.randint(1,100) = MT19937 + rejection of (w>>25) >= 100
 *
 * Exactness notes: CPython's 64-bit tuple hash; Python float ** float is
 * libm pow() (glibc), evaluated left to right without contraction (compile with
 * -ffp-contract=off); sorted(..., reverse=True) is stable, so ties keep next_queue order.
 *
 * State encoding shared with the engine (2 x u64, see include/splendor_beam.h):
 *   lo = cards 0..63 bitmask
 *   hi = cards 64..89 (bits 0..25) | gems g_i at bits 26+3i (3 bits each) | pts bits 41..48
 *        | saved bits 49..63
 */
#include <fcntl.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#define NCARDS 90
#define NCOL 5
#define MAXG 7

/* ------------------------------------------------------------------ deck / tables */
typedef struct { int cost[NCOL]; int pt; int color; } card_t;
static card_t DECK[NCARDS];
static int DECK_READY = 0;

/* take patterns per bucket: 0 (sum<=7), 1 (==8), 2 (==9), 3 (==10) */
typedef struct { int d[NCOL]; int two_at; /* -1 for take-3 family */ } pat_t;
static pat_t PATS[4][128];
static int NPATS[4];

static int next_perm(int* a, int n) {   /* lexicographic next permutation of a multiset */
    int i = n - 2;
    while (i >= 0 && a[i] >= a[i + 1]) i--;
    if (i < 0) return 0;
    int j = n - 1;
    while (a[j] <= a[i]) j--;
    int t = a[i]; a[i] = a[j]; a[j] = t;
    for (int l = i + 1, r = n - 1; l < r; l++, r--) { t = a[l]; a[l] = a[r]; a[r] = t; }
    return 1;
}

static int cmp_int(const void* x, const void* y) { return *(const int*)x - *(const int*)y; }

/* append distinct_permutations(p) (src/gems.py:17-19: sorted input, lexicographic order) */
static void add_perms(int bucket, const int p[NCOL], int is_two) {
    int a[NCOL];
    memcpy(a, p, sizeof a);
    qsort(a, NCOL, sizeof(int), cmp_int);
    do {
        pat_t* q = &PATS[bucket][NPATS[bucket]++];
        memcpy(q->d, a, sizeof a);
        q->two_at = -1;
        if (is_two) for (int i = 0; i < NCOL; i++) if (a[i] == 2) { q->two_at = i; break; }
    } while (next_perm(a, NCOL));
}

static void build_patterns(void) {
    /* src/gems.py:22-37 and take_gems order (:85-108): take-3 family first, then take-2 */
    static const int t7[NCOL] = {1, 1, 1, 0, 0};
    static const int t8a[NCOL] = {1, 1, 1, -1, 0}, t8b[NCOL] = {1, 1, 0, 0, 0};
    static const int t9a[NCOL] = {1, 1, 1, -1, -1}, t9b[NCOL] = {1, 1, -1, 0, 0}, t9c[NCOL] = {1, 0, 0, 0, 0};
    static const int t10a[NCOL] = {1, 1, -1, -1, 0}, t10b[NCOL] = {1, -1, 0, 0, 0};
    static const int w8[NCOL] = {2, 0, 0, 0, 0}, w9[NCOL] = {2, -1, 0, 0, 0};
    static const int w10a[NCOL] = {2, -1, -1, 0, 0}, w10b[NCOL] = {2, -2, 0, 0, 0};
    memset(NPATS, 0, sizeof NPATS);
    add_perms(0, t7, 0);  add_perms(0, w8, 1);
    add_perms(1, t8a, 0); add_perms(1, t8b, 0); add_perms(1, w8, 1);
    add_perms(2, t9a, 0); add_perms(2, t9b, 0); add_perms(2, t9c, 0); add_perms(2, w9, 1);
    add_perms(3, t10a, 0); add_perms(3, t10b, 0); add_perms(3, w10a, 1); add_perms(3, w10b, 1);
}

/* deck rows: cost[5], pt, color  (7 ints per card, deck order = cards.csv order) */
int oc_init(const int32_t* deck_rows) {
    for (int c = 0; c < NCARDS; c++) {
        for (int i = 0; i < NCOL; i++) DECK[c].cost[i] = deck_rows[c * 7 + i];
        DECK[c].pt = deck_rows[c * 7 + 5];
        DECK[c].color = deck_rows[c * 7 + 6];
    }
    build_patterns();
    DECK_READY = 1;
    return 0;
}

/* export the pattern table (for tests / engine table cross-checks) */
int oc_patterns(int bucket, int32_t* out, int cap) {
    if (bucket < 0 || bucket > 3) return -1;
    int n = NPATS[bucket] < cap ? NPATS[bucket] : cap;
    for (int k = 0; k < n; k++) {
        for (int i = 0; i < NCOL; i++) out[k * 6 + i] = PATS[bucket][k].d[i];
        out[k * 6 + 5] = PATS[bucket][k].two_at;
    }
    return NPATS[bucket];
}

/* ------------------------------------------------------------------ state codec */
typedef struct { uint64_t lo, hi; } st_t;

static inline int st_gem(st_t s, int i) { return (int)((s.hi >> (26 + 3 * i)) & 7); }
static inline int st_pts(st_t s) { return (int)((s.hi >> 41) & 0xFF); }
static inline int st_saved(st_t s) { return (int)(s.hi >> 49); }
static inline int st_has(st_t s, int c) { return c < 64 ? (int)((s.lo >> c) & 1) : (int)((s.hi >> (c - 64)) & 1); }

static inline st_t st_make(uint64_t lo, uint64_t cards_hi, const int g[NCOL], int pts, int saved) {
    st_t s;
    s.lo = lo;
    s.hi = cards_hi & ((1ull << 26) - 1);
    for (int i = 0; i < NCOL; i++) s.hi |= (uint64_t)g[i] << (26 + 3 * i);
    s.hi |= (uint64_t)pts << 41;
    s.hi |= (uint64_t)saved << 49;
    return s;
}

static void st_bonus(st_t s, int b[NCOL]) {
    for (int i = 0; i < NCOL; i++) b[i] = 0;
    for (uint64_t m = s.lo; m; m &= m - 1) b[DECK[__builtin_ctzll(m)].color]++;
    for (uint64_t m = s.hi & ((1ull << 26) - 1); m; m &= m - 1) b[DECK[64 + __builtin_ctzll(m)].color]++;
}

/* ------------------------------------------------------------------ CPython tuple hash */
#define XXP1 11400714785074694791ull
#define XXP2 14029467366897019727ull
#define XXP5 2870177450012600261ull
static inline uint64_t rotl31(uint64_t x) { return (x << 31) | (x >> 33); }
static inline uint64_t th_step(uint64_t acc, uint64_t lane) { acc += lane * XXP2; acc = rotl31(acc); return acc * XXP1; }
static inline uint64_t th_fin(uint64_t acc, uint64_t len) {
    acc += len ^ (XXP5 ^ 3527539ull);
    return acc == ~0ull ? 1546275796ull : acc;
}

static uint64_t hash_cards(st_t s) {   /* sorted card tuple: ascending bit order */
    uint64_t acc = XXP5; int n = 0;
    for (uint64_t m = s.lo; m; m &= m - 1, n++) acc = th_step(acc, (uint64_t)__builtin_ctzll(m));
    for (uint64_t m = s.hi & ((1ull << 26) - 1); m; m &= m - 1, n++) acc = th_step(acc, (uint64_t)(64 + __builtin_ctzll(m)));
    return th_fin(acc, (uint64_t)n);
}
static uint64_t hash_gems(const int g[NCOL]) {
    uint64_t acc = XXP5;
    for (int i = 0; i < NCOL; i++) acc = th_step(acc, (uint64_t)g[i]);
    return th_fin(acc, NCOL);
}
static uint64_t key_of(uint64_t hcards, uint64_t hgems) {
    uint64_t acc = XXP5;
    acc = th_step(acc, hcards);
    acc = th_step(acc, hgems);
    return th_fin(acc, 2);
}
uint64_t oc_state_key(uint64_t lo, uint64_t hi) {
    st_t s = {lo, hi};
    int g[NCOL];
    for (int i = 0; i < NCOL; i++) g[i] = st_gem(s, i);
    return key_of(hash_cards(s), hash_gems(g));
}

/* ------------------------------------------------------------------ successors */
/* Writes children of s in the reference's order (src/solver.py:357-388). Returns count. */
static int successors(st_t s, st_t* out) {
    int g[NCOL], b[NCOL], n = 0;
    for (int i = 0; i < NCOL; i++) g[i] = st_gem(s, i);
    st_bonus(s, b);
    int pts = st_pts(s), saved = st_saved(s);
    /* 1. buys, deck order */
    for (int c = 0; c < NCARDS; c++) {
        int ok = !st_has(s, c);
        for (int i = 0; ok && i < NCOL; i++) {
            int key = g[i] + b[i] < MAXG ? g[i] + b[i] : MAXG;
            if (DECK[c].cost[i] > key) ok = 0;
        }
        if (!ok) continue;
        int ng[NCOL], sv = 0;
        for (int i = 0; i < NCOL; i++) {
            int cc = DECK[c].cost[i] - b[i]; if (cc < 0) cc = 0;
            if (cc < DECK[c].cost[i]) sv += DECK[c].cost[i] - cc;
            int x = g[i] - cc; ng[i] = x < 0 ? 0 : x;
        }
        uint64_t lo = s.lo, hi = s.hi;
        if (c < 64) lo |= 1ull << c; else hi |= 1ull << (c - 64);
        out[n++] = st_make(lo, hi, ng, pts + DECK[c].pt, saved + sv);
    }
    /* 2. takes from the bucketed pattern table (src/gems.py:85-108) */
    int tot = g[0] + g[1] + g[2] + g[3] + g[4];
    if (tot <= 10) {
        int bk = tot <= 7 ? 0 : tot - 7;
        for (int k = 0; k < NPATS[bk]; k++) {
            const pat_t* p = &PATS[bk][k];
            if (p->two_at >= 0 && g[p->two_at] > MAXG - 4) continue;
            int ng[NCOL], ok = 1;
            for (int i = 0; i < NCOL; i++) { ng[i] = g[i] + p->d[i]; if (ng[i] < 0 || ng[i] > MAXG) ok = 0; }
            if (ok) out[n++] = st_make(s.lo, s.hi, ng, pts, saved);
        }
    }
    return n;
}

int oc_successors(uint64_t lo, uint64_t hi, uint64_t* out_lo, uint64_t* out_hi, uint64_t* out_key) {
    st_t kids[256];
    int n = successors((st_t){lo, hi}, kids);
    for (int k = 0; k < n; k++) {
        out_lo[k] = kids[k].lo; out_hi[k] = kids[k].hi;
        out_key[k] = oc_state_key(kids[k].lo, kids[k].hi);
    }
    return n;
}

/* ------------------------------------------------------------------ heuristics */
enum { H_SIMPLE = 0, H_BALANCED = 1, H_AGGRESSIVE = 2, H_EFFICIENCY = 3 };

static double score_base(st_t s, int h, double noise) {
    int b[NCOL]; st_bonus(s, b);
    int pts = st_pts(s), saved = st_saved(s);
    int G = 0, B = 0, U = 0, ncards = 0;
    for (int i = 0; i < NCOL; i++) { G += st_gem(s, i); B += b[i]; U += b[i] > 0; }
    ncards = B;
    switch (h) {
    case H_SIMPLE:      /* src/solver.py:215 */
        return pow((double)saved, 0.4) * pow((double)pts, 2.5) + noise;
    case H_BALANCED: {  /* src/solver.py:229-249 */
        double ps = pow((double)pts, 2.8), ss = pow((double)saved, 0.5);
        double rs = pow((double)(G + B * 2), 0.3), cs = pow((double)ncards, 0.6), ds = pow((double)U, 0.4);
        return ps * 100 + ss * 10 + rs * 5 + cs * 3 + ds * 2 + noise;
    }
    case H_AGGRESSIVE: { /* src/solver.py:257-262 */
        double ps = pow((double)pts, 3.2), ss = pow((double)saved, 0.3), bs = pow((double)B, 0.5);
        return ps * 200 + ss * 5 + bs * 2 + noise;
    }
    default: {          /* efficiency, src/solver.py:271-286 */
        double ps = pow((double)pts, 2.0), ss = pow((double)saved, 0.7);
        double bs = pow((double)B, 1.2), ds = pow((double)U, 0.8);
        return ps * 50 + ss * 30 + bs * 20 + ds * 10 + noise;
    }
    }
}

double oc_score(uint64_t lo, uint64_t hi, int h, int k) { return score_base((st_t){lo, hi}, h, (double)k * 0.01); }

/* ------------------------------------------------------------------ MT19937 (CPython _random) */
typedef struct { uint32_t mt[624]; int idx; uint64_t words; } mt_t;

static uint32_t mt_next(mt_t* m) {
    if (m->idx >= 624) {
        static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
        int kk; uint32_t y;
        for (kk = 0; kk < 624 - 397; kk++) {
            y = (m->mt[kk] & 0x80000000u) | (m->mt[kk + 1] & 0x7fffffffu);
            m->mt[kk] = m->mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1u];
        }
        for (; kk < 623; kk++) {
            y = (m->mt[kk] & 0x80000000u) | (m->mt[kk + 1] & 0x7fffffffu);
            m->mt[kk] = m->mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
        }
        y = (m->mt[623] & 0x80000000u) | (m->mt[0] & 0x7fffffffu);
        m->mt[623] = m->mt[396] ^ (y >> 1) ^ mag01[y & 1u];
        m->idx = 0;
    }
    uint32_t y = m->mt[m->idx++];
    y ^= (y >> 11); y ^= (y << 7) & 0x9d2c5680u; y ^= (y << 15) & 0xefc60000u; y ^= (y >> 18);
    m->words++;
    return y;
}
/* random.randint(1, 100): _randbelow(100) with k = 7 bits */
static int mt_randint100(mt_t* m) {
    for (;;) { uint32_t r = mt_next(m) >> 25; if (r < 100) return (int)r + 1; }
}

/* raw words for tests */
int oc_mt_words(const uint32_t* state625, uint32_t* out, int n) {
    mt_t m; memcpy(m.mt, state625, 624 * 4); m.idx = (int)state625[624]; m.words = 0;
    for (int i = 0; i < n; i++) out[i] = mt_next(&m);
    return 0;
}

/* ------------------------------------------------------------------ visited set (u64 keys) */
/* The trail's capacity never changes a result (membership only).  Large tables (C5: about 2G keys)
 * are reserved up front on 2 MB pages and may fill to 90% instead of doubling past the host's RAM. */
typedef struct { uint64_t* slot; uint64_t mask; uint64_t n; uint64_t soft_cap; } hset_t;
static inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x;
}
static void* big_alloc(size_t bytes) {
    void* p = NULL;
    if (bytes >= (1u << 21)) {
        if (posix_memalign(&p, 1u << 21, bytes)) return NULL;
        madvise(p, bytes, MADV_HUGEPAGE);
        return p;
    }
    return malloc(bytes);
}
static int hs_init(hset_t* h, uint64_t cap_pow2) {
    h->slot = (uint64_t*)big_alloc(cap_pow2 * 8);
    if (!h->slot) return -1;
    memset(h->slot, 0xFF, cap_pow2 * 8);
    h->mask = cap_pow2 - 1; h->n = 0;
    return 0;
}
static int hs_rehash(hset_t* h, uint64_t slots) {
    hset_t g;
    if (hs_init(&g, slots)) return -1;
    g.soft_cap = h->soft_cap;
    for (uint64_t i = 0; i <= h->mask; i++) {
        uint64_t k = h->slot[i];
        if (k == ~0ull) continue;
        uint64_t j = mix64(k) & g.mask;
        while (g.slot[j] != ~0ull) j = (j + 1) & g.mask;
        g.slot[j] = k; g.n++;
    }
    free(h->slot); *h = g;
    return 0;
}
static inline int hs_full(const hset_t* h) {
    uint64_t slots = h->mask + 1;
    if (h->soft_cap && slots >= h->soft_cap) return (h->n + 1) * 10 > slots * 9;
    return (h->n + 1) * 2 > slots;
}
/* returns 1 if inserted (new), 0 if present; key ~0 never occurs (tuple hash maps -1 away) */
static int hs_insert(hset_t* h, uint64_t k) {
    if (hs_full(h) && hs_rehash(h, (h->mask + 1) * 2)) { fprintf(stderr, "oracle: visited set OOM\n"); abort(); }
    uint64_t j = mix64(k) & h->mask;
    for (;;) {
        uint64_t v = h->slot[j];
        if (v == k) return 0;
        if (v == ~0ull) { h->slot[j] = k; h->n++; return 1; }
        j = (j + 1) & h->mask;
    }
}

/* ------------------------------------------------------------------ beam solve handle */
typedef struct {
    st_t* st;        /* states of this turn, queue order (NULL once spilled to the spill file) */
    uint32_t* par;   /* parent rank in previous turn */
    int64_t n;
    int64_t spill_off;
} turn_t;

typedef struct {
    int heuristic, use_heuristic;
    int64_t beam_width;
    int goal;
    int turn;
    int done;
    int64_t winner_rank;
    int max_pts;
    mt_t mt;
    hset_t visited;
    turn_t* turns; int nturns, capturns;
    int spill_fd;    /* >= 0: earlier turns' states live in this (unlinked) file */
    int64_t spill_end;
    FILE* key_dump;  /* analysis: every turn's next_queue score keys (u64, next_queue order) appended here */
} oc_handle;

typedef struct {
    int64_t n_parents, n_raw, n_unique, n_kept;
    int32_t done;
    int64_t winner_rank;
    int32_t n_records;
    int64_t record_rank[32];
    int32_t record_pts[32];
    uint64_t mt_words;
} oc_stats;

static void push_turn(oc_handle* h, st_t* st, uint32_t* par, int64_t n) {
    if (h->nturns == h->capturns) {
        h->capturns = h->capturns ? h->capturns * 2 : 16;
        h->turns = (turn_t*)realloc(h->turns, sizeof(turn_t) * h->capturns);
    }
    h->turns[h->nturns].st = st; h->turns[h->nturns].par = par; h->turns[h->nturns].n = n;
    h->turns[h->nturns].spill_off = -1;
    h->nturns++;
}

/* Memory knobs for the C5-width golden (W=32M; results do not depend on them):
 * reserve the visited set at 2^log2_slots (it then fills to 90% before doubling) and keep every
 * turn but the newest in a spill file under `dir` instead of RAM. */
int oc_set_lean(oc_handle* h, int log2_slots, const char* dir) {
    if (log2_slots > 0) {
        h->visited.soft_cap = 1ull << log2_slots;
        if (h->visited.mask + 1 < h->visited.soft_cap && hs_rehash(&h->visited, h->visited.soft_cap)) return -1;
    }
    if (dir && dir[0]) {
        char path[4096];
        snprintf(path, sizeof path, "%s/oracle_spill_XXXXXX", dir);
        int fd = mkstemp(path);
        if (fd < 0) return -2;
        unlink(path);
        h->spill_fd = fd;
    }
    return 0;
}

/* analysis aid (profiles/analysis/): append each turn's next_queue score keys to `path` */
int oc_dump_keys(oc_handle* h, const char* path) {
    h->key_dump = fopen(path, "wb");
    return h->key_dump ? 0 : -1;
}

static int spill_turn(oc_handle* h, int t) {
    turn_t* tt = &h->turns[t];
    if (h->spill_fd < 0 || !tt->st) return 0;
    const char* p = (const char*)tt->st;
    int64_t left = tt->n * (int64_t)sizeof(st_t), off = h->spill_end;
    while (left > 0) {
        ssize_t w = pwrite(h->spill_fd, p, left > (1 << 30) ? (1 << 30) : left, off);
        if (w <= 0) return -1;
        p += w; off += w; left -= w;
    }
    tt->spill_off = h->spill_end; h->spill_end = off;
    free(tt->st); tt->st = NULL;
    return 0;
}

static st_t turn_state(oc_handle* h, int t, int64_t r) {
    turn_t* tt = &h->turns[t];
    if (tt->st) return tt->st[r];
    st_t s = {0, 0};
    if (pread(h->spill_fd, &s, sizeof s, tt->spill_off + r * (int64_t)sizeof(st_t)) != (ssize_t)sizeof s) abort();
    return s;
}

oc_handle* oc_create(int goal, int use_heuristic, int heuristic, int64_t beam_width,
                     const uint32_t* mt_state625, uint64_t root_lo, uint64_t root_hi) {
    if (!DECK_READY) return NULL;
    oc_handle* h = (oc_handle*)calloc(1, sizeof(oc_handle));
    h->goal = goal; h->use_heuristic = use_heuristic; h->heuristic = heuristic; h->beam_width = beam_width;
    h->spill_fd = -1;
    memcpy(h->mt.mt, mt_state625, 624 * 4); h->mt.idx = (int)mt_state625[624]; h->mt.words = 0;
    hs_init(&h->visited, 1u << 20);
    st_t* root = (st_t*)malloc(sizeof(st_t)); root->lo = root_lo; root->hi = root_hi;
    uint32_t* rp = (uint32_t*)malloc(4); rp[0] = 0xFFFFFFFFu;
    push_turn(h, root, rp, 1);
    hs_insert(&h->visited, oc_state_key(root_lo, root_hi));
    h->winner_rank = -1;
    return h;
}

void oc_destroy(oc_handle* h) {
    if (!h) return;
    for (int t = 0; t < h->nturns; t++) { free(h->turns[t].st); free(h->turns[t].par); }
    if (h->spill_fd >= 0) close(h->spill_fd);
    if (h->key_dump) fclose(h->key_dump);
    free(h->turns); free(h->visited.slot); free(h);
}

/* stable LSD radix sort of (key desc) over indices: returns idx sorted */
static void sort_desc_stable(const uint64_t* key, uint32_t* idx, int64_t n) {
    uint32_t* tmp = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    uint64_t* kk = (uint64_t*)malloc(sizeof(uint64_t) * (n ? n : 1));
    uint64_t* kt = (uint64_t*)malloc(sizeof(uint64_t) * (n ? n : 1));
    for (int64_t i = 0; i < n; i++) { idx[i] = (uint32_t)i; kk[i] = ~key[i]; }  /* ascending on ~key */
    for (int pass = 0; pass < 8; pass++) {
        int sh = pass * 8;
        int64_t cnt[257] = {0};
        for (int64_t i = 0; i < n; i++) cnt[((kk[i] >> sh) & 0xFF) + 1]++;
        if (cnt[((kk[0] >> sh) & 0xFF) + 1] == n) continue;   /* constant digit */
        for (int d = 0; d < 256; d++) cnt[d + 1] += cnt[d];
        for (int64_t i = 0; i < n; i++) {
            int d = (int)((kk[i] >> sh) & 0xFF);
            int64_t p = cnt[d]++;
            tmp[p] = idx[i]; kt[p] = kk[i];
        }
        memcpy(idx, tmp, sizeof(uint32_t) * n); memcpy(kk, kt, sizeof(uint64_t) * n);
    }
    free(tmp); free(kk); free(kt);
}

/* Stable top-W of `key` (descending, ties in index order) as ascending candidate indices: an MSB
 * radix select (16-bit digits) finds the W-th largest value T; every key > T is kept, and the first
 * W - #(> T) keys equal to T in index order.  Returns the count (min(n, W)).  Same set and order as
 * a full stable sort followed by [:W] (src/solver.py:452-456), with sort scratch for W entries only. */
static int64_t select_top(const uint64_t* key, int64_t n, int64_t W, uint32_t* out) {
    if (n <= W) { for (int64_t i = 0; i < n; i++) out[i] = (uint32_t)i; return n; }
    uint64_t prefix = 0, pmask = 0;
    int64_t need = W;
    int64_t* hist = (int64_t*)malloc(sizeof(int64_t) * 65536);
    for (int sh = 48; sh >= 0; sh -= 16) {
        memset(hist, 0, sizeof(int64_t) * 65536);
        for (int64_t i = 0; i < n; i++)
            if ((key[i] & pmask) == prefix) hist[(key[i] >> sh) & 0xFFFF]++;
        int64_t above = 0;
        int d = 65535;
        for (; d > 0 && above + hist[d] < need; d--) above += hist[d];
        need -= above;
        prefix |= (uint64_t)d << sh; pmask |= 0xFFFFull << sh;
    }
    free(hist);
    int64_t m = 0;
    for (int64_t i = 0; i < n; i++) {
        if (key[i] > prefix) out[m++] = (uint32_t)i;
        else if (key[i] == prefix && need > 0) { out[m++] = (uint32_t)i; need--; }
    }
    return m;
}

/* Test entry: the speedrun prune as oc_step runs it (select_top, then the stable sort of the W candidates),
 * as indices into key in kept order; returns the count.  tests/test_oracle.py checks it against a full stable
 * sort followed by [:W] (the reference's sorted(...)[:beam_width], src/solver.py:452-456). */
int64_t oc_debug_prune(const uint64_t* key, int64_t n, int64_t W, uint32_t* out) {
    int64_t k = n < W ? n : W;
    uint32_t* cand = (uint32_t*)malloc(sizeof(uint32_t) * (k ? k : 1));
    int64_t nk = select_top(key, n, k, cand);
    uint64_t* ckey = (uint64_t*)malloc(sizeof(uint64_t) * (nk ? nk : 1));
    uint32_t* idx = (uint32_t*)malloc(sizeof(uint32_t) * (nk ? nk : 1));
    for (int64_t i = 0; i < nk; i++) ckey[i] = key[cand[i]];
    sort_desc_stable(ckey, idx, nk);
    for (int64_t i = 0; i < nk; i++) out[i] = cand[idx[i]];
    free(cand); free(ckey); free(idx);
    return nk;
}

/* One beam step (src/solver.py:434-457). */
int oc_step(oc_handle* h, oc_stats* out) {
    memset(out, 0, sizeof *out);
    if (h->done) { out->done = 1; out->winner_rank = h->winner_rank; return 0; }
    int tcur = h->nturns - 1;
    turn_t* cur = &h->turns[tcur];
    out->n_parents = cur->n;
    /* goal check + max_pts records in queue order (:438-445) */
    for (int64_t r = 0; r < cur->n; r++) {
        int p = st_pts(cur->st[r]);
        if (p > h->max_pts) {
            h->max_pts = p;
            if (out->n_records < 32) { out->record_rank[out->n_records] = r; out->record_pts[out->n_records] = p; out->n_records++; }
        }
        if (p >= h->goal) {
            h->done = 1; h->winner_rank = r;
            out->done = 1; out->winner_rank = r; out->mt_words = h->mt.words;
            return 0;
        }
    }
    /* expansion + trail dedup (:446-450).  Children of PB parents are generated and their slots
     * prefetched together, then inserted one by one in (parent rank, ordinal) order. */
    enum { PB = 16 };
    int64_t cap = cur->n * 32 + 256, nq = 0, nraw = 0;
    st_t* nxt = (st_t*)big_alloc(sizeof(st_t) * cap);
    uint32_t* npar = (uint32_t*)big_alloc(sizeof(uint32_t) * cap);
    static __thread st_t kids[PB * 256];
    static __thread uint64_t kkey[PB * 256];
    static __thread int kcnt[PB];
    for (int64_t r0 = 0; r0 < cur->n; r0 += PB) {
        int np = cur->n - r0 < PB ? (int)(cur->n - r0) : PB, tot = 0;
        for (int j = 0; j < np; j++) {
            int nk = successors(cur->st[r0 + j], kids + tot);
            for (int k = 0; k < nk; k++) {
                uint64_t key = oc_state_key(kids[tot + k].lo, kids[tot + k].hi);
                kkey[tot + k] = key;
                __builtin_prefetch(&h->visited.slot[mix64(key) & h->visited.mask]);
            }
            kcnt[j] = nk; tot += nk;
        }
        nraw += tot;
        for (int j = 0, e = 0; j < np; j++) {
            for (int k = 0; k < kcnt[j]; k++, e++) {
                if (!hs_insert(&h->visited, kkey[e])) continue;
                if (nq == cap) {
                    cap *= 2;
                    nxt = (st_t*)realloc(nxt, sizeof(st_t) * cap);
                    npar = (uint32_t*)realloc(npar, sizeof(uint32_t) * cap);
                }
                nxt[nq] = kids[e]; npar[nq] = (uint32_t)(r0 + j); nq++;
            }
        }
    }
    out->n_raw = nraw; out->n_unique = nq;
    if (nq == 0) {           /* queue empties: `puzzle` is the last parent (:438, :459) */
        h->done = 1; h->winner_rank = cur->n - 1;
        out->done = 1; out->winner_rank = cur->n - 1; out->mt_words = h->mt.words;
        free(nxt); free(npar);
        return 0;
    }
    if (h->use_heuristic) {  /* sorted(next_queue, key=heuristic, reverse=True)[:beam_width] (:452-456) */
        uint64_t* key = (uint64_t*)big_alloc(sizeof(uint64_t) * nq);
        for (int64_t i = 0; i < nq; i++) {
            double sc = score_base(nxt[i], h->heuristic, (double)mt_randint100(&h->mt) * 0.01);
            memcpy(&key[i], &sc, 8);   /* scores are > 0: IEEE bits order == numeric order */
        }
        if (h->key_dump) {
            int64_t nn = nq;
            fwrite(&nn, 8, 1, h->key_dump);
            fwrite(key, 8, (size_t)nq, h->key_dump);
        }
        int64_t W = nq < h->beam_width ? nq : h->beam_width;
        uint32_t* cand = (uint32_t*)malloc(sizeof(uint32_t) * (W ? W : 1));
        int64_t nk = select_top(key, nq, W, cand);
        uint64_t* ckey = (uint64_t*)malloc(sizeof(uint64_t) * (nk ? nk : 1));
        uint32_t* idx = (uint32_t*)malloc(sizeof(uint32_t) * (nk ? nk : 1));
        for (int64_t i = 0; i < nk; i++) ckey[i] = key[cand[i]];
        free(key);
        sort_desc_stable(ckey, idx, nk);
        st_t* ks = (st_t*)malloc(sizeof(st_t) * (nk ? nk : 1));
        uint32_t* kp = (uint32_t*)malloc(sizeof(uint32_t) * (nk ? nk : 1));
        for (int64_t i = 0; i < nk; i++) { ks[i] = nxt[cand[idx[i]]]; kp[i] = npar[cand[idx[i]]]; }
        free(ckey); free(idx); free(cand); free(nxt); free(npar);
        push_turn(h, ks, kp, nk);
        out->n_kept = nk;
    } else {
        push_turn(h, nxt, npar, nq);
        out->n_kept = nq;
    }
    if (spill_turn(h, tcur)) return -3;
    h->turn++;
    out->mt_words = h->mt.words;
    return 0;
}

int64_t oc_turn_size(oc_handle* h, int t) { return (t < 0 || t >= h->nturns) ? -1 : h->turns[t].n; }
int oc_nturns(oc_handle* h) { return h->nturns; }

int oc_read_turn(oc_handle* h, int t, int64_t start, int64_t n, uint64_t* lo, uint64_t* hi, uint32_t* par, uint64_t* key) {
    if (t < 0 || t >= h->nturns) return -1;
    turn_t* tt = &h->turns[t];
    if (start < 0 || start + n > tt->n) return -2;
    st_t* blk = tt->st ? tt->st + start : NULL;
    if (!blk) {   /* spilled turn: one read of the range */
        blk = (st_t*)malloc(sizeof(st_t) * (n ? n : 1));
        const int64_t bytes = n * (int64_t)sizeof(st_t);
        for (int64_t done = 0; done < bytes;) {
            ssize_t r = pread(h->spill_fd, (char*)blk + done, bytes - done, tt->spill_off + start * (int64_t)sizeof(st_t) + done);
            if (r <= 0) { free(blk); return -3; }
            done += r;
        }
    }
    for (int64_t i = 0; i < n; i++) {
        st_t s = blk[i];
        if (lo) lo[i] = s.lo;
        if (hi) hi[i] = s.hi;
        if (par) par[i] = tt->par[start + i];
        if (key) key[i] = oc_state_key(s.lo, s.hi);
    }
    if (blk != (tt->st ? tt->st + start : NULL)) free(blk);
    return 0;
}

/* root..winner path (src/solver.py:459-464); out arrays hold `cap` states */
int oc_path(oc_handle* h, uint64_t* lo, uint64_t* hi, int cap) {
    if (!h->done) return -1;
    int t = h->nturns - 1;
    int64_t r = h->winner_rank;
    int len = t + 1;
    if (len > cap) return -2;
    for (; t >= 0; t--) {
        st_t s = turn_state(h, t, r);
        lo[t] = s.lo; hi[t] = s.hi;
        r = (int64_t)h->turns[t].par[r];
    }
    return len;
}

int oc_get_mt_state(oc_handle* h, uint32_t* out625) {
    memcpy(out625, h->mt.mt, 624 * 4); out625[624] = (uint32_t)h->mt.idx;
    return 0;
}
uint64_t oc_visited_size(oc_handle* h) { return h->visited.n; }
/* the trail's keys (any order), at most cap; returns the count written */
int64_t oc_visited_keys(oc_handle* h, uint64_t* out, int64_t cap) {
    int64_t m = 0;
    for (uint64_t i = 0; i <= h->visited.mask && m < cap; i++)
        if (h->visited.slot[i] != ~0ull) out[m++] = h->visited.slot[i];
    return m;
}

/* ====================================================================================== */
/* Realistic multi-player mode (src/solver.py:25-200, 471-860): TEST INFRASTRUCTURE ONLY.
 *
 *   MultiPlayerState.__hash__ = hash((players, pool, visible, current_player))   (:495-500)
 *     with PlayerState hashed as its field tuple (player_id, cards, bonus, gems, pts, saved)
 *   __iter__: buys over visible cards t1+t2+t3 (:574-632, can_afford :192-200, market.buy_card
 *     :121-170 appends the deck head to the END of the tier, pool.return_gems :75-80, final-round
 *     bookkeeping :606-615), then realistic takes (:664-748): combinations of available colours
 *     taken 3 (hand + 3 <= 10), then 2-same by colour (pool >= 4, hand + 2 <= 10)
 *   solve (:750-860): is_game_over before the max_pts record, always sorts with
 *     multi_competitive_heuristic (:778-812), 1000-turn cap (:849-852)
 *
 * Packed form (12 x u64, shared with the engine and the host):
 *   w[2i], w[2i+1]  player i (i < 4): cards lo | hi = cards 64..89, gems 26+3c, pts 41..48, saved 49..63
 *   w[8]  pool 3 bits x5 (0..14) | cp 15..16 | frt 17 | frp 18..20 (7 = None) | deck pointers 6 bits
 *         x3 (21..38) | visible counts 3 bits x3 (39..47)
 *   w[9]  tier-1 visible 4 x 7 bits (0..27), tier-2 visible (28..55);  w[10] tier-3 visible (0..27)
 *   w[11] infinite_resources=True only: pool 12 bits x5 (it grows by the gems paid for cards; the
 *         3-bit pool field of w[8] is then 0)
 * infinite_resources=True (:635-659): takes are the speedrun take table of the current player's gems
 * (get_takes()[gems], the pool untouched); buys as above (the pool grows by the gems paid).
 */
#define RW 12
typedef struct { int P, target; int tier[3][40]; int tlen[3]; int inf; } rgame_t;
typedef struct { uint64_t w[RW]; } rst_t;

static inline int r_pool(const rgame_t* G, const rst_t* s, int c) {
    return G->inf ? (int)((s->w[11] >> (12 * c)) & 4095) : (int)((s->w[8] >> (3 * c)) & 7);
}
static inline int r_cp(const rst_t* s) { return (int)((s->w[8] >> 15) & 3); }
static inline int r_frt(const rst_t* s) { return (int)((s->w[8] >> 17) & 1); }
static inline int r_frp(const rst_t* s) { int v = (int)((s->w[8] >> 18) & 7); return v == 7 ? -1 : v; }
static inline int r_dptr(const rst_t* s, int t) { return (int)((s->w[8] >> (21 + 6 * t)) & 63); }
static inline int r_nvis(const rst_t* s, int t) { return (int)((s->w[8] >> (39 + 3 * t)) & 7); }
static inline int r_vis(const rst_t* s, int t, int j) {
    uint64_t w = t < 2 ? s->w[9] >> (28 * t) : s->w[10];
    return (int)((w >> (7 * j)) & 127);
}
static inline st_t r_player(const rst_t* s, int i) { st_t p = {s->w[2 * i], s->w[2 * i + 1]}; return p; }
static inline void r_set_player(rst_t* s, int i, st_t p) { s->w[2 * i] = p.lo; s->w[2 * i + 1] = p.hi; }

static void r_set_meta(const rgame_t* G, rst_t* s, const int pool[5], int cp, int frt, int frp, const int dptr[3],
                       const int nvis[3], const int vis[3][4]) {
    uint64_t m = 0;
    if (G->inf) {
        uint64_t w11 = 0;
        for (int c = 0; c < 5; c++) w11 |= (uint64_t)pool[c] << (12 * c);
        s->w[11] = w11;
    } else {
        for (int c = 0; c < 5; c++) m |= (uint64_t)pool[c] << (3 * c);
    }
    m |= (uint64_t)cp << 15;
    m |= (uint64_t)(frt ? 1 : 0) << 17;
    m |= (uint64_t)(frp < 0 ? 7 : frp) << 18;
    for (int t = 0; t < 3; t++) m |= (uint64_t)dptr[t] << (21 + 6 * t);
    for (int t = 0; t < 3; t++) m |= (uint64_t)nvis[t] << (39 + 3 * t);
    s->w[8] = m;
    uint64_t v0 = 0, v1 = 0;
    for (int t = 0; t < 3; t++)
        for (int j = 0; j < nvis[t]; j++) {
            uint64_t c = (uint64_t)vis[t][j];
            if (t == 0) v0 |= c << (7 * j);
            else if (t == 1) v0 |= c << (28 + 7 * j);
            else v1 |= c << (7 * j);
        }
    s->w[9] = v0;
    s->w[10] = v1;
}

static uint64_t th_tuple(const uint64_t* lanes, int n) {
    uint64_t acc = XXP5;
    for (int i = 0; i < n; i++) acc = th_step(acc, lanes[i]);
    return th_fin(acc, (uint64_t)n);
}

static uint64_t r_key(const rgame_t* G, const rst_t* s) {
    uint64_t hp[4];
    for (int i = 0; i < G->P; i++) {
        st_t p = r_player(s, i);
        int b[NCOL], g[NCOL];
        st_bonus(p, b);
        uint64_t lb[5], lg[5];
        for (int c = 0; c < 5; c++) { lb[c] = (uint64_t)b[c]; g[c] = st_gem(p, c); lg[c] = (uint64_t)g[c]; }
        uint64_t f[6] = {(uint64_t)i, hash_cards(p), th_tuple(lb, 5), th_tuple(lg, 5), (uint64_t)st_pts(p),
                         (uint64_t)st_saved(p)};
        hp[i] = th_tuple(f, 6);
    }
    uint64_t lp[5], lv[12];
    for (int c = 0; c < 5; c++) lp[c] = (uint64_t)r_pool(G, s, c);
    int nv = 0;
    for (int t = 0; t < 3; t++)
        for (int j = 0; j < r_nvis(s, t); j++) lv[nv++] = (uint64_t)r_vis(s, t, j);
    uint64_t outer[4] = {th_tuple(hp, G->P), th_tuple(lp, 5), th_tuple(lv, nv), (uint64_t)r_cp(s)};
    return th_tuple(outer, 4);
}

static int r_can_afford(st_t p, int c) {
    int b[NCOL];
    st_bonus(p, b);
    for (int i = 0; i < NCOL; i++)
        if (st_gem(p, i) + b[i] < DECK[c].cost[i]) return 0;
    return 1;
}

static void r_unpack_meta(const rgame_t* G, const rst_t* s, int pool[5], int dptr[3], int nvis[3], int vis[3][4]) {
    for (int c = 0; c < 5; c++) pool[c] = r_pool(G, s, c);
    for (int t = 0; t < 3; t++) {
        dptr[t] = r_dptr(s, t);
        nvis[t] = r_nvis(s, t);
        for (int j = 0; j < nvis[t]; j++) vis[t][j] = r_vis(s, t, j);
    }
}

static int r_successors(const rgame_t* G, const rst_t* s, rst_t* out) {
    const int cur = r_cp(s), nxt = (cur + 1) % G->P, frt = r_frt(s), frp = r_frp(s);
    int pool[5], dptr[3], nvis[3], vis[3][4];
    r_unpack_meta(G, s, pool, dptr, nvis, vis);
    st_t me = r_player(s, cur);
    int g[NCOL], b[NCOL];
    for (int c = 0; c < NCOL; c++) g[c] = st_gem(me, c);
    st_bonus(me, b);
    int n = 0;
    for (int t = 0; t < 3; t++)
        for (int j = 0; j < nvis[t]; j++) {       /* buys, visible order t1+t2+t3 */
            const int card = vis[t][j];
            if (st_has(me, card) || !r_can_afford(me, card)) continue;
            int ng[NCOL], sv = 0, np[5];
            for (int c = 0; c < NCOL; c++) {
                int cc = DECK[card].cost[c] - b[c]; if (cc < 0) cc = 0;
                if (cc < DECK[card].cost[c]) sv += DECK[card].cost[c] - cc;
                int x = g[c] - cc; ng[c] = x < 0 ? 0 : x;
                np[c] = pool[c] + (g[c] - ng[c]);
            }
            uint64_t lo = me.lo, hi = me.hi;
            if (card < 64) lo |= 1ull << card; else hi |= 1ull << (card - 64);
            const int npts = st_pts(me) + DECK[card].pt;
            st_t pl = st_make(lo, hi, ng, npts, st_saved(me) + sv);
            int nv2[3] = {nvis[0], nvis[1], nvis[2]}, vis2[3][4], dp2[3] = {dptr[0], dptr[1], dptr[2]};
            memcpy(vis2, vis, sizeof vis2);
            for (int k = j; k + 1 < nv2[t]; k++) vis2[t][k] = vis2[t][k + 1];
            nv2[t]--;
            if (dp2[t] < G->tlen[t] - 4) { vis2[t][nv2[t]++] = G->tier[t][4 + dp2[t]]; dp2[t]++; }
            const int frt2 = frt || npts >= G->target;
            const int frp2 = frt ? frp : (frt2 ? cur : -1);
            rst_t c2 = *s;
            r_set_player(&c2, cur, pl);
            r_set_meta(G, &c2, np, nxt, frt2, frp2, dp2, nv2, vis2);
            out[n++] = c2;
        }
    if (G->inf) {                                 /* speedrun take table, pool untouched (:635-659) */
        const int tot = g[0] + g[1] + g[2] + g[3] + g[4];
        if (tot <= 10) {
            const int bk = tot <= 7 ? 0 : tot - 7;
            for (int k = 0; k < NPATS[bk]; k++) {
                const pat_t* p = &PATS[bk][k];
                if (p->two_at >= 0 && g[p->two_at] > MAXG - 4) continue;
                int ng[NCOL], ok = 1;
                for (int i = 0; i < NCOL; i++) { ng[i] = g[i] + p->d[i]; if (ng[i] < 0 || ng[i] > MAXG) ok = 0; }
                if (!ok) continue;
                rst_t c2 = *s;
                r_set_player(&c2, cur, st_make(me.lo, me.hi, ng, st_pts(me), st_saved(me)));
                r_set_meta(G, &c2, pool, nxt, frt, frp, dptr, nvis, vis);
                out[n++] = c2;
            }
        }
        return n;
    }
    int avail[5], na = 0, tot = 0;
    for (int c = 0; c < 5; c++) { if (pool[c] > 0) avail[na++] = c; tot += g[c]; }
    for (int x = 0; x < na; x++)                  /* combinations(available, 3) */
        for (int y = x + 1; y < na; y++)
            for (int z = y + 1; z < na; z++) {
                if (tot + 3 > 10) continue;
                int ng[NCOL], np[5];
                for (int c = 0; c < 5; c++) { ng[c] = g[c]; np[c] = pool[c]; }
                int cs[3] = {avail[x], avail[y], avail[z]};
                for (int k = 0; k < 3; k++) { ng[cs[k]]++; np[cs[k]]--; }
                rst_t c2 = *s;
                r_set_player(&c2, cur, st_make(me.lo, me.hi, ng, st_pts(me), st_saved(me)));
                r_set_meta(G, &c2, np, nxt, frt, frp, dptr, nvis, vis);
                out[n++] = c2;
            }
    for (int x = 0; x < na; x++) {                /* two of one colour */
        const int c0 = avail[x];
        if (pool[c0] < 4 || tot + 2 > 10) continue;
        int ng[NCOL], np[5];
        for (int c = 0; c < 5; c++) { ng[c] = g[c]; np[c] = pool[c]; }
        ng[c0] += 2; np[c0] -= 2;
        rst_t c2 = *s;
        r_set_player(&c2, cur, st_make(me.lo, me.hi, ng, st_pts(me), st_saved(me)));
        r_set_meta(G, &c2, np, nxt, frt, frp, dptr, nvis, vis);
        out[n++] = c2;
    }
    return n;
}

/* multi_competitive_heuristic (src/solver.py:778-812) */
static double r_score(const rgame_t* G, const rst_t* s, double noise) {
    const int cp = r_cp(s), prev = ((cp - 1) % G->P + G->P) % G->P;
    st_t me = r_player(s, prev), op = r_player(s, cp);
    int bm[NCOL], bo[NCOL];
    st_bonus(me, bm);
    st_bonus(op, bo);
    const int mp = st_pts(me), opp = st_pts(op);
    double pd = mp > opp ? pow((double)(mp - opp), 2.5) : -pow((double)(opp - mp), 2.5);
    int mr = 0, orr = 0, div = 0;
    for (int c = 0; c < NCOL; c++) { mr += st_gem(me, c) + bm[c] * 2; orr += st_gem(op, c) + bo[c] * 2; div += bm[c] > 0; }
    double rd = mr > orr ? pow((double)(mr - orr), 0.5) : 0.0;
    int ma = 0, oa = 0;
    for (int t = 0; t < 3; t++)
        for (int j = 0; j < r_nvis(s, t); j++) { int c = r_vis(s, t, j); ma += r_can_afford(me, c); oa += r_can_afford(op, c); }
    const int mc = (ma - oa) * 5;
    double r = pd * 100;
    r = r + rd * 20;
    r = r + (double)mc;
    r = r + pow((double)div, 0.5) * 3;
    return r + noise;
}

static int r_game_over(const rgame_t* G, const rst_t* s) {
    if (!r_frt(s)) {
        for (int i = 0; i < G->P; i++) if (st_pts(r_player(s, i)) >= G->target) return 1;
        return 0;
    }
    return r_cp(s) == r_frp(s);
}

/* total order of doubles as u64 (negatives flipped, -0.0 == +0.0 as in Python) */
static inline uint64_t f64_key(double d) {
    if (d == 0.0) d = 0.0;
    uint64_t u;
    memcpy(&u, &d, 8);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

/* ---- ctypes surface for tests */
/* params: [players, target, tier lengths x3, infinite_resources] */
static int r_load_game(rgame_t* G, const int32_t* params, const int32_t* tiers) {
    G->P = params[0]; G->target = params[1]; G->inf = params[5] != 0;
    for (int t = 0; t < 3; t++) { G->tlen[t] = params[2 + t]; for (int k = 0; k < G->tlen[t]; k++) G->tier[t][k] = tiers[t * 40 + k]; }
    return (G->P >= 2 && G->P <= 4) ? 0 : -1;
}

uint64_t ort_key(const int32_t* params, const int32_t* tiers, const uint64_t* w) {
    rgame_t G; r_load_game(&G, params, tiers);
    rst_t s; memcpy(s.w, w, sizeof s.w);
    return r_key(&G, &s);
}

int ort_successors(const int32_t* params, const int32_t* tiers, const uint64_t* w, uint64_t* out, uint64_t* keys) {
    rgame_t G; r_load_game(&G, params, tiers);
    rst_t s; memcpy(s.w, w, sizeof s.w);
    rst_t kids[128];
    int n = r_successors(&G, &s, kids);
    for (int k = 0; k < n; k++) { memcpy(out + k * RW, kids[k].w, sizeof kids[k].w); keys[k] = r_key(&G, &kids[k]); }
    return n;
}

double ort_score(const int32_t* params, const int32_t* tiers, const uint64_t* w, int k) {
    rgame_t G; r_load_game(&G, params, tiers);
    rst_t s; memcpy(s.w, w, sizeof s.w);
    return r_score(&G, &s, (double)k * 0.01);
}

int ort_game_over(const int32_t* params, const int32_t* tiers, const uint64_t* w) {
    rgame_t G; r_load_game(&G, params, tiers);
    rst_t s; memcpy(s.w, w, sizeof s.w);
    return r_game_over(&G, &s);
}

/* ---- realistic beam solve (src/solver.py:774-860) */
typedef struct { rst_t* st; uint32_t* par; int64_t n; } rturn_t;
typedef struct {
    rgame_t G;
    int64_t beam_width;
    int turn, done, max_pts;
    int64_t winner_rank;
    mt_t mt;
    hset_t visited;
    rturn_t* turns; int nturns, capturns;
} ort_handle;

static void r_push(ort_handle* h, rst_t* st, uint32_t* par, int64_t n) {
    if (h->nturns == h->capturns) {
        h->capturns = h->capturns ? h->capturns * 2 : 64;
        h->turns = (rturn_t*)realloc(h->turns, sizeof(rturn_t) * h->capturns);
    }
    h->turns[h->nturns].st = st; h->turns[h->nturns].par = par; h->turns[h->nturns].n = n;
    h->nturns++;
}

ort_handle* ort_create(const int32_t* params, const int32_t* tiers, int64_t beam_width, const uint32_t* mt_state625,
                       const uint64_t* root_w) {
    if (!DECK_READY) return NULL;
    ort_handle* h = (ort_handle*)calloc(1, sizeof(ort_handle));
    if (r_load_game(&h->G, params, tiers)) { free(h); return NULL; }
    h->beam_width = beam_width;
    memcpy(h->mt.mt, mt_state625, 624 * 4); h->mt.idx = (int)mt_state625[624];
    hs_init(&h->visited, 1u << 16);
    rst_t* root = (rst_t*)malloc(sizeof(rst_t)); memcpy(root->w, root_w, sizeof root->w);
    uint32_t* rp = (uint32_t*)malloc(4); rp[0] = 0xFFFFFFFFu;
    r_push(h, root, rp, 1);
    hs_insert(&h->visited, r_key(&h->G, root));
    h->winner_rank = -1;
    return h;
}

void ort_destroy(ort_handle* h) {
    if (!h) return;
    for (int t = 0; t < h->nturns; t++) { free(h->turns[t].st); free(h->turns[t].par); }
    free(h->turns); free(h->visited.slot); free(h);
}

int ort_step(ort_handle* h, oc_stats* out) {
    memset(out, 0, sizeof *out);
    if (h->done) { out->done = 1; out->winner_rank = h->winner_rank; return 0; }
    rturn_t* cur = &h->turns[h->nturns - 1];
    out->n_parents = cur->n;
    for (int64_t r = 0; r < cur->n; r++) {       /* game over first, then the record (:826-836) */
        if (r_game_over(&h->G, &cur->st[r])) {
            h->done = 1; h->winner_rank = r; out->done = 1; out->winner_rank = r; out->mt_words = h->mt.words;
            return 0;
        }
        int mp = 0;
        for (int i = 0; i < h->G.P; i++) { int p = st_pts(r_player(&cur->st[r], i)); if (p > mp) mp = p; }
        if (mp > h->max_pts) {
            h->max_pts = mp;
            if (out->n_records < 32) { out->record_rank[out->n_records] = r; out->record_pts[out->n_records] = mp; out->n_records++; }
        }
    }
    int64_t cap = cur->n * 32 + 64, nq = 0, nraw = 0;
    rst_t* nxt = (rst_t*)malloc(sizeof(rst_t) * cap);
    uint32_t* npar = (uint32_t*)malloc(sizeof(uint32_t) * cap);
    rst_t kids[128];
    for (int64_t r = 0; r < cur->n; r++) {
        int nk = r_successors(&h->G, &cur->st[r], kids);
        nraw += nk;
        for (int k = 0; k < nk; k++) {
            if (!hs_insert(&h->visited, r_key(&h->G, &kids[k]))) continue;
            if (nq == cap) { cap *= 2; nxt = (rst_t*)realloc(nxt, sizeof(rst_t) * cap); npar = (uint32_t*)realloc(npar, 4 * cap); }
            nxt[nq] = kids[k]; npar[nq] = (uint32_t)r; nq++;
        }
    }
    out->n_raw = nraw; out->n_unique = nq;
    if (nq == 0) {
        h->done = 1; h->winner_rank = cur->n - 1; out->done = 1; out->winner_rank = cur->n - 1;
        free(nxt); free(npar); out->mt_words = h->mt.words;
        return 0;
    }
    uint64_t* key = (uint64_t*)malloc(8 * nq);
    uint32_t* idx = (uint32_t*)malloc(4 * nq);
    for (int64_t i = 0; i < nq; i++) key[i] = f64_key(r_score(&h->G, &nxt[i], (double)mt_randint100(&h->mt) * 0.01));
    sort_desc_stable(key, idx, nq);
    int64_t nk = nq < h->beam_width ? nq : h->beam_width;
    rst_t* ks = (rst_t*)malloc(sizeof(rst_t) * nk);
    uint32_t* kp = (uint32_t*)malloc(4 * nk);
    for (int64_t i = 0; i < nk; i++) { ks[i] = nxt[idx[i]]; kp[i] = npar[idx[i]]; }
    free(key); free(idx); free(nxt); free(npar);
    r_push(h, ks, kp, nk);
    out->n_kept = nk;
    h->turn++;
    if (h->turn > 1000) {   /* safety cap (:849-852): `puzzle` is the last parent of this turn */
        h->done = 1; h->winner_rank = cur->n - 1; out->done = 1; out->winner_rank = cur->n - 1;
        /* the reference stops with the previous queue's last state; drop the new turn from the path */
        h->nturns--; free(ks); free(kp);
    }
    out->mt_words = h->mt.words;
    return 0;
}

int64_t ort_turn_size(ort_handle* h, int t) { return (t < 0 || t >= h->nturns) ? -1 : h->turns[t].n; }
int ort_nturns(ort_handle* h) { return h->nturns; }
int ort_read_turn(ort_handle* h, int t, uint64_t* w, uint32_t* par, uint64_t* key) {
    if (t < 0 || t >= h->nturns) return -1;
    rturn_t* tt = &h->turns[t];
    for (int64_t i = 0; i < tt->n; i++) {
        if (w) memcpy(w + i * RW, tt->st[i].w, 8 * RW);
        if (par) par[i] = tt->par[i];
        if (key) key[i] = r_key(&h->G, &tt->st[i]);
    }
    return 0;
}
int ort_path(ort_handle* h, uint64_t* w, int cap) {
    if (!h->done) return -1;
    int t = h->nturns - 1;
    int64_t r = h->winner_rank;
    if (t + 1 > cap) return -2;
    int len = t + 1;
    for (; t >= 0; t--) { memcpy(w + t * RW, h->turns[t].st[r].w, 8 * RW); r = (int64_t)h->turns[t].par[r]; }
    return len;
}
int ort_get_mt_state(ort_handle* h, uint32_t* out625) {
    memcpy(out625, h->mt.mt, 624 * 4); out625[624] = (uint32_t)h->mt.idx; return 0;
}
