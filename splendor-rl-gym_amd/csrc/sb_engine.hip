// sb_engine.hip — MI355X beam-search step engine for the Splendor speedrun solver.
//
// One sb_step() = one iteration of `while queue:` in State.solve (src/solver.py:434-457):
//
//   goal check      first queue state with pts >= goal wins (src/solver.py:443-445) — from the
//                   per-pts first-rank table built by the previous step's gather (no extra pass)
//   k_expand        block-cooperative successor enumeration (buys in deck order, then takes,
//                   src/solver.py:357-388) into an LDS child queue; the queue is then processed
//                   densely (one child per lane): CPython tuple hash, visited-set probe/insert and
//                   an atomicMin claim of the child's (turn, parent rank, ordinal) tag
//                   — a claimant that displaces a same-turn holder marks it lost, so a child
//                   survives iff it claimed and was never displaced: exactly
//                   `if next_step in trail: continue` with first-occurrence order (src/solver.py:446-450)
//   scan            survivor counts (cand & ~lost) -> next_queue offsets (parent rank, ordinal order)
//   k_emit_w        survivors' packed states, parent links and heuristic scores, built densely 64 at a
//                   time (sb_wave.inc); the noise of next_queue element k is the k-th accepted MT19937
//                   draw (sb_mt.hip)
//   top-k           stable descending sort + truncate (src/solver.py:452-456; sb_sort.hip)
//   k_gather        the kept beam for the next turn + the per-pts first-rank table
//
// Visited set: open addressing over 16-byte entries {key, tag}; tag = EMPTY marks a free slot (the tag is
// claimed first, the key stored after: probe_insert).
// The tag is (turn+1) << 40 | parent rank << 8 | ordinal; tag prefix 0 is the root's turn.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "../../include/splendor_beam.h"
#include "sb_block.h"
#include "sb_device.h"
#include "sb_internal.h"

namespace sb {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

static std::string gib(double b) {
    char buf[64];
    snprintf(buf, sizeof buf, "%.3f GiB", b / (double)(1ull << 30));
    return buf;
}

std::string oom_message(const char* what, size_t bytes, hipError_t code) {
    std::string m = std::string(what) + ": hipMalloc of " + gib((double)bytes) + " (" + std::to_string(bytes) +
                    " bytes) failed: " + hipGetErrorString(code);
    size_t freeb = 0, totalb = 0;
    const hipError_t e = hipMemGetInfo(&freeb, &totalb);
    if (e == hipSuccess) m += "; free HBM " + gib((double)freeb) + " of " + gib((double)totalb);
    else m += std::string("; free HBM unknown (hipMemGetInfo: ") + hipGetErrorString(e) + ")";
    (void)hipGetLastError();
    return m;
}

// SB_DEBUG_HBM_LIMIT (tests): allocations above it fail as if the HBM were full
static bool debug_hbm_allows(size_t bytes) {
    static const char* lim = std::getenv("SB_DEBUG_HBM_LIMIT");
    return !lim || (double)bytes <= std::strtod(lim, nullptr);
}

void dev_malloc(void** p, size_t bytes, const char* what) {
    static const char* lim = std::getenv("SB_DEBUG_HBM_LIMIT");
    hipError_t e;
    if (lim && (double)bytes > std::strtod(lim, nullptr)) {
        e = hipErrorOutOfMemory;
        throw HipError{e, oom_message(what, bytes, e) + " [SB_DEBUG_HBM_LIMIT=" + lim + "]"};
    }
    e = hipMalloc(p, bytes);
    if (e != hipSuccess) {
        *p = nullptr;
        (void)hipGetLastError();
        throw HipError{e, oom_message(what, bytes, e)};
    }
}

static Tables g_host_tables;
static bool g_tables_ready = false;

struct alignas(16) Entry {
    uint64_t key;
    uint64_t tag;
};

constexpr int MAX_PROBE = 4096;

// ------------------------------------------------------------------ visited-set probe
// Slot protocol (tag first): a free slot has tag == EMPTY.  An inserter claims the slot AND sets its tag
// with one 64-bit CAS on the tag word, then stores the key (write-through to L2).  A reader that finds a
// tag but no key yet (the inserter's store is in flight) reads the slot again on its next loop iteration;
// the inserter never waits on anyone and its store precedes that re-read in the wave's instruction
// stream, so the wait always ends (a spin inside one iteration could deadlock a wave whose own lane won).  A new key thus costs one CAS + one store instead of
// a key CAS + a tag atomicMin (profiles/micro/r1_claimcost.txt: cas+st_sc1 12.1 G/s vs cas+amin 10.6 G/s
// over a 32 GiB table).  -DSB_KEY_FIRST builds the previous protocol (key CAS, then atomicMin of the tag).
//
// probe_insert: returns 1 when this call inserted `key` (its tag is in place), 0 when the key was
// found (slot h, tag *cur as read: stale reads only over-estimate, tags only decrease), -1 on overflow.
// losing CAS attempts store here (see probe_insert); spread over 256 lines so they do not serialise
__device__ unsigned long long g_claim_sink[4096];

// hash(gems) of every 15-bit gem field (5 x 3 bits), 256 KB, L2-resident: the sharded key passes (VALU-bound: nothing
// to hide the hashing under, unlike k_expand's probes) look a child's gem hash up instead of folding five lanes
__device__ uint64_t g_hgems[1 << 15];
__global__ void k_init_hgems() {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < (1 << 15)) g_hgems[i] = hash_gems((uint32_t)i);
}
__device__ __forceinline__ uint64_t hash_gems_t(uint32_t gf) { return g_hgems[gf & 0x7FFFu]; }

// Probe loads of the visited set.  -DSB_PROBE_NT=1 makes them non-temporal (global_load_dwordx4 ... nt):
// alone, a random 16-B nt probe of a 32 GiB table runs at the cache-resident rate (54 G/s against 48 G/s,
// profiles/micro/r2_randaccess2.txt), but inside k_expand it is 33% slower (expand 3.42 -> 4.56 ms,
// profiles/r2_ab_probe_nt.txt): the probe's plain load leaves the line where the tag CAS that follows on
// the same line finds it.  Plain loads are the default.
#ifndef SB_PROBE_NT
#define SB_PROBE_NT 0
#endif
__device__ __forceinline__ ulonglong2 load_entry(const Entry* __restrict__ e) {
#if SB_PROBE_NT
    const unsigned long long* p = reinterpret_cast<const unsigned long long*>(e);
    return make_ulonglong2(__builtin_nontemporal_load(p), __builtin_nontemporal_load(p + 1));
#else
    return *reinterpret_cast<const ulonglong2*>(e);
#endif
}

template <bool PRE>
__device__ __forceinline__ int probe_insert(Entry* __restrict__ tab, uint64_t mask, uint64_t key, ulonglong2 ent,
                                            uint64_t tag, uint64_t& h, uint64_t& cur, uint32_t* err) {
    h = mix64(key) & mask;
    int wait = 0;
    for (int probe = 0;;) {
        if (!PRE || probe > 0 || wait > 0) ent = load_entry(&tab[h]);   // key and tag, one load
        uint64_t k = ent.x, tg = ent.y;
#ifndef SB_KEY_FIRST
        if (tg == EMPTY) {
            const uint64_t prev = atomicCAS((unsigned long long*)&tab[h].tag, (unsigned long long)EMPTY,
                                            (unsigned long long)tag);
            const bool won = prev == EMPTY;
            // every CAS attempt stores (a loser into the sink), so the winner's store cannot be sunk onto
            // the loop's exit path: it is issued before any lane of this wave reads a slot again
            __hip_atomic_store(won ? (unsigned long long*)&tab[h].key : &g_claim_sink[(h * 16) & 4095],
                               (unsigned long long)key,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (won) return 1;
            tg = prev;
        }
        if (k == EMPTY)
            k = __hip_atomic_load((unsigned long long*)&tab[h].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == EMPTY) {   // tag claimed, the key store still in flight: read the slot again (no advance)
            if (++wait > (1 << 24)) {
                atomicOr(err, 1u);
                return -1;
            }
            continue;
        }
        if (k == key) {
            cur = tg;
            return 0;
        }
#else
        if (k == EMPTY) {
            const uint64_t prev = atomicCAS((unsigned long long*)&tab[h].key, (unsigned long long)EMPTY,
                                            (unsigned long long)key);
            if (prev == EMPTY) {
                const uint64_t old = atomicMin((unsigned long long*)&tab[h].tag, (unsigned long long)tag);
                if (old == EMPTY) return 1;
                cur = old;   // a same-turn duplicate set its tag between our CAS and atomicMin
                return 0;
            }
            if (prev == key) {
                cur = tab[h].tag;
                return 0;
            }
            k = prev;
        }
        if (k == key) {
            cur = tg;
            return 0;
        }
#endif
        h = (h + 1) & mask;
        if (++probe > MAX_PROBE) {
            atomicOr(err, 1u);
            return -1;
        }
    }
}

// Claim with displacement marking (single-GPU speedrun path).  The winner of a key within a turn is
// the smallest tag (parent rank, ordinal) — the reference's first occurrence in next_queue order.  A
// claimant that lowers a same-turn tag marks the displaced holder in `lost`; one whose atomicMin finds
// a smaller tag has lost itself.  Every duplicate is therefore resolved by exactly one of the two, and
// once the grid drains the survivors are cand & ~lost — no second pass over the table.
// Sharded tags (sb_dist.inc): (turn+1) << 40 | source rank << SH_Q_SHIFT | local order, the local order of
// a child claimed by its own rank being (local parent rank << 8 | dsc) and of a record received from rank q
// its index among q's records to this owner.  Ordered like the global (parent rank, ordinal) order.
constexpr int SH_Q_SHIFT = 34;
constexpr uint64_t SH_LOCAL_MASK = (1ull << SH_Q_SHIFT) - 1;
constexpr uint64_t SH_RANK_MASK = (1ull << (SH_Q_SHIFT - 8)) - 1;   // local parent ranks < 2^26

// the top 24 bits of the key's mix scaled to [0, world) (multiply-shift, not a 64-bit modulo: a division routine
// per child in the key pass)
__host__ __device__ __forceinline__ uint32_t owner_of(uint64_t key, uint32_t world) {
    return (uint32_t)(((mix64(key) >> 40) * (uint64_t)world) >> 24);
}

template <bool PRE, bool SH = false>
__device__ __forceinline__ bool claim_lm(Entry* __restrict__ tab, uint64_t mask, uint64_t key, ulonglong2 ent,
                                         uint64_t tag, unsigned long long* __restrict__ lost, uint32_t* err) {
    uint64_t h, cur = EMPTY;
    const int r = probe_insert<PRE>(tab, mask, key, ent, tag, h, cur, err);
#ifdef SB_CLAIM_STATS
    // err[1] old-turn keys, err[2] inserted, err[3] same-turn early-out, err[4] lost at atomicMin, err[5] displaced
    if (r == 1) atomicAdd(err + 2, 1u);
    else if (r == 0 && cur < (tag & ~((1ull << 40) - 1))) atomicAdd(err + 1, 1u);
    else if (r == 0 && cur < tag) atomicAdd(err + 3, 1u);
    // err[6]: the key is already held by a same-turn child of the same 32-parent k_expand group
    // (the share an in-LDS pre-dedup of a group's children would take off the visited set)
    if (r == 0 && cur != EMPTY && cur >= (tag & ~((1ull << 40) - 1)) &&
        (((cur >> 8) & 0xFFFFFFFFull) >> 5) == (((tag >> 8) & 0xFFFFFFFFull) >> 5))
        atomicAdd(err + 6, 1u);
#endif
    if (r != 0) return r == 1;
    if (cur < tag) return false;
    const uint64_t old = atomicMin((unsigned long long*)&tab[h].tag, (unsigned long long)tag);
#ifdef SB_CLAIM_STATS
    if (old < tag) atomicAdd(err + 4, 1u);
    else atomicAdd(err + 5, 1u);
#endif
    if (old < tag) return false;
    if (old != EMPTY) {   // old > tag >= this turn's prefix: a same-turn holder, now displaced
        const uint64_t ro = (old >> 8) & (SH ? SH_RANK_MASK : 0xFFFFFFFFull);
        const uint32_t oo = (uint32_t)(old & 255);
        atomicOr(&lost[ro * 3 + (oo >> 6)], 1ull << (oo & 63));
    }
    return true;
}

__device__ __forceinline__ bool visit_claim_lm(Entry* __restrict__ tab, uint64_t mask, uint64_t key, uint64_t tag,
                                               unsigned long long* __restrict__ lost, uint32_t* err) {
    return claim_lm<false>(tab, mask, key, make_ulonglong2(0, 0), tag, lost, err);
}

// visit_claim_lm with the entry at the key's home slot already loaded (ent)
template <bool SH = false>
__device__ __forceinline__ bool visit_claim_lm_pre(Entry* __restrict__ tab, uint64_t mask, uint64_t key, ulonglong2 ent,
                                                   uint64_t tag, unsigned long long* __restrict__ lost, uint32_t* err) {
    return claim_lm<true, SH>(tab, mask, key, ent, tag, lost, err);
}

__device__ __forceinline__ uint64_t lookup_tag(const Entry* __restrict__ tab, uint64_t mask, uint64_t key) {
    uint64_t h = mix64(key) & mask;
    for (int probe = 0; probe <= MAX_PROBE; probe++) {
        uint64_t k = tab[h].key;
        if (k == key) return tab[h].tag;
        if (k == EMPTY) return EMPTY;
        h = (h + 1) & mask;
    }
    return EMPTY;
}

__global__ void k_insert_root(Entry* tab, uint64_t mask, uint64_t key) {
    uint64_t h = mix64(key) & mask;
    while (tab[h].key != EMPTY) h = (h + 1) & mask;
    tab[h].key = key;
    tab[h].tag = 0;   // turn prefix 0: in trail before the first step
}

// ------------------------------------------------------------------ visited-set growth
// The reference's `trail` is an unbounded dict (src/solver.py:425-426,447-450).  Between turns (no claim
// in flight) a table whose next turn could push it past GROW_LOAD is rebuilt at 2^k times the slots:
// every entry is re-inserted with its key AND tag, so the first-occurrence claims of later turns see
// exactly the set they would have seen (results do not depend on the capacity; tests/test_gpu_growth.py).
// Coalesced 16-B reads of the old table, one tag CAS + key store per entry into the new one.
__global__ __launch_bounds__(256) void k_rehash(const Entry* __restrict__ old, uint64_t n_old, Entry* __restrict__ neu,
                                                uint64_t mask, uint32_t* __restrict__ err) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_old; i += (uint64_t)gridDim.x * blockDim.x) {
        const ulonglong2 e = *reinterpret_cast<const ulonglong2*>(&old[i]);
        if (e.y == EMPTY) continue;
        uint64_t h = mix64(e.x) & mask;
        for (int probe = 0;; probe++) {
            if (atomicCAS((unsigned long long*)&neu[h].tag, (unsigned long long)EMPTY, (unsigned long long)e.y) == EMPTY) {
                neu[h].key = e.x;   // visible to the next turn's kernels (kernel boundary)
                break;
            }
            h = (h + 1) & mask;
            if (probe >= MAX_PROBE) {
                atomicOr(err, 1u);
                break;
            }
        }
    }
}

// ------------------------------------------------------------------ k_expand
// tuning knobs (overridable with -D for experiments; see profiles/variants.sh)
#ifndef SB_XP_PAR
#define SB_XP_PAR 32
#endif
#ifndef SB_XP_WAVES
#define SB_XP_WAVES 8   // min waves per SIMD: caps VGPRs at 64 (a 24 B/lane spill) for 8 waves; with
#endif                  // 16-bit queues (17 KB LDS) the block fits 9 per CU: more probes in flight
#ifndef SB_XP_NT
#define SB_XP_NT 256
#endif
#ifndef SB_XP_U
#define SB_XP_U 1          // children per thread per phase-B round (probe loads in flight together)
#endif
constexpr int XP_U = SB_XP_U;

#ifndef SB_XP_GRID_CAP
#define SB_XP_GRID_CAP 2560   // ~2 blocks per resident slot (5 per CU); groups come from a counter
#endif
constexpr int XP_NT = SB_XP_NT;       // 4 waves
constexpr int XP_PAR = SB_XP_PAR;     // parents per block iteration (<= 32)
#ifndef SB_XP_DQ
#define SB_XP_DQ 4   // A/B profiles/r2_ab_expand_dq.txt: 1 / 2 / 4 -> k_expand 3.35 / 3.30 / 3.24 ms (3 rounds)
#endif
constexpr uint32_t XP_DQ = SB_XP_DQ;  // parent groups per work-counter add
static_assert(XP_PAR <= 32 && (31 | ((NCARDS + 127) << 5)) <= 0xFFFF, "k_expand queue entries: 5-bit s, 16-bit entry");

struct XpShared {
    uint32_t card[NCARDS];
    int32_t pdelta[4][NPAT_MAX];
    uint64_t mlo[NCOL];
    uint32_t mhi[NCOL];
    uint64_t alo[NCOL][8];
    uint32_t ahi[NCOL][8];
    uint64_t plo[XP_PAR], phi[XP_PAR], phc[XP_PAR];
    uint64_t ptm[XP_PAR][2];
    uint64_t pbl[XP_PAR];
    uint32_t pbh[XP_PAR];
    uint32_t pbon[XP_PAR];
    int32_t pbk[XP_PAR];
    unsigned long long cmask[XP_PAR][3];
    // 16-bit entries (s < 32, dsc < 192: 13 bits): the queues are most of the block's LDS, and LDS is
    // what bounds k_expand's occupancy (29.5 KB/block with 32-bit entries: 5 blocks per CU)
    uint16_t qb[XP_PAR * NCARDS];     // buy children (s | dsc << 5)
    uint16_t qt[XP_PAR * NPAT_MAX];   // take children: phase B runs all buys, then all takes, so a
    uint32_t nqb, nqt, nraw;          // wave rarely mixes the two (a buy re-hashes its card tuple)
    uint32_t proff[XP_PAR];           // SH: first record of each parent
    uint32_t grp[3];                  // this, next and next-but-one parent group
    uint32_t dq_next, dq_left;        // groups left from the last dequeue (XP_DQ per counter add)
};

// enumeration tables into LDS: cards, colour masks, affordability masks, pattern deltas
__device__ __forceinline__ void load_enum_lds(const Tables* __restrict__ T, uint32_t* card, uint64_t* mlo, uint32_t* mhi,
                                              uint64_t (*alo)[8], uint32_t (*ahi)[8], int32_t (*pdelta)[NPAT_MAX]) {
    for (int i = threadIdx.x; i < NCARDS; i += blockDim.x) card[i] = T->card[i];
    for (int i = threadIdx.x; i < 4 * NPAT_MAX; i += blockDim.x) (&pdelta[0][0])[i] = (&T->pdelta[0][0])[i];
    for (int i = threadIdx.x; i < NCOL * 8; i += blockDim.x) {
        (&alo[0][0])[i] = (&T->aff_lo[0][0])[i];
        (&ahi[0][0])[i] = (&T->aff_hi[0][0])[i];
    }
    if (threadIdx.x < NCOL) {
        mlo[threadIdx.x] = T->colmask_lo[threadIdx.x];
        mhi[threadIdx.x] = T->colmask_hi[threadIdx.x];
    }
}

__device__ __forceinline__ void load_tables_lds(const Tables* __restrict__ T, uint32_t* card, uint32_t (*pat)[NPAT_MAX],
                                                int32_t* npat, uint64_t* mlo, uint32_t* mhi) {
    for (int i = threadIdx.x; i < NCARDS; i += blockDim.x) card[i] = T->card[i];
    for (int i = threadIdx.x; i < 4 * NPAT_MAX; i += blockDim.x) (&pat[0][0])[i] = (&T->pat[0][0])[i];
    if (threadIdx.x < 4) npat[threadIdx.x] = T->npat[threadIdx.x];
    if (threadIdx.x < NCOL) {
        mlo[threadIdx.x] = T->colmask_lo[threadIdx.x];
        mhi[threadIdx.x] = T->colmask_hi[threadIdx.x];
    }
}

__device__ __forceinline__ void derive_lds(const uint64_t* mlo, const uint32_t* mhi, uint64_t lo, uint64_t hi, Derived& d) {
    uint32_t chi = st_chi(hi);
#pragma unroll
    for (int i = 0; i < NCOL; i++) {
        d.g[i] = st_gem(hi, i);
        d.b[i] = __popcll(lo & mlo[i]) + __popc(chi & mhi[i]);
    }
    d.pts = st_pts(hi);
    d.saved = st_saved(hi);
}

// Parents [0, n): every raw child is probed/claimed in the visited set; candidate bitmask (3 x u64)
// per parent.  Successor order (src/solver.py:357-388) comes from masks: the buy set in deck order
// (AND of per-colour affordability masks minus owned cards), then the valid take patterns of the
// gem field in bucket order (Tables::tmask).  A child is named by its move descriptor dsc (card
// 0..89, NCARDS + take-pattern bit): dsc order IS the canonical order, so the claim tag
// (turn, parent rank, dsc) orders exactly like (turn, parent rank, ordinal), and the candidate /
// lost bits of a parent are indexed by dsc (the 192-bit move space of move_space()).
// Displaced same-turn claims are marked in `lost` (lost marking).
// SH (sharded step, sb_dist.inc): the children this rank owns (owner_of(key) == me) are claimed here in
// its owner shard `tab` with tag (me, local rank, dsc); every other child becomes a record for its owner:
// key and owner digit at roff[parent] + ordinal (digit 0xFF = claimed here), the layout the owner
// partition reads.  cand / lost then hold the own children's claims only.
template <bool SH>
__global__ __launch_bounds__(XP_NT, SB_XP_WAVES) void k_expand(const Tables* __restrict__ T, const uint64_t* __restrict__ blo,
                                                  const uint64_t* __restrict__ bhi, int64_t n, Entry* __restrict__ tab,
                                                  uint64_t mask, uint64_t turn_tag, unsigned long long* __restrict__ cand,
                                                  unsigned long long* __restrict__ lost,
                                                  unsigned long long* __restrict__ nraw_total, uint32_t* __restrict__ err,
                                                  uint32_t* __restrict__ work, uint32_t me, uint32_t world,
                                                  const uint32_t* __restrict__ roff, uint64_t* __restrict__ rkey,
                                                  uint8_t* __restrict__ rdig, uint64_t rcap, uint8_t* __restrict__ rdsc) {
    __shared__ XpShared S;
    load_enum_lds(T, S.card, S.mlo, S.mhi, S.alo, S.ahi, S.pdelta);
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const uint64_t lt = lanemask_lt();
    if (t == 0) S.nraw = 0;
    // parent words of a group, one per thread (t < 16: lo, t < 32: hi), loaded a group ahead
    auto fetch = [&](int64_t b) -> uint64_t {
        const int64_t r = b + (t & (XP_PAR - 1));
        if (t >= 2 * XP_PAR || r >= n) return 0ull;
        return t < XP_PAR ? blo[r] : bhi[r];
    };
    // groups are handed out in rank order by a counter (not a grid stride), so claims run roughly in
    // tag order and fewer same-turn holders get displaced; each block fetches a group ahead
    // XP_DQ consecutive groups per counter add: one counter word serialises its atomics (MI355X: ~88 per
    // us), so fewer adds keep the dequeue off the expansion's critical path
    auto next_group = [&]() -> uint32_t {
        if (S.dq_left == 0) {
            S.dq_next = atomicAdd(work, 1u) * XP_DQ;
            S.dq_left = XP_DQ;
        }
        S.dq_left--;
        return S.dq_next++;
    };
    if (t == 0) {
        S.dq_left = 0;
        S.grp[0] = next_group();
        S.grp[1] = next_group();
    }
    __syncthreads();
    int64_t base = (int64_t)S.grp[0] * XP_PAR, nxt = (int64_t)S.grp[1] * XP_PAR;
    uint64_t pf = base < n ? fetch(base) : 0ull;
    while (base < n) {
        if (t == 0) {
            S.nqb = S.nqt = 0;
            S.grp[2] = next_group();   // the group after next; read after the barrier below
        }
        if (t < XP_PAR * 3) (&S.cmask[0][0])[t] = 0;
        if (t < XP_PAR) S.plo[t] = pf;
        else if (t < 2 * XP_PAR) S.phi[t - XP_PAR] = pf;
        __syncthreads();
        const int64_t nxt2 = (int64_t)S.grp[2] * XP_PAR;
        if (nxt < n) pf = fetch(nxt);
        // prologue, a lane per parent: buy set, bucket, take mask, packed bonus, hash of the card tuple
        if (t < XP_PAR) {
            const uint64_t lo = S.plo[t], hi = S.phi[t];
            Derived d;
            derive_lds(S.mlo, S.mhi, lo, hi, d);
            uint64_t bl;
            uint32_t bh;
            buy_set(S.alo, S.ahi, d, lo, hi, &bl, &bh);
            const int bk = take_bucket(d);
            uint64_t t0 = 0, t1 = 0;
            if (bk >= 0) {
                const uint32_t gf = st_gemfield(hi);
                t0 = T->tmask[gf][0];
                t1 = T->tmask[gf][1];
            }
            S.pbl[t] = bl;
            S.pbh[t] = bh;
            S.ptm[t][0] = t0;
            S.ptm[t][1] = t1;
            S.pbon[t] = pack_bonus(d);
            S.pbk[t] = bk;
            if (SH) S.proff[t] = base + t < n ? roff[base + t] : 0u;
        } else if (t < 2 * XP_PAR) {
            const int s = t - XP_PAR;
            S.phc[s] = hash_cards(S.plo[s], st_chi(S.phi[s]));
        }
        __syncthreads();
        // ---- phase A: a wave per parent lays its children out in canonical order
        for (int s = w; s < XP_PAR; s += XP_NT / 64) {
            const int64_t r = base + s;
            if (r >= n) break;
            const uint64_t bl = S.pbl[s], t0 = S.ptm[s][0], t1 = S.ptm[s][1];
            const uint32_t bh = S.pbh[s];
            const int nbl = __popcll(bl), nb = nbl + __popc(bh), nt0 = __popcll(t0);
            const int nt = nt0 + __popcll(t1);
            uint32_t qb = 0, qt = 0;
            if (lane == 0) {
                qb = atomicAdd(&S.nqb, (uint32_t)nb);
                qt = atomicAdd(&S.nqt, (uint32_t)nt);
                atomicAdd(&S.nraw, (uint32_t)(nb + nt));
            }
            qb = __shfl(qb, 0, 64);
            qt = __shfl(qt, 0, 64);
            if ((bl >> lane) & 1) S.qb[qb + __popcll(bl & lt)] = (uint16_t)(s | (lane << 5));
            if (lane < 26 && ((bh >> lane) & 1))
                S.qb[qb + nbl + __popc(bh & (uint32_t)lt)] = (uint16_t)(s | ((64 + lane) << 5));
            if ((t0 >> lane) & 1) S.qt[qt + __popcll(t0 & lt)] = (uint16_t)(s | ((NCARDS + lane) << 5));
            if ((t1 >> lane) & 1) S.qt[qt + nt0 + __popcll(t1 & lt)] = (uint16_t)(s | ((NCARDS + 64 + lane) << 5));
        }
        __syncthreads();
        // ---- phase B: dense child processing: key, visited probe + claim; XP_U children per thread
        // with their first probe loads issued together (more misses in flight per wave).
        const uint32_t nqb = S.nqb, nq = nqb + S.nqt;
        auto child_key = [&](uint32_t e) -> uint64_t {
            const int s = (int)(e & 31), dsc = (int)(e >> 5);
            const uint64_t lo = S.plo[s], hi = S.phi[s];
            if (dsc < NCARDS) {
                Derived d;
                derive_packed(hi, S.pbon[s], d);
                uint64_t clo = lo;
                const uint64_t chi = buy_child_hi(S.card[dsc], dsc, d, hi, &clo);
                return state_key(hash_cards(clo, st_chi(chi)), hash_gems(st_gemfield(chi)));
            }
            const uint32_t gf = (uint32_t)((int32_t)st_gemfield(hi) + S.pdelta[S.pbk[s]][dsc - NCARDS]);
            return state_key(S.phc[s], hash_gems(gf));
        };
        for (uint32_t i0 = t; i0 < nq; i0 += XP_NT * XP_U) {
            uint32_t e[XP_U];
            uint64_t key[XP_U];
            ulonglong2 ent[XP_U];
#pragma unroll
            for (int u = 0; u < XP_U; u++) {
                const uint32_t i = i0 + u * XP_NT;
                e[u] = i < nqb ? (uint32_t)S.qb[i] : (i < nq ? (uint32_t)S.qt[i - nqb] : 0xFFFFFFFFu);
                key[u] = e[u] != 0xFFFFFFFFu ? child_key(e[u]) : 0;
            }
            if (!SH) {   // the home slot's entry, loaded for all children together (SH: own children only, below)
#pragma unroll
                for (int u = 0; u < XP_U; u++)
                    if (e[u] != 0xFFFFFFFFu) ent[u] = load_entry(&tab[mix64(key[u]) & mask]);
            }
#pragma unroll
            for (int u = 0; u < XP_U; u++) {
                if (e[u] == 0xFFFFFFFFu) continue;
                const int s = (int)(e[u] & 31), dsc = (int)(e[u] >> 5);
                if (SH && world > 1) {
                    // record slot: the parent's first record + the child's ordinal (set bits below dsc in
                    // its move space: buys 0..89, then the take patterns)
                    uint64_t ms[3];
                    move_space(S.pbl[s], S.pbh[s], S.ptm[s][0], S.ptm[s][1], ms);
                    const int w0 = dsc >> 6;
                    const uint64_t below = (1ull << (dsc & 63)) - 1;
                    const uint32_t ord = (uint32_t)((w0 > 0 ? __popcll(ms[0]) : 0) + (w0 > 1 ? __popcll(ms[1]) : 0) +
                                                    __popcll(ms[w0] & below));
                    const uint32_t ri = S.proff[s] + ord;
                    if (ri >= rcap) {   // compact record buffers (flags bit 5) overflowed: sbd_expand_counts fails
                        atomicOr(err, 64u);
                        continue;
                    }
                    const uint32_t ow = owner_of(key[u], world);
                    rdig[ri] = ow == me ? (uint8_t)0xFF : (uint8_t)ow;
                    if (ow != me) {
                        rkey[ri] = key[u];
                        rdsc[ri] = (uint8_t)dsc;   // the apply maps this record's answer to its move directly
                        continue;
                    }
                }
                const uint64_t tag = SH ? turn_tag | ((uint64_t)me << SH_Q_SHIFT) | ((uint64_t)(base + s) << 8) | (uint64_t)dsc
                                        : turn_tag | ((uint64_t)(base + s) << 8) | (uint64_t)dsc;
                if (SH) ent[u] = load_entry(&tab[mix64(key[u]) & mask]);
                if (visit_claim_lm_pre<SH>(tab, mask, key[u], ent[u], tag, lost, err))
                    atomicOr(&S.cmask[s][dsc >> 6], 1ull << (dsc & 63));
            }
        }
        __syncthreads();
        if (t < XP_PAR * 3) {
            const int s = t / 3, j = t % 3;
            if (base + s < n) cand[(base + s) * 3 + j] = S.cmask[s][j];
        }
        __syncthreads();
        base = nxt;
        nxt = nxt2;
    }
    if (t == 0 && S.nraw) atomicAdd(nraw_total, (unsigned long long)S.nraw);
}

// ------------------------------------------------------------------ survivors of the lost-marking path
// survivors per parent = popcount(cand & ~lost) over the move space, with the scan's first kernel folded in:
// a block counts one SCAN_TILE tile of parents (strided, coalesced) and stores the tile's sum for
// scan_exclusive_u32_sums (k_scan_reduce would read cnt again).  (1024 threads with every mask load issued
// first measured slower: 52-60 against 43-47 us)
constexpr int CLT_NT = 256;
__global__ __launch_bounds__(CLT_NT) void k_count_lm_tiles(int64_t n, const unsigned long long* __restrict__ cand,
                                                           const unsigned long long* __restrict__ lost,
                                                           uint32_t* __restrict__ cnt, uint32_t* __restrict__ tile_sums) {
    __shared__ uint32_t lds[CLT_NT / 64 + 1];
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + threadIdx.x;
    uint32_t s = 0;
#pragma unroll 4
    for (int j = 0; j < SCAN_TILE / CLT_NT; j++) {
        const int64_t r = base + (int64_t)j * CLT_NT;
        if (r < n) {
            const uint32_t c = __popcll(cand[r * 3] & ~lost[r * 3]) + __popcll(cand[r * 3 + 1] & ~lost[r * 3 + 1]) +
                               __popcll(cand[r * 3 + 2] & ~lost[r * 3 + 2]);
            cnt[r] = c;
            s += c;
        }
    }
    uint32_t tot;
    block_excl_scan<CLT_NT>(s, lds, &tot);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
}

#include "sb_wave.inc"

// ------------------------------------------------------------------ beam write + per-pts first rank
__global__ __launch_bounds__(256) void k_gather(const uint32_t* __restrict__ idx, int64_t m,
                                                const uint64_t* __restrict__ nlo, const uint64_t* __restrict__ nhi,
                                                const uint32_t* __restrict__ npar, uint64_t* __restrict__ olo,
                                                uint64_t* __restrict__ ohi, uint32_t* __restrict__ opar,
                                                uint32_t* __restrict__ first) {
    __shared__ uint32_t f[256];
    f[threadIdx.x] = 0xFFFFFFFFu;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t j = idx ? idx[i] : (uint32_t)i;
        const uint64_t h = nhi[j];
        olo[i] = nlo[j];
        ohi[i] = h;
        opar[i] = npar[j];
        atomicMin(&f[st_pts(h)], (uint32_t)i);
    }
    __syncthreads();
    if (f[threadIdx.x] != 0xFFFFFFFFu) atomicMin(&first[threadIdx.x], f[threadIdx.x]);
}

// kept beam rebuilt from descriptors (parent rank << 8 | dsc) + the per-pts first-rank table
__global__ __launch_bounds__(256) void k_gather_d(const Tables* __restrict__ T, const uint32_t* __restrict__ idx, int64_t m,
                                                  const uint64_t* __restrict__ ndesc, const uint64_t* __restrict__ plo,
                                                  const uint64_t* __restrict__ phi, uint64_t* __restrict__ olo,
                                                  uint64_t* __restrict__ ohi, uint32_t* __restrict__ opar,
                                                  uint32_t* __restrict__ first, int desc_in_idx,
                                                  unsigned long long* __restrict__ zlost) {
    __shared__ uint32_t f[256];
    __shared__ uint32_t card[NCARDS];
    __shared__ int32_t pdelta[4][NPAT_MAX];
    __shared__ uint64_t mlo[NCOL];
    __shared__ uint32_t mhi[NCOL];
    f[threadIdx.x] = 0xFFFFFFFFu;
    for (int i = threadIdx.x; i < NCARDS; i += blockDim.x) card[i] = T->card[i];
    for (int i = threadIdx.x; i < 4 * NPAT_MAX; i += blockDim.x) (&pdelta[0][0])[i] = (&T->pdelta[0][0])[i];
    if (threadIdx.x < NCOL) {
        mlo[threadIdx.x] = T->colmask_lo[threadIdx.x];
        mhi[threadIdx.x] = T->colmask_hi[threadIdx.x];
    }
    __syncthreads();
    const int64_t gstride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gstride) {
        const uint64_t dd = desc_in_idx ? (uint64_t)idx[i] : ndesc[idx[i]];   // the top-k carried the descriptor itself
        const uint32_t r = (uint32_t)(dd >> 8);
        const int dsc = (int)(dd & 255);
        const uint64_t lo = plo[r], hi = phi[r];
        Derived d;
        derive_lds(mlo, mhi, lo, hi, d);
        uint64_t clo = lo, chi;
        if (dsc < NCARDS) chi = buy_child_hi(card[dsc], dsc, d, hi, &clo);
        else chi = st_with_gems(hi, (uint32_t)((int32_t)st_gemfield(hi) + pdelta[take_bucket(d)][dsc - NCARDS]));
        olo[i] = clo;
        ohi[i] = chi;
        opar[i] = r;
        atomicMin(&f[st_pts(chi)], (uint32_t)i);
        if (zlost) {   // the next turn's lost marks of parent i start at zero (no 24 B/parent memset before it)
            zlost[i * 3] = 0ull;
            zlost[i * 3 + 1] = 0ull;
            zlost[i * 3 + 2] = 0ull;
        }
    }
    __syncthreads();
    if (f[threadIdx.x] != 0xFFFFFFFFu) atomicMin(&first[threadIdx.x], f[threadIdx.x]);
}

__global__ void k_front_reset(unsigned long long* __restrict__ nraw, uint32_t* __restrict__ small) {
    const int t = threadIdx.x;
    if (t == 0) {
        *nraw = 0ull;
        small[264] = 0u;
    }
    if (t < 6) small[2 + t] = 0u;
}

__global__ void k_pts_first(const uint64_t* __restrict__ bhi, int64_t m, uint32_t* __restrict__ first) {
    __shared__ uint32_t f[256];
    f[threadIdx.x] = 0xFFFFFFFFu;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        atomicMin(&f[st_pts(bhi[i])], (uint32_t)i);
    __syncthreads();
    if (f[threadIdx.x] != 0xFFFFFFFFu) atomicMin(&first[threadIdx.x], f[threadIdx.x]);
}

__global__ void k_keys(const uint64_t* __restrict__ lo, const uint64_t* __restrict__ hi, int64_t n, uint64_t* __restrict__ key) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        key[i] = key_of(lo[i], hi[i]);
}

// ------------------------------------------------------------------ debug kernels (parity tests)
__global__ void k_debug_succ(const Tables* __restrict__ T, const uint64_t* __restrict__ lo, const uint64_t* __restrict__ hi,
                             int64_t n, uint64_t* olo, uint64_t* ohi, uint64_t* okey, int32_t* ocnt) {
    __shared__ uint32_t card[NCARDS];
    __shared__ uint32_t pat[4][NPAT_MAX];
    __shared__ int32_t npat[4];
    __shared__ uint64_t mlo[NCOL];
    __shared__ uint32_t mhi[NCOL];
    load_tables_lds(T, card, pat, npat, mlo, mhi);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint64_t lt = lanemask_lt();
    const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (r >= n) return;
    const uint64_t plo = lo[r], phi = hi[r];
    Derived d;
    derive_lds(mlo, mhi, plo, phi, d);
    const uint64_t hc = hash_cards(plo, st_chi(phi));
    int ord = 0;
    for (int pass = 0; pass < 2; pass++) {
        const int c = pass * 64 + lane;
        const bool v = c < NCARDS && !st_owns(plo, phi, c) && affordable(card[c < NCARDS ? c : 0], d);
        const uint64_t m = __ballot(v);
        if (v) {
            const int o = ord + __popcll(m & lt);
            uint64_t clo = plo;
            const uint64_t chi = buy_child_hi(card[c], c, d, phi, &clo);
            olo[r * MAX_CHILDREN + o] = clo;
            ohi[r * MAX_CHILDREN + o] = chi;
            okey[r * MAX_CHILDREN + o] = state_key(hash_cards(clo, st_chi(chi)), hash_gems(st_gemfield(chi)));
        }
        ord += __popcll(m);
    }
    const int bk = take_bucket(d);
    if (bk >= 0) {
        const int np = npat[bk];
        for (int p0 = 0; p0 < np; p0 += 64) {
            const int p = p0 + lane;
            uint32_t gf;
            const bool v = p < np && take_child(pat[bk][p < np ? p : 0], d, &gf);
            const uint64_t m = __ballot(v);
            if (v) {
                const int o = ord + __popcll(m & lt);
                olo[r * MAX_CHILDREN + o] = plo;
                ohi[r * MAX_CHILDREN + o] = st_with_gems(phi, gf);
                okey[r * MAX_CHILDREN + o] = state_key(hc, hash_gems(gf));
            }
            ord += __popcll(m);
        }
    }
    if (lane == 0) ocnt[r] = ord;
}

template <int H>
__global__ void k_debug_scores(const Tables* __restrict__ T, const uint64_t* lo, const uint64_t* hi, const int32_t* k,
                               int64_t n, double* out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = score_of<H>(T->pw, *T, lo[i], hi[i], T->noise[k[i] - 1]);
}

// ------------------------------------------------------------------ tables
static int npat_host(int b) { return g_host_tables.npat[b]; }

static void build_patterns(Tables& T) {
    // distinct_permutations (sorted input, lexicographic order) of the src/gems.py:22-37 patterns
    auto add = [&](int bucket, std::vector<int> p, bool two) {
        std::sort(p.begin(), p.end());
        do {
            uint32_t w = 0;
            int two_at = 7;
            for (int i = 0; i < NCOL; i++) {
                w |= (uint32_t)(p[i] + 2) << (3 * i);
                if (two && p[i] == 2 && two_at == 7) two_at = i;
            }
            w |= (uint32_t)two_at << 15;
            T.pat[bucket][T.npat[bucket]++] = w;
        } while (std::next_permutation(p.begin(), p.end()));
    };
    for (int b = 0; b < 4; b++) T.npat[b] = 0;
    add(0, {1, 1, 1, 0, 0}, false);
    add(0, {2, 0, 0, 0, 0}, true);
    add(1, {1, 1, 1, -1, 0}, false);
    add(1, {1, 1, 0, 0, 0}, false);
    add(1, {2, 0, 0, 0, 0}, true);
    add(2, {1, 1, 1, -1, -1}, false);
    add(2, {1, 1, -1, 0, 0}, false);
    add(2, {1, 0, 0, 0, 0}, false);
    add(2, {2, -1, 0, 0, 0}, true);
    add(3, {1, 1, -1, -1, 0}, false);
    add(3, {1, -1, 0, 0, 0}, false);
    add(3, {2, -1, -1, 0, 0}, true);
    add(3, {2, -2, 0, 0, 0}, true);
}

// masks and packed deltas for mask enumeration (see Tables); restates affordable() / take_child()
static void build_enum_tables(Tables& T) {
    for (int i = 0; i < NCOL; i++)
        for (int v = 0; v < 8; v++) {
            T.aff_lo[i][v] = 0;
            T.aff_hi[i][v] = 0;
            for (int c = 0; c < NCARDS; c++)
                if ((int)((T.card[c] >> (3 * i)) & 7) <= v) {
                    if (c < 64) T.aff_lo[i][v] |= 1ull << c;
                    else T.aff_hi[i][v] |= 1u << (c - 64);
                }
        }
    for (int b = 0; b < 4; b++)
        for (int p = 0; p < NPAT_MAX; p++) {
            int32_t dl = 0;
            if (p < T.npat[b])
                for (int i = NCOL - 1; i >= 0; i--) dl = dl * 8 + ((int)((T.pat[b][p] >> (3 * i)) & 7) - 2);
            T.pdelta[b][p] = dl;
        }
    for (int gf = 0; gf < (1 << 15); gf++) {
        int g[NCOL], tot = 0;
        for (int i = 0; i < NCOL; i++) tot += g[i] = (gf >> (3 * i)) & 7;
        T.tmask[gf][0] = T.tmask[gf][1] = 0;
        const int bk = tot > 10 ? -1 : (tot <= 7 ? 0 : tot - 7);
        if (bk < 0) continue;
        for (int p = 0; p < T.npat[bk]; p++) {
            const uint32_t w = T.pat[bk][p];
            const int two = (int)((w >> 15) & 7);
            bool ok = true;
            for (int i = 0; i < NCOL; i++) {
                const int x = g[i] + (int)((w >> (3 * i)) & 7) - 2;
                ok &= x >= 0 && x <= MAXG;
                if (two == i) ok &= g[i] <= MAXG - 4;
            }
            if (ok) T.tmask[gf][p >> 6] |= 1ull << (p & 63);
        }
    }
}

// ------------------------------------------------------------------ engine
// realistic-mode game constants (sb_realistic.inc)
struct RGame {
    int P, target;
    int tlen[3];
    uint8_t tier[3][40];
    int inf;   // infinite_resources=True: speedrun takes, pool in w[11] (sb_realistic.inc)
};

struct Turn {
    uint64_t* lo = nullptr;
    uint64_t* hi = nullptr;
    uint32_t* par = nullptr;
    int64_t n = 0;
};

static unsigned grid_cap(int64_t work, int per_block, unsigned cap) {
    int64_t g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    return (unsigned)std::min<int64_t>(g, cap);
}

// owner emission (sb_oe.inc): row group starts (card-set owners) / received source segments, start[ng] = n
struct OeGroups {
    uint32_t start[65];
    int ng;
};

struct Engine {
    sb_config cfg{};
    int dev = 0;
    hipStream_t s = nullptr, s_mt = nullptr;
    bool s_external = false;                // sbd_set_stream: the caller's stream (not destroyed here)
    Tables* d_tables = nullptr;
    Entry* tab = nullptr;
    uint64_t tab_mask = 0;
    uint64_t visited = 1;
    std::vector<Turn> turns;
    DBuf<uint8_t> desc;
    DBuf<uint32_t> rslot;
    DBuf<unsigned long long> cand, surv, lost;
    DBuf<uint32_t> cnt, off;
    DBuf<uint64_t> nlo, nhi, skey;
    DBuf<uint32_t> npar, kidx;
    uint32_t* d_small = nullptr;            // [0] n_unique total  [1] err  [2..8) claim stats ; [8..8+256) first-rank table ; [264] k_expand group counter ; [266..268) u64 sharded owner key count
    unsigned long long* d_nraw = nullptr;
    uint32_t* h_small = nullptr;            // pinned mirror of d_small (272 words)
    unsigned long long* h_nraw = nullptr;
    ScanScratch scan;
    TopkScratch topk;
    NoiseStream noise;
    int turn = 0;
    bool done = false;
    int64_t winner_rank = -1;
    int max_pts = 0;
    uint64_t last_nu = 0;
    int front_turn = -1;                    // turn whose front half (expand .. readback) is in flight
    bool lookahead = true;                  // finish_turn launches the next front half (sb_set_lookahead)
    int64_t lost_zero = 0;                  // lost[0 .. 3 * lost_zero) is known zero (the emission cleared it)
    bool first_reset = false;               // this turn's first-rank table was reset with the top-k's range
    std::vector<hipEvent_t> tev;            // per-turn timing events (TEV_RING x 7)
    Arena turn_mem;
    hipEvent_t ev[8] = {};
    // distributed mode (world_size > 1): owner shard of the global visited set + exchange staging
    Entry* own = nullptr;
    uint64_t own_mask = 0;
    int64_t ncand = 0, nuniq_local = 0, nkept_local = 0;
    int64_t goff = 0;
    int part_D = 1;
    // realistic mode (mode 1): 12-word states in Turn::lo
    int mode = 0;
    RGame rgame_storage{};
    RGame* rgame = nullptr;
    uint32_t* d_rfirst = nullptr;
    uint32_t* h_rfirst = nullptr;
    DBuf<uint64_t> nw;
    DBuf<uint64_t> cand_key, cand_tag;
    DBuf<uint32_t> cand_ro, cand_pos, own_slot, part_hist;
    DBuf<unsigned long long> own_lost;
    int64_t own_n = 0;                    // sharded: records claimed at this owner this turn
    DBuf<uint64_t> dsel, dsel_c;          // joint select: prefixes / histograms, candidate keys
    DBuf<uint32_t> dsel_t;                // joint select: compaction tile offsets
    DBuf<uint32_t> dsel_ci;               // joint select: candidates' indices (the tie counts per tile)
    int dsel_npos = 1;                    // joint select: positions (histogram rows)
    DBuf<uint64_t> rkey;                  // sharded receive: keys of the received records
    DBuf<uint8_t> digit;
    DBuf<uint8_t> rdsc;                   // sharded: each record's move descriptor, at its raw position
    DBuf<uint16_t> mrj;                   // card-set records: (parent in chunk << 8) | move, at the record's slot
    DBuf<uint8_t> snv;                    // sharded emission: each survivor's noise draw (3-word kept records)
    DBuf<uint8_t> gdig;                   // grouped kept records: group starts by destination
    DBuf<uint32_t> gk_hist, gk_off, gk_cnt, gk_coff;   // ... group partition, buffer layout; receive: start flags, scan
    DBuf<uint64_t> gk_tab;                // ... receive (block-cyclic slices): the permutation and parent-map runs
    DBuf<uint64_t> rkey2;                 // owner emission: received records' re-scored keys, arrival order
    bool sdesc = false, sdesc32 = false;  // sharded emission wrote descriptors (4-byte when sdesc32) into nlo
    int64_t sdesc_goff = 0;               // ... global ranks: the slice's parents start at this one
    DBuf<uint32_t> mcrec;                 // card-set records per 64-parent chunk of the expand list
    // visited-set growth (grow_table): largest raw children per parent seen so far, tables rebuilt
    double raw_ratio = 32.0;
    int n_grow = 0;
    // growth that fell short (ranks sharing one GPU's HBM can leave less than the sizing saw): a
    // table rebuilt smaller than the turn's worst case wanted, a rebuild wanted and none made; the peak load (keys /
    // slots after a turn) — all reported by sb_visited_stats and the bench lines, never silent
    int n_grow_short = 0, n_grow_skip = 0;
    double peak_load = 0.0;
    uint64_t own_visited = 1;             // sharded: keys held by this owner shard (root counted at every rank)
    bool records = true;                  // sharded: this turn made records for other owners (world > 1)
    int64_t rec_per_parent = MAX_CHILDREN;   // sharded record slots per parent (flags bit 5: 48, overflow checked)
    size_t rcap_turn = 0;                 // sharded: record slots of the expansion in flight
    bool apply_pending = false;           // sharded: sbd_apply done, sbd_apply_finish not yet
    bool expand_pending = false;          // sharded: sbd_expand_launch done, sbd_expand_counts not yet
    bool goal_copied = false;             // sharded: the slice's goal table is on its way to h_small (event ev[0])
    bool raw_pending = false;             // sharded world 1: sbd_expand_defer done, sbd_raw_total not yet
    int expand_world = 1;
    uint64_t own_pending = 0;             // sharded: children this rank may have claimed in its expansion (bound)
    std::vector<int64_t> srcb;            // sharded: first answer index of each source's records this turn
    int64_t pending_host = -1;
    // sharded key pass (sb_keypass.inc, world > 1, sbd_expand_parts): the slice's children in ks_parts exchange
    // parts (64-parent chunks [ks_c[j], ks_c[j+1])), enqueued back to back on the engine stream; per raw child
    // its (owner, move, rank) word; per part its (owner, chunk) table + scan, per-owner counts (pinned mirror),
    // an event; received records' claims run on s_claim (sbd_set_claim_stream) beside the later parts
    bool ks_pipe = false;                 // this turn's expansion is the pipelined key pass
    bool goc = false;                     // global-order claims (cfg flags bit 11, sb_dist.inc k_claim_goc)
    bool kept20 = false;                  // this turn's kept records are 20 bytes (sbd_pack_kept rec20)
    DBuf<uint64_t> goc_seg;               // their segment table (v start, physical start)
    uint64_t* h_goc = nullptr;            // pinned staging of it
    hipEvent_t goc_ev = nullptr;          // ... recorded after its copy (the next turn's rewrite waits for that only)
    int ks_parts = 0;
    int64_t ks_c[17] = {};
    int64_t ks_pb[17] = {};               // each part's first local parent (ks_pb[ks_parts] = n): chunk c of part j holds
                                          // parents ks_pb[j] + 64 (c - ks_c[j]) .. (block-cyclic parts: any bounds)
    bool ks_bounds = false;               // this turn's parts came from the caller's bounds (block-cyclic slices)
    size_t ks_ccoff[17] = {};
    uint64_t ks_sbase[17] = {};           // each part's first index in the turn's send buffers (sbd_part_pack)
    hipEvent_t ks_ev[16] = {};
    bool goc_tk_clear = false;            // sbd_expand_parts cleared the parts' claim tickets for this turn
    uint32_t* h_pc = nullptr;             // pinned: per part, per owner record counts (16 x 64)
    uint64_t lostb_cap = 0;               // answers (received records) the lost bits / claims may index this turn
    hipStream_t s_claim = nullptr;
    DBuf<uint32_t> ks_rdr, ks_sown, ks_cc, ks_tot, ks_pc, ks_tk;   // ks_tk: the parts' chunk tickets
    DBuf<uint64_t> ks_send;               // global-order claims: the turn's packed records (sbd_send_buffer)
    // card-set ownership of the sharded dedup (sb_mig.inc, cfg flags bit 8): range side (parents' owner digits,
    // their rows' send positions, the partition histogram, per-owner counts), expand side (the received parents
    // as SoA + global ranks, raw counts / offsets), gmap (global rank -> expand index | first received record),
    // mtag (received records' tags by answer index)
    bool mig = false, mig_pending = false;
    int64_t mig_n = 0;
    DBuf<uint8_t> mdig;
    DBuf<uint32_t> mpos, mhist, xg, xcnt, xoff, gmap, mraw, mrawsend, mrawoff;
    DBuf<uint64_t> mrawown;
    DBuf<uint64_t> xlo, xhi, mtag;
    uint32_t* h_mpc = nullptr;
    hipEvent_t mig_ev = nullptr;
    // owner emission (sb_oe.inc, cfg flags bit 9 with bit 8): the expand list's survivor masks and offsets, the
    // emitted survivors' next_queue positions, the keep boundary's tie positions, the second receive order
    bool oe = false;
    int64_t oe_n = 0;                     // survivors emitted on this rank (the expand list's)
    DBuf<unsigned long long> xsurv;
    DBuf<uint32_t> xsoff, kpos, tpos, rowcnt, rownb, kidx2, rpos, oe_small;
    OeGroups oe_rg{};   // owner emission: the next sbd_receive's source segments (sbd_oe_segments)
    uint32_t* h_oe = nullptr;             // pinned: per-group totals, tie count
    // sharded key pass timing (flags bit 0): an event pair around each part's key kernel (k_keys_a / k_mkeys_a)
    hipEvent_t kp_ev[32] = {};
    int kp_n = 0;
    double htr[3] = {};                   // SB_HOST_TRACE: host times (ms) of the step's sync start / end, emission            // host-scored turn (SB_HEUR_HOST): next_queue size awaiting sb_prune
};

// Visited-set capacity policy.  A table is rebuilt larger before a turn whose worst case (every raw
// child a new key) could take it past GROW_LOAD; the size doubles while the free HBM allows (old and
// new coexist during the rehash, GROW_RESERVE kept free for the step buffers).  If no larger table
// fits, the old one stays and the HARD_LOAD check after the turn is the capacity limit.
constexpr double GROW_LOAD = 0.6;
constexpr double HARD_LOAD = 0.85;
constexpr size_t GROW_RESERVE = (size_t)4 << 30;

// SB_DEBUG_VISITED_MAX=<slots> (tests): a visited-set rebuild above it fails as if the HBM were taken
static bool debug_visited_allows(uint64_t slots) {
    const char* lim = std::getenv("SB_DEBUG_VISITED_MAX");
    return !lim || (double)slots <= std::strtod(lim, nullptr);
}

static void grow_table(Engine& E, Entry*& tab, uint64_t& mask, double projected) {
    const uint64_t cap = mask + 1;
    uint64_t ncap = cap;
    const double grow_load = (E.cfg.flags & 16) ? 0.25 : GROW_LOAD;   // flags bit 4 (test): eager growth
    while (projected > grow_load * (double)ncap && ncap < (1ull << 36)) ncap <<= 1;
    if (ncap == cap) return;
    const uint64_t want = ncap;
    size_t freeb = 0, totalb = 0;
    SB_HIP(hipMemGetInfo(&freeb, &totalb));
    while (ncap > cap && ncap * sizeof(Entry) + GROW_RESERVE > freeb) ncap >>= 1;
    // Another process on the GPU (ranks sharing it) may take HBM between the sizing and the allocation: then a
    // smaller table, or none — growth is ahead of need, and the HARD_LOAD check after the turn is the limit.  Either
    // is counted (n_grow_short, n_grow_skip: sb_visited_stats)
    Entry* nt = nullptr;
    for (; ncap > cap; ncap >>= 1) {
        if (debug_visited_allows(ncap) && debug_hbm_allows(ncap * sizeof(Entry)) &&
            hipMalloc((void**)&nt, ncap * sizeof(Entry)) == hipSuccess)
            break;
        (void)hipGetLastError();
        nt = nullptr;
    }
    if (!nt) {
        E.n_grow_skip++;
        return;
    }
    if (ncap < want) E.n_grow_short++;
    SB_HIP(hipMemsetAsync(nt, 0xFF, ncap * sizeof(Entry), E.s));
    hipLaunchKernelGGL(k_rehash, dim3(grid_cap((int64_t)std::min<uint64_t>(cap, 1ull << 40), 256, 1u << 16)), dim3(256), 0,
                       E.s, tab, cap, nt, ncap - 1, E.d_small + 1);
    SB_HIP(hipGetLastError());
    SB_HIP(hipStreamSynchronize(E.s));
    SB_HIP(hipFree(tab));
    tab = nt;
    mask = ncap - 1;
    E.n_grow++;
}

// initial capacity (log2 entries) when visited_log2 = 0: `want` entries, at most a third of the free HBM
static int auto_visited_log2(double want) {
    size_t freeb = 0, totalb = 0;
    SB_HIP(hipMemGetInfo(&freeb, &totalb));
    int lg = 20;
    while ((double)(1ull << lg) < want && lg < 34 && (double)(2ull << lg) * sizeof(Entry) <= (double)freeb / 3.0) lg++;
    return lg;
}

static void check_err_word(Engine& E) {
    uint32_t e = E.h_small[1];
    if (e & 1u) throw HipError{hipErrorOutOfMemory, "visited set overfull (probe limit); raise visited_log2"};
    if (e & 2u) throw HipError{hipErrorInvalidValue, "saved >= 256 exceeds the pow tables"};
    if (e & 4u) throw HipError{hipErrorLaunchFailure, "top-k sort look-back wait exceeded its bound"};
    if (e & 8u) throw HipError{hipErrorLaunchFailure, "sharded answers do not match the parents' move counts"};
    if (e & 16u) throw HipError{hipErrorInvalidValue, "heuristic returned NaN: no stable sort order exists"};
    if (e & 32u) throw HipError{hipErrorLaunchFailure, "top-k sort fix-up: more distinct keys in one prefix run than it holds"};
    if (e & 64u) throw HipError{hipErrorOutOfMemory, "sharded records exceed the compact record buffers (flags bit 5)"};
    if (e & 128u) throw HipError{hipErrorLaunchFailure, "card-set sharded claims: a displaced record is not where its parent maps"};
    if (e & 256u) throw HipError{hipErrorLaunchFailure, "grouped kept records: a segment's groups do not add up to its children"};
}

static float ev_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 0.f;
    return ms;
}

// Step buffers sized up front for a saturated beam (about 12.5 unique children per parent at most on
// the goal-15 trajectories; DBuf grows past that if ever needed): a hipMalloc/hipFree on the step
// path would serialise against in-flight work.
// Sharded mode: the per-rank buffers of a saturated step sized up front from the local share of the
// beam (records ≈ b_raw ≤ 32 per parent, survivors ≤ 14 per parent, 25% slack for uneven owners),
// so that no hipMalloc lands in a timed step.
static void preallocate_dist(Engine& E) {
    const size_t wl = (size_t)(E.cfg.beam_width / std::max(1, (int)E.cfg.world_size) + 1) * 5 / 4;
    const size_t nr = wl * 32, nu = wl * 14;
    E.surv.ensure(wl * 3);
    E.cnt.ensure(wl);
    E.off.ensure(wl);
    E.cand.ensure(wl * 3);
    E.lost.ensure(wl * 3);
    if (E.cfg.world_size > 1) {   // record buffers for the worst case: sbd_expand_launch needs no host count
        E.cand_key.ensure(wl * E.rec_per_parent);
        E.cand_pos.ensure(wl * E.rec_per_parent);
        E.digit.ensure(wl * E.rec_per_parent);
        E.rdsc.ensure(wl * E.rec_per_parent);
    }
    E.own_lost.ensure(nr / 64 + 1);
    E.nlo.ensure(nu);
    E.nhi.ensure(nu);
    E.npar.ensure(nu);
    E.skey.ensure(nu);
    E.dsel_c.ensure(nu);
    E.dsel_ci.ensure(nu);
    // the joint select's tile counts, tie tiles and destinations grow with the turn's unique children:
    // a mid-step regrowth (hipFree) waits for the device to drain (0.2-0.5 ms each, sbd_sel_compact /
    // sbd_partition); tiles of 4096 keys (sb_dist.inc PT_TILE)
    const size_t dtiles = nu / 4096 + 2;
    E.dsel_t.ensure(dtiles);
    E.digit.ensure(nu);
    E.part_hist.ensure(dtiles * (size_t)std::max(1, (int)E.cfg.world_size) + 80 + 16 * 64);
    E.kidx.ensure(wl);
    E.rkey.ensure(wl);
    topk_reserve(E.topk, (int64_t)wl, (int64_t)wl);   // the receive sort (the joint select is k_ds_*) ...
    E.topk.tile_a.ensure(dtiles + 1);                 // ... and the joint select's tie / destination tiles
    E.scan.tiles.ensure(nr / SCAN_TILE + 1);
    E.turn_mem.reserve(wl * 20 * 24);
}

static void preallocate(Engine& E) {
    const size_t W = (size_t)E.cfg.beam_width, nu = W * 14;
    E.cand.ensure(W * 3);
    E.lost.ensure(W * 3);
    E.cnt.ensure(W);
    E.off.ensure(W);
    E.nlo.ensure(nu);
    E.nhi.ensure(nu);
    E.npar.ensure(nu);
    E.skey.ensure(nu);
    E.kidx.ensure(W);
    topk_reserve(E.topk, (int64_t)nu, (int64_t)W);
    E.scan.tiles.ensure(W / SCAN_TILE + 1);
    E.turn_mem.block_bytes = std::max(E.turn_mem.block_bytes, W * 20 * 8);   // eight beams per block
    E.turn_mem.reserve(W * 20 * 24);   // a goal-15 run keeps < 24 saturated beams: no hipMalloc mid-run
}

// Per-turn device timing (flags bit 0): event set [turn % TEV_RING]: 0 expand start, 1 expand end,
// 2 count+scan end, 3 emit start, 4 emit end, 5 top-k end, 6 gather end.
constexpr int TEV_RING = 64;

static hipEvent_t* tev(Engine& E, int turn) {
    if (E.tev.empty()) {
        E.tev.resize((size_t)TEV_RING * 7);
        for (auto& ev : E.tev) SB_HIP(hipEventCreate(&ev));
    }
    return &E.tev[(size_t)(turn % TEV_RING) * 7];
}

// Front half of a step for the current beam, launched as soon as that beam exists (right after the
// previous gather): expansion + claims, survivor counts and offsets, then one readback of the
// small state: n_unique, error word, the beam's per-pts first-rank table (gather) and n_raw.  The
// next sb_step waits on this readback only — the goal check and the sizes come from one round trip.
// The engine stream and the noise producers' side stream.  SB_STREAM_PRIO=1: the side stream at the lowest
// priority, the engine stream at the highest, so a noise chunk's kernels would take only CUs the step's
// kernels leave (a chunk's placement kernel landing on the emission cost it ~100 us in one traced turn).
// A/B over three interleaved rounds (profiles/r3/s5/ab_front.txt): 866.7 M states/s either way (the
// expansion's box drift, 3.19-3.52 ms, is larger than any effect); off by default
#ifndef SB_STREAM_PRIO
#define SB_STREAM_PRIO 0
#endif
static void create_streams(hipStream_t& s, hipStream_t& s_mt) {
    int least = 0, greatest = 0;
    if (SB_STREAM_PRIO) SB_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    if (SB_STREAM_PRIO && least != greatest) {
        SB_HIP(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest));
        SB_HIP(hipStreamCreateWithPriority(&s_mt, hipStreamNonBlocking, least));
    } else {
        SB_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        SB_HIP(hipStreamCreateWithFlags(&s_mt, hipStreamNonBlocking));
    }
}

static void launch_front(Engine& E) {
    const bool timing = E.cfg.flags & 1;
    Turn& cur = E.turns.back();
    const int64_t n = cur.n;
    hipEvent_t* ev = timing ? tev(E, E.turn) : nullptr;
    // the claims below must fit: worst case every raw child is a new key
    grow_table(E, E.tab, E.tab_mask, (double)E.visited + E.raw_ratio * (double)n);
    E.cand.ensure((size_t)n * 3);
    const unsigned long long* lost_was = E.lost.p;
    E.lost.ensure((size_t)n * 3);
    if (E.lost.p != lost_was) E.lost_zero = 0;   // reallocated
    E.cnt.ensure((size_t)n);
    E.off.ensure((size_t)n);
    {
        const int64_t z = std::min<int64_t>(E.lost_zero, n);
        if (n > z) SB_HIP(hipMemsetAsync(E.lost.p + (size_t)z * 3, 0, (size_t)(n - z) * 24, E.s));
        E.lost_zero = 0;   // the expansion below marks [0, n)
    }
    // raw count, claim statistics (SB_CLAIM_STATS builds: [2..8)) and k_expand's group counter: one launch
    hipLaunchKernelGGL(k_front_reset, dim3(1), dim3(64), 0, E.s, E.d_nraw, E.d_small);
    const uint64_t turn_tag = (uint64_t)(E.turn + 1) << 40;
    if (timing) SB_HIP(hipEventRecord(ev[0], E.s));
    if (n > 0) {
        // a capped grid pulling groups of XP_PAR parents from a counter in rank order (a grid-stride
        // walk ran blocks a million ranks apart side by side: more displaced same-turn claims)
        hipLaunchKernelGGL(k_expand<false>, dim3(grid_cap(n, XP_PAR, SB_XP_GRID_CAP)), dim3(XP_NT), 0, E.s, E.d_tables,
                           cur.lo, cur.hi, n, E.tab, E.tab_mask, turn_tag, E.cand.p, E.lost.p, E.d_nraw, E.d_small + 1,
                           E.d_small + 264, 0u, 1u, (const uint32_t*)nullptr, (uint64_t*)nullptr, (uint8_t*)nullptr, 0ull,
                           (uint8_t*)nullptr);
    }
    if (timing) SB_HIP(hipEventRecord(ev[1], E.s));
    if (n > 0) {   // survivors per parent + their tile sums, then the offsets (next_queue order)
        E.scan.tiles.ensure((size_t)((n + SCAN_TILE - 1) / SCAN_TILE));
        hipLaunchKernelGGL(k_count_lm_tiles, dim3((unsigned)((n + SCAN_TILE - 1) / SCAN_TILE)), dim3(CLT_NT), 0, E.s, n,
                           E.cand.p, E.lost.p, E.cnt.p, E.scan.tiles.p);
        scan_exclusive_u32_sums(E.cnt.p, E.off.p, n, E.d_small, E.scan, E.s);
    } else {
        scan_exclusive_u32(E.cnt.p, E.off.p, n, E.d_small, E.scan, E.s);
    }
    if (timing) SB_HIP(hipEventRecord(ev[2], E.s));
    SB_HIP(hipMemcpyAsync(E.h_small, E.d_small, 264 * 4, hipMemcpyDeviceToHost, E.s));
    SB_HIP(hipMemcpyAsync(E.h_nraw, E.d_nraw, 8, hipMemcpyDeviceToHost, E.s));
    SB_HIP(hipGetLastError());
    E.front_turn = E.turn;
}

static void finish_turn(Engine& E, int64_t nu, bool heur, bool desc, const double* host_scores, sb_step_stats* out);
#ifndef SB_TOPK_DESC
#define SB_TOPK_DESC 1   // the top-k carries each kept survivor's descriptor (rank << 8 | dsc) instead of its index
#endif
// descriptor-only emission writes 4-byte descriptors that the top-k carries as its payload while parent
// ranks < 2^24 (else 8-byte descriptors and the gather reads them at the kept indices)
static bool desc_payload_ok(int64_t n_parents) { return SB_TOPK_DESC && n_parents < ((int64_t)1 << 24); }
static double host_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// f64 scores of a host heuristic -> u64 keys whose unsigned order is the scores' order (-0.0 == 0.0 as in
// Python's comparisons); a NaN has no place in that order (sorted() would not be a total order): error bit 16
__global__ void k_order_keys(uint64_t* __restrict__ k, int64_t n, uint32_t* __restrict__ err) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t b = k[i];
        if ((b & 0x7FFFFFFFFFFFFFFFull) > 0x7FF0000000000000ull) atomicOr(err, 16u);
        if (b == 0x8000000000000000ull) b = 0;
        k[i] = (b >> 63) ? ~b : (b | 0x8000000000000000ull);
    }
}

static void engine_step(Engine& E, sb_step_stats* out) {
    memset(out, 0, sizeof *out);
    out->turn = E.turn;
    if (E.done) {
        out->done = 1;
        out->winner_rank = E.winner_rank;
        return;
    }
    const bool timing = E.cfg.flags & 1;
    Turn& cur = E.turns.back();
    const int64_t n = cur.n;
    out->n_parents = n;
    if (E.front_turn != E.turn) launch_front(E);
    E.htr[0] = host_ms();
    SB_HIP(hipStreamSynchronize(E.s));
    E.htr[1] = host_ms();
    E.front_turn = -1;
    // ---- goal check and max_pts records, in queue order (src/solver.py:438-445)
    const uint32_t* first = E.h_small + 8;
    {
        int64_t win = -1;
        for (int p = E.cfg.goal_pts < 0 ? 0 : E.cfg.goal_pts; p < 256; p++)
            if (first[p] != 0xFFFFFFFFu && (win < 0 || first[p] < (uint32_t)win)) win = first[p];
        // records: successive minima of first[p] over p > running max, stopping at the winner
        int64_t last_rank = -1;
        for (;;) {
            int64_t best = -1;
            int bp = -1;
            for (int p = E.max_pts + 1; p < 256; p++)
                if (first[p] != 0xFFFFFFFFu && (best < 0 || first[p] < (uint32_t)best)) {
                    best = first[p];
                    bp = p;
                }
            if (best < 0 || (win >= 0 && best > win) || best <= last_rank) break;
            E.max_pts = bp;
            if (out->n_records < 32) {
                out->record_rank[out->n_records] = best;
                out->record_pts[out->n_records] = bp;
                out->n_records++;
            }
            last_rank = best;
        }
        if (win >= 0) {   // the speculative front half of this turn is discarded
            E.done = true;
            E.winner_rank = win;
            out->done = 1;
            out->winner_rank = win;
            out->noise_draws = E.noise.consumed;
            return;
        }
    }
    check_err_word(E);
#ifdef SB_CLAIM_STATS
    // err = d_small + 1: err[k] is h_small[k + 1]
    fprintf(stderr, "claims turn %d: old %u inserted %u early-out %u lost-at-min %u displaced %u in-group-dup %u\n",
            E.turn, E.h_small[2], E.h_small[3], E.h_small[4], E.h_small[5], E.h_small[6], E.h_small[7]);
#endif
    const bool heur = E.cfg.use_heuristic != 0;
    const bool host = heur && E.cfg.heuristic == SB_HEUR_HOST;   // scores from a host callable (sb_prune)
    const int64_t nu = E.h_small[0];
    out->n_raw = (int64_t)*E.h_nraw;
    out->n_unique = nu;
    E.visited += (uint64_t)nu;
    E.peak_load = std::max(E.peak_load, (double)E.visited / (double)(E.tab_mask + 1));
    if (n > 0) E.raw_ratio = std::max(E.raw_ratio, (double)out->n_raw / (double)n);
    if ((double)E.visited > HARD_LOAD * (double)(E.tab_mask + 1))
        throw HipError{hipErrorOutOfMemory, "visited set above 85% load and no larger table fits in free HBM"};
    if (nu == 0) {   // the queue empties: `puzzle` is the last parent expanded (src/solver.py:438,459)
        E.done = true;
        E.winner_rank = n - 1;
        out->done = 1;
        out->winner_rank = n - 1;
        out->noise_draws = E.noise.consumed;
        return;
    }
    E.nlo.ensure(nu);
    E.nhi.ensure(nu);
    E.npar.ensure(nu);
    if (heur && !host) {
        E.skey.ensure(nu);
        const auto t0 = std::chrono::steady_clock::now();
        noise_ensure(E.noise, (uint64_t)nu, E.s_mt);
        out->ms_sort = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
        E.last_nu = (uint64_t)nu;
    }
    hipEvent_t* ev = timing ? tev(E, E.turn) : nullptr;
    if (timing) SB_HIP(hipEventRecord(ev[3], E.s));
    E.htr[2] = host_ms();
    const unsigned eg = grid_cap(n, 256, 8192);
    const uint64_t rbase = E.noise.consumed;
#define EMIT_K(H) k_emit_w<H>
    if (!heur || host) {   // full states + parent links, no scores
        hipLaunchKernelGGL(EMIT_K(-1), dim3(eg), dim3(256), 0, E.s, E.d_tables, cur.lo, cur.hi, n, E.cand.p, E.lost.p,
                           E.off.p, E.nlo.p, E.nhi.p, E.npar.p, E.skey.p, E.noise.ring.p, E.noise.ring_mask, rbase, 0u,
                           E.d_small + 1, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                           (const uint64_t*)nullptr, 0);
    } else {
        const bool fused = !(E.cfg.flags & 4);
        // the gather's per-pts first-rank table reset by the same launch (the last turn's was read back in
        // launch_front, ahead on the stream)
        unsigned long long* krange = topk_range_reset(E.topk, E.s, fused, (E.cfg.flags & 8) != 0, E.d_small + 8);
        E.first_reset = true;
        unsigned long long* fh = topk_fused_hist(E.topk);
        const uint64_t* fb = topk_fused_base(E.topk);
#ifndef SB_EMIT_GRID
#define SB_EMIT_GRID 1536   // = resident blocks (24 KB LDS: 6 per CU): no partial second round of blocks
#endif
        const unsigned egf = grid_cap(n, 256, SB_EMIT_GRID);   // fewer blocks: one histogram flush per block
        const bool desc32 = desc_payload_ok(n);   // 4-byte descriptors, carried by the top-k (finish_turn)
        switch (E.cfg.heuristic) {
#define EMIT(H)                                                                                                   \
    hipLaunchKernelGGL((k_emit_w<H, false>), dim3(egf), dim3(256), 0, E.s, E.d_tables, cur.lo, cur.hi, n, E.cand.p, \
                       E.lost.p, E.off.p, E.nlo.p, E.nhi.p, E.npar.p, E.skey.p, E.noise.ring.p, E.noise.ring_mask, \
                       rbase, 0u, E.d_small + 1, krange, fh, fb, (int)desc32);                                    \
    break;
            case 1: EMIT(1)
            case 2: EMIT(2)
            case 3: EMIT(3)
            default: EMIT(0)
#undef EMIT
        }
#undef EMIT_K
        E.noise.consumed += (uint64_t)nu;
    }
    if (SB_EMIT_ZERO_LOST) E.lost_zero = n;   // k_emit_w cleared lost[0 .. 3n) after reading it
    if (timing) SB_HIP(hipEventRecord(ev[4], E.s));
    if (host) {   // the turn ends in sb_prune, once the caller has scored next_queue (sb_read_next)
        SB_HIP(hipGetLastError());
        E.pending_host = nu;
        out->n_kept = 0;
        return;
    }
    finish_turn(E, nu, heur, heur, nullptr, out);
}

// The prune and the next beam (src/solver.py:452-457): stable descending top-k of the score keys (heur),
// the kept states written as the next turn (rebuilt from descriptors when `desc`), then the next turn's
// expansion is launched.  host_scores: caller-supplied f64 scores of next_queue (custom heuristics).
static void finish_turn(Engine& E, int64_t nu, bool heur, bool desc, const double* host_scores, sb_step_stats* out) {
    const bool timing = E.cfg.flags & 1;
    Turn& cur = E.turns.back();
    const int64_t n = cur.n;
    hipEvent_t* ev = timing ? tev(E, E.turn) : nullptr;
    // ---- prune + next beam
    int64_t m = nu;
    uint32_t* idx = nullptr;
    const bool desc_pay = desc && heur && !host_scores && desc_payload_ok(n);
    if (heur) {
        E.kidx.ensure(std::min<int64_t>(nu, E.cfg.beam_width));
        if (host_scores) {   // f64 scores -> order-preserving u64 keys (a NaN sets error bit 16)
            SB_HIP(hipMemcpyAsync(E.skey.p, host_scores, (size_t)nu * 8, hipMemcpyHostToDevice, E.s));
            hipLaunchKernelGGL(k_order_keys, dim3(grid_cap(nu, 256, 8192)), dim3(256), 0, E.s, E.skey.p, nu, E.d_small + 1);
            m = topk_stable_desc(E.skey.p, nu, E.cfg.beam_width, E.kidx.p, E.topk, E.s, /*range_ready=*/false,
                                 E.d_small + 1, /*fused=*/false, nullptr, /*full_key=*/true);
        } else {
            m = topk_stable_desc(E.skey.p, nu, E.cfg.beam_width, E.kidx.p, E.topk, E.s, /*range_ready=*/true,
                                 E.d_small + 1, /*fused=*/!(E.cfg.flags & 4),
                                 desc_pay ? reinterpret_cast<const uint32_t*>(E.nlo.p) : nullptr);
        }
        idx = E.kidx.p;
    }
    if (timing) SB_HIP(hipEventRecord(ev[5], E.s));
    Turn nt;
    nt.lo = (uint64_t*)E.turn_mem.alloc(m * 8);
    nt.hi = (uint64_t*)E.turn_mem.alloc(m * 8);
    nt.par = (uint32_t*)E.turn_mem.alloc(m * 4);
    nt.n = m;
    if (!E.first_reset) SB_HIP(hipMemsetAsync(E.d_small + 8, 0xFF, 256 * 4, E.s));
    E.first_reset = false;
#ifndef SB_GATHER_GRID
#define SB_GATHER_GRID 4096   // blocks of the descriptor gather (each thread walks m / (256 * grid) kept states)
#endif
#ifndef SB_GATHER_ZERO_LOST
#define SB_GATHER_ZERO_LOST 0   // 1: the gather clears the next turn's lost marks instead of a memset before the
                                // expansion.  A/B (profiles/r3/s5/ab_front.txt): gather +12-16 us, memset -14 us
#endif
    if (desc) {   // emission wrote descriptors only: rebuild the kept states from their parents
        unsigned long long* zl = SB_GATHER_ZERO_LOST && E.lost.cap >= (size_t)m * 3 ? E.lost.p : nullptr;
        hipLaunchKernelGGL(k_gather_d, dim3(grid_cap(m, 256, SB_GATHER_GRID)), dim3(256), 0, E.s, E.d_tables, idx, m, E.nlo.p,
                           cur.lo, cur.hi, nt.lo, nt.hi, nt.par, E.d_small + 8, (int)desc_pay, zl);
        if (zl) E.lost_zero = m;
    } else
        hipLaunchKernelGGL(k_gather, dim3(grid_cap(m, 256, 4096)), dim3(256), 0, E.s, idx, m, E.nlo.p, E.nhi.p, E.npar.p,
                           nt.lo, nt.hi, nt.par, E.d_small + 8);
    if (timing) SB_HIP(hipEventRecord(ev[6], E.s));
    SB_HIP(hipGetLastError());
    E.turns.push_back(nt);
    E.turn++;
    out->n_kept = m;
    out->noise_draws = E.noise.consumed;
    static const bool htrace = getenv("SB_HOST_TRACE") != nullptr;
    const double h3 = host_ms();
#ifndef SB_MT_GATE
#define SB_MT_GATE 1   // noise generation starts after this turn's gather: beside the next expansion, not the top-k
#endif
    if (SB_MT_GATE && heur && !host_scores) SB_HIP(hipEventRecord(E.ev[1], E.s));
    if (E.lookahead) launch_front(E);   // the next turn's expansion follows the gather on the stream
    const double h4 = host_ms();
    if (htrace)
        fprintf(stderr, "turn %d sync %.3f pre-emit %.3f back %.3f front %.3f | old %u ins %u dup_early %u dup_lost %u displaced %u\n",
                E.turn, E.htr[1] - E.htr[0], E.htr[2] - E.htr[1], h3 - E.htr[2], h4 - h3, E.h_small[2], E.h_small[3],
                E.h_small[4], E.h_small[5], E.h_small[6]);
    // noise for the next turns on the side stream, overlapping that (latency-bound) expansion:
    // keep about three steps of accepted draws ahead
    if (heur && !host_scores && E.noise.produced - E.noise.consumed < 3 * (uint64_t)nu + (uint64_t)n) {
        if (SB_MT_GATE) SB_HIP(hipStreamWaitEvent(E.s_mt, E.ev[1], 0));
        noise_generate_async(E.noise, E.s_mt);
    }
}

// device phase times of a completed turn (timing flag): expand, count+scan, host gap, emit, top-k,
// gather, total
static void turn_times(Engine& E, int turn, float* out7) {
    if (E.tev.empty() || turn < 0 || turn >= E.turn || E.turn - turn > TEV_RING)
        throw HipError{hipErrorInvalidValue, "no timing for that turn (timing flag off or too old)"};
    hipEvent_t* ev = tev(E, turn);
    SB_HIP(hipEventSynchronize(ev[6]));
    out7[0] = ev_ms(ev[0], ev[1]);
    out7[1] = ev_ms(ev[1], ev[2]);
    out7[2] = ev_ms(ev[2], ev[3]);
    out7[3] = ev_ms(ev[3], ev[4]);
    out7[4] = ev_ms(ev[4], ev[5]);
    out7[5] = ev_ms(ev[5], ev[6]);
    out7[6] = ev_ms(ev[0], ev[6]);
}

}  // namespace sb

// ====================================================================== C-ABI
using namespace sb;

struct sb_engine {
    Engine E;
};

template <class F>
static int guarded(F&& f) {
    try {
        return f();
    } catch (const HipError& e) {
        set_error(e.what);
        return e.code == hipErrorOutOfMemory ? SB_ERR_CAPACITY : SB_ERR_HIP;
    } catch (const std::exception& e) {
        set_error(e.what());
        return SB_ERR_HIP;
    }
}

extern "C" {

int sb_version(void) { return 1; }

// one device allocation of `bytes` through the engine's allocator (then freed): its failure message, as every
// engine allocation reports it (what, bytes requested, free HBM); SB_DEBUG_HBM_LIMIT forces the failure (tests, CPU)
int sb_debug_alloc(uint64_t bytes) {
    return guarded([&]() {
        void* p = nullptr;
        dev_malloc(&p, (size_t)bytes, "sb_debug_alloc");
        SB_HIP(hipFree(p));
        return SB_OK;
    });
}
#ifndef SB_BUILD_ID
#define SB_BUILD_ID "unknown"
#endif
// sha256 of the sources this library was compiled from (_lib.source_hash): the loader refuses a stale build
const char* sb_build_id(void) { return SB_BUILD_ID; }
const char* sb_last_error(void) { return g_err.c_str(); }

int sb_init_tables(const int32_t* deck_rows, const double* pow_tables, const double* noise) {
    if (!deck_rows || !pow_tables || !noise) {
        set_error("sb_init_tables: null argument");
        return SB_ERR_ARG;
    }
    static Tables T;   // validated copy; published to g_host_tables only on success
    memset(&T, 0, sizeof T);
    for (int c = 0; c < NCARDS; c++) {
        const int32_t* r = deck_rows + c * 7;
        uint32_t w = 0;
        for (int i = 0; i < NCOL; i++) {
            if (r[i] < 0 || r[i] > MAXG) {
                set_error("sb_init_tables: card cost out of range");
                return SB_ERR_ARG;
            }
            w |= (uint32_t)r[i] << (3 * i);
        }
        if (r[5] < 0 || r[5] > 7 || r[6] < 0 || r[6] >= NCOL) {
            set_error("sb_init_tables: card pt/colour out of range");
            return SB_ERR_ARG;
        }
        w |= (uint32_t)r[5] << 15;
        w |= (uint32_t)r[6] << 18;
        T.card[c] = w;
        if (c < 64) T.colmask_lo[r[6]] |= 1ull << c;
        else T.colmask_hi[r[6]] |= 1u << (c - 64);
    }
    build_patterns(T);
    build_enum_tables(T);
    memcpy(T.pw, pow_tables, sizeof T.pw);
    memcpy(T.noise, noise, sizeof T.noise);
    (void)npat_host;
    g_host_tables = T;
    g_tables_ready = true;
    return SB_OK;
}

static Tables* upload_tables(hipStream_t st) {
    Tables* d = nullptr;
    SB_HIP(hipMalloc((void**)&d, sizeof(Tables)));
    SB_HIP(hipMemcpyAsync(d, &g_host_tables, sizeof(Tables), hipMemcpyHostToDevice, st));
    return d;
}

int sb_create(const sb_config* cfg, const uint32_t* mt_state625, uint64_t root_lo, uint64_t root_hi, sb_engine** out) {
    if (!cfg || !mt_state625 || !out) {
        set_error("sb_create: null argument");
        return SB_ERR_ARG;
    }
    if (!g_tables_ready) {
        set_error("sb_create: call sb_init_tables first");
        return SB_ERR_NOTABLES;
    }
    if (cfg->beam_width <= 0 || mt_state625[624] > 624) {
        set_error("sb_create: bad beam_width or MT position");
        return SB_ERR_ARG;
    }
    if ((cfg->world_size > 1 || (cfg->flags & 2)) && cfg->use_heuristic &&
        (cfg->beam_width + std::max(1, (int)cfg->world_size) - 1) / std::max(1, (int)cfg->world_size) > (int64_t)SH_RANK_MASK + 1) {
        // sharded: a rank's slice of the beam indexes its own claims' tags in 26 bits (SH_RANK_MASK)
        set_error("sb_create: beam_width / world_size exceeds 2^26 parents per rank (sharded claim tags); use more ranks");
        return SB_ERR_CAPACITY;
    }
    sb_engine* h = new sb_engine();
    int rc = guarded([&]() {
        Engine& E = h->E;
        E.cfg = *cfg;
        {   // turn storage blocks of about four beams
            const int64_t wl = cfg->beam_width / std::max(1, (int)cfg->world_size) + 1;
            E.turn_mem.block_bytes = std::max<size_t>((size_t)256 << 20, (size_t)wl * 4 * 20);
        }
        if (cfg->flags & 32) E.rec_per_parent = 48;   // compact sharded record buffers (several ranks per GPU)
        E.dev = cfg->device;
        SB_HIP(hipSetDevice(E.dev));
        create_streams(E.s, E.s_mt);
        hipLaunchKernelGGL(k_init_hgems, dim3((1 << 15) / 256), dim3(256), 0, E.s);   // (per process and device: cheap)
        for (auto& e : E.ev) SB_HIP(hipEventCreate(&e));
        E.d_tables = upload_tables(E.s);
        int lg = cfg->visited_log2;
        if (lg <= 0)   // ~10 unique children per parent per turn, ~20 turns, <= 50% load; grown past that
            lg = auto_visited_log2((double)cfg->beam_width * 10.0 * 20.0 * 2.0 / (cfg->world_size > 1 ? cfg->world_size : 1));
        if (lg < 10 || lg > 34) throw HipError{hipErrorInvalidValue, "visited_log2 out of range [10, 34]"};
        const uint64_t cap = 1ull << lg;
        const bool distm = cfg->world_size > 1 || (cfg->flags & 2);   // bit 1: sharded protocol at any world size
        const uint64_t tcap = distm ? 1024 : cap;   // sharded: the trail lives in the owner shards (E.own)
        E.tab_mask = tcap - 1;
        dev_malloc((void**)&E.tab, tcap * sizeof(Entry), "visited set");
        SB_HIP(hipMemsetAsync(E.tab, 0xFF, tcap * sizeof(Entry), E.s));
        if (distm) {
            if (cfg->rank < 0 || cfg->rank >= cfg->world_size || cfg->world_size > 64)
                throw HipError{hipErrorInvalidValue, "bad rank / world_size (<= 64)"};
            E.own_mask = cap - 1;
            E.mig = (cfg->flags & 256) != 0 && cfg->world_size > 1;   // card-set ownership (sb_mig.inc)
            E.oe = E.mig && (cfg->flags & 512) != 0;                    // owner emission (sb_oe.inc)
            E.goc = !E.mig && (cfg->flags & 2048) != 0;                 // global-order claims (key ownership)
            dev_malloc((void**)&E.own, cap * sizeof(Entry), "owner visited shard");
            SB_HIP(hipMemsetAsync(E.own, 0xFF, cap * sizeof(Entry), E.s));
        }
        SB_HIP(hipMalloc((void**)&E.d_small, 272 * 4));
        SB_HIP(hipMalloc((void**)&E.d_nraw, 8));
        SB_HIP(hipHostMalloc((void**)&E.h_small, 272 * 4, hipHostMallocDefault));
        SB_HIP(hipHostMalloc((void**)&E.h_nraw, 8, hipHostMallocDefault));
        SB_HIP(hipMemsetAsync(E.d_small, 0, 272 * 4, E.s));
        // root: turn 0, visited = {root}
        Turn t0;
        t0.lo = (uint64_t*)E.turn_mem.alloc(8);
        t0.hi = (uint64_t*)E.turn_mem.alloc(8);
        t0.par = (uint32_t*)E.turn_mem.alloc(4);
        uint32_t nopar = 0xFFFFFFFFu;
        SB_HIP(hipMemcpyAsync(t0.lo, &root_lo, 8, hipMemcpyHostToDevice, E.s));
        SB_HIP(hipMemcpyAsync(t0.hi, &root_hi, 8, hipMemcpyHostToDevice, E.s));
        SB_HIP(hipMemcpyAsync(t0.par, &nopar, 4, hipMemcpyHostToDevice, E.s));
        t0.n = (!distm || cfg->rank == 0) ? 1 : 0;   // sharded: the root is global rank 0, held by rank 0
        E.turns.push_back(t0);
        hipLaunchKernelGGL(k_insert_root, dim3(1), dim3(1), 0, E.s, E.tab, E.tab_mask, key_of(root_lo, root_hi));
        if (distm) hipLaunchKernelGGL(k_insert_root, dim3(1), dim3(1), 0, E.s, E.own, E.own_mask, key_of(root_lo, root_hi));
        SB_HIP(hipMemsetAsync(E.d_small + 8, 0xFF, 256 * 4, E.s));
        hipLaunchKernelGGL(k_pts_first, dim3(1), dim3(256), 0, E.s, t0.hi, t0.n, E.d_small + 8);
        // MT chunk = 256 producers x twists x 624 words ~ 16 draws per beam slot; ring >= 4 chunks
        int64_t twists = 1;
        while (twists < 4096 && (double)twists * 256 * 624 < (double)cfg->beam_width * 16) twists <<= 1;
        if (distm) {   // sharded: one round (a chunk per rank) covers >= 2 steps (~12.5 W draws per step)
            twists = 1;
            while (twists < 4096 && (double)twists * 256 * 624 * std::max(1, (int)cfg->world_size) <
                                        (double)cfg->beam_width * 64)
                twists <<= 1;
        }
        uint64_t ring = 1ull << 24;
        while ((ring < (uint64_t)cfg->beam_width * 64 || ring < 4ull * 256 * 624 * (uint64_t)twists) &&
               ring < (1ull << 35))
            ring <<= 1;
        noise_init(E.noise, mt_state625, ring, twists, E.s);
        if (distm && cfg->use_heuristic) noise_shard_setup(E.noise, cfg->rank, cfg->world_size, E.s);
        if (!distm && cfg->use_heuristic && cfg->beam_width <= (1ll << 24)) preallocate(E);
        if (distm && cfg->use_heuristic && cfg->beam_width / std::max(1, (int)cfg->world_size) <= (1ll << 24))
            preallocate_dist(E);
        SB_HIP(hipStreamSynchronize(E.s));
        return SB_OK;
    });
    if (rc != SB_OK) {
        sb_destroy(h);
        return rc;
    }
    *out = h;
    return SB_OK;
}

int sb_step(sb_engine* h, sb_step_stats* out) {
    if (!h || !out) {
        set_error("sb_step: null argument");
        return SB_ERR_ARG;
    }
    if (h->E.mode != 0) {
        set_error("sb_step: realistic handle (use sbr_step)");
        return SB_ERR_STATE;
    }
    if (h->E.pending_host >= 0) {
        set_error("sb_step: the previous turn awaits its host scores (sb_prune)");
        return SB_ERR_STATE;
    }
    return guarded([&]() {
        SB_HIP(hipSetDevice(h->E.dev));
        engine_step(h->E, out);
        return SB_OK;
    });
}

int sb_read_next(sb_engine* h, int64_t start, int64_t n, uint64_t* lo, uint64_t* hi) {
    if (!h || h->E.pending_host < 0) {
        set_error("sb_read_next: no host-scored turn pending");
        return SB_ERR_STATE;
    }
    Engine& E = h->E;
    if (start < 0 || n < 0 || start + n > E.pending_host) {
        set_error("sb_read_next: range out of bounds");
        return SB_ERR_ARG;
    }
    if (n == 0) return SB_OK;
    return guarded([&]() {
        SB_HIP(hipSetDevice(E.dev));
        if (lo) SB_HIP(hipMemcpyAsync(lo, E.nlo.p + start, n * 8, hipMemcpyDeviceToHost, E.s));
        if (hi) SB_HIP(hipMemcpyAsync(hi, E.nhi.p + start, n * 8, hipMemcpyDeviceToHost, E.s));
        SB_HIP(hipStreamSynchronize(E.s));
        return SB_OK;
    });
}

int sb_prune(sb_engine* h, const double* scores, int64_t n, int64_t* n_kept) {
    if (!h || !scores || !n_kept) {
        set_error("sb_prune: null argument");
        return SB_ERR_ARG;
    }
    Engine& E = h->E;
    if (E.pending_host < 0) {
        set_error("sb_prune: no host-scored turn pending");
        return SB_ERR_STATE;
    }
    if (n != E.pending_host) {
        set_error("sb_prune: one score per next_queue entry expected");
        return SB_ERR_ARG;
    }
    return guarded([&]() {
        SB_HIP(hipSetDevice(E.dev));
        sb_step_stats st;
        memset(&st, 0, sizeof st);
        E.skey.ensure((size_t)n);
        E.htr[2] = host_ms();
        E.pending_host = -1;
        finish_turn(E, n, true, false, scores, &st);
        SB_HIP(hipStreamSynchronize(E.s));   // the caller's score buffer is free on return
        check_err_word(E);
        *n_kept = st.n_kept;
        return SB_OK;
    });
}

int sb_turn_times(sb_engine* h, int32_t turn, float* out7) {
    if (!h || !out7) return SB_ERR_ARG;
    return guarded([&]() {
        SB_HIP(hipSetDevice(h->E.dev));
        turn_times(h->E, turn, out7);
        return SB_OK;
    });
}

int sb_num_turns(sb_engine* h, int32_t* out) {
    if (!h || !out) return SB_ERR_ARG;
    *out = (int32_t)h->E.turns.size();
    return SB_OK;
}

int sb_turn_size(sb_engine* h, int32_t turn, int64_t* out) {
    if (!h || !out || turn < 0 || turn >= (int32_t)h->E.turns.size()) {
        set_error("sb_turn_size: bad turn");
        return SB_ERR_ARG;
    }
    *out = h->E.turns[turn].n;
    return SB_OK;
}

int sb_read_turn(sb_engine* h, int32_t turn, int64_t start, int64_t n, uint64_t* lo, uint64_t* hi, uint32_t* par,
                 uint64_t* key) {
    if (!h || turn < 0 || turn >= (int32_t)h->E.turns.size()) {
        set_error("sb_read_turn: bad turn");
        return SB_ERR_ARG;
    }
    Engine& E = h->E;
    const Turn& t = E.turns[turn];
    if (start < 0 || n < 0 || start + n > t.n) {
        set_error("sb_read_turn: range out of bounds");
        return SB_ERR_ARG;
    }
    if (n == 0) return SB_OK;
    return guarded([&]() {
        SB_HIP(hipSetDevice(E.dev));
        if (lo) SB_HIP(hipMemcpyAsync(lo, t.lo + start, n * 8, hipMemcpyDeviceToHost, E.s));
        if (hi) SB_HIP(hipMemcpyAsync(hi, t.hi + start, n * 8, hipMemcpyDeviceToHost, E.s));
        if (par) SB_HIP(hipMemcpyAsync(par, t.par + start, n * 4, hipMemcpyDeviceToHost, E.s));
        if (key) {
            uint64_t* dk = nullptr;
            SB_HIP(hipMalloc((void**)&dk, n * 8));
            hipLaunchKernelGGL(k_keys, dim3(grid_cap(n, 256, 4096)), dim3(256), 0, E.s, t.lo + start, t.hi + start, n, dk);
            SB_HIP(hipMemcpyAsync(key, dk, n * 8, hipMemcpyDeviceToHost, E.s));
            SB_HIP(hipStreamSynchronize(E.s));
            SB_HIP(hipFree(dk));
        }
        SB_HIP(hipStreamSynchronize(E.s));
        return SB_OK;
    });
}

int sb_path(sb_engine* h, uint64_t* lo, uint64_t* hi, int32_t cap, int32_t* len) {
    if (!h || !lo || !hi || !len) return SB_ERR_ARG;
    Engine& E = h->E;
    if (!E.done) {
        set_error("sb_path: search not finished");
        return SB_ERR_STATE;
    }
    const int T = (int)E.turns.size();
    if (cap < T) {
        set_error("sb_path: cap too small");
        return SB_ERR_ARG;
    }
    return guarded([&]() {
        SB_HIP(hipSetDevice(E.dev));
        SB_HIP(hipStreamSynchronize(E.s));
        int64_t r = E.winner_rank;
        for (int t = T - 1; t >= 0; t--) {
            uint32_t p = 0;
            SB_HIP(hipMemcpy(&lo[t], E.turns[t].lo + r, 8, hipMemcpyDeviceToHost));
            SB_HIP(hipMemcpy(&hi[t], E.turns[t].hi + r, 8, hipMemcpyDeviceToHost));
            SB_HIP(hipMemcpy(&p, E.turns[t].par + r, 4, hipMemcpyDeviceToHost));
            r = p;
        }
        *len = T;
        return SB_OK;
    });
}

int sb_get_mt_state(sb_engine* h, uint32_t* out625) {
    if (!h || !out625) return SB_ERR_ARG;
    noise_mt_state(h->E.noise, out625);
    return SB_OK;
}

int sb_set_lookahead(sb_engine* h, int32_t on) {
    if (!h) return SB_ERR_ARG;
    h->E.lookahead = on != 0;
    return SB_OK;
}

int sb_sync_engine(sb_engine* h) {
    if (!h) return SB_ERR_ARG;
    return guarded([&]() {
        SB_HIP(hipSetDevice(h->E.dev));
        SB_HIP(hipStreamSynchronize(h->E.s));
        return SB_OK;
    });
}

int sb_sync(sb_engine* h) {
    if (!h) return SB_ERR_ARG;
    return guarded([&]() {
        SB_HIP(hipSetDevice(h->E.dev));
        SB_HIP(hipStreamSynchronize(h->E.s));
        SB_HIP(hipStreamSynchronize(h->E.s_mt));
        return SB_OK;
    });
}

int sb_visited_size(sb_engine* h, uint64_t* out) {
    if (!h || !out) return SB_ERR_ARG;
    *out = h->E.visited;
    return SB_OK;
}

int sb_visited_stats(sb_engine* h, uint64_t* out6) {
    if (!h || !out6) return SB_ERR_ARG;
    const Engine& E = h->E;
    out6[0] = (E.own ? E.own_mask : E.tab_mask) + 1;
    out6[1] = (uint64_t)E.n_grow;
    out6[2] = (uint64_t)E.n_grow_short;
    out6[3] = (uint64_t)E.n_grow_skip;
    out6[4] = (uint64_t)(E.peak_load * 1e6 + 0.5);   // ppm
    out6[5] = E.own ? E.own_visited : E.visited;
    return SB_OK;
}

int sb_visited_capacity(sb_engine* h, uint64_t* capacity, int32_t* rebuilds) {
    if (!h || !capacity || !rebuilds) return SB_ERR_ARG;
    const Engine& E = h->E;
    *capacity = (E.own ? E.own_mask : E.tab_mask) + 1;
    *rebuilds = E.n_grow;
    return SB_OK;
}

void sb_destroy(sb_engine* h) {
    if (!h) return;
    Engine& E = h->E;
    (void)hipSetDevice(E.dev);
    if (E.s) (void)hipStreamSynchronize(E.s);
    if (E.s_mt) (void)hipStreamSynchronize(E.s_mt);
    E.turn_mem.release();
    E.desc.release();
    E.rslot.release();
    E.cand.release();
    E.lost.release();
    E.surv.release();
    E.cnt.release();
    E.off.release();
    E.nlo.release();
    E.nhi.release();
    E.skey.release();
    E.npar.release();
    E.kidx.release();
    E.scan.tiles.release();
    E.topk.release();
    noise_free(E.noise);
    if (E.tab) (void)hipFree(E.tab);
    if (E.own) (void)hipFree(E.own);
    if (E.d_rfirst) (void)hipFree(E.d_rfirst);
    if (E.h_rfirst) (void)hipHostFree(E.h_rfirst);
    E.nw.release();
    E.cand_key.release();
    E.cand_tag.release();
    E.cand_ro.release();
    E.cand_pos.release();
    E.own_slot.release();
    E.own_lost.release();
    E.dsel.release();
    E.dsel_c.release();
    E.dsel_t.release();
    E.dsel_ci.release();
    E.rkey.release();
    E.part_hist.release();
    E.digit.release();
    E.rdsc.release();
    E.mrj.release();
    E.snv.release();
    E.rkey2.release();
    E.mcrec.release();
    if (E.s_claim) (void)hipStreamSynchronize(E.s_claim);
    E.ks_rdr.release();
    E.ks_sown.release();
    E.ks_cc.release();
    E.ks_tot.release();
    E.ks_pc.release();
    E.ks_tk.release();
    E.mdig.release();
    E.mpos.release();
    E.mhist.release();
    E.xg.release();
    E.xcnt.release();
    E.xoff.release();
    E.gmap.release();
    E.xlo.release();
    E.xhi.release();
    E.mtag.release();
    E.mraw.release();
    E.mrawsend.release();
    E.mrawoff.release();
    E.mrawown.release();
    E.xsurv.release();
    E.xsoff.release();
    E.kpos.release();
    E.gdig.release();
    E.gk_hist.release();
    E.gk_off.release();
    E.gk_cnt.release();
    E.gk_coff.release();
    E.tpos.release();
    E.rowcnt.release();
    E.rownb.release();
    E.kidx2.release();
    E.rpos.release();
    E.oe_small.release();
    if (E.h_oe) (void)hipHostFree(E.h_oe);
    if (E.h_mpc) (void)hipHostFree(E.h_mpc);
    if (E.mig_ev) (void)hipEventDestroy(E.mig_ev);
    for (auto& e : E.kp_ev)
        if (e) (void)hipEventDestroy(e);
    if (E.h_pc) (void)hipHostFree(E.h_pc);
    if (E.h_goc) (void)hipHostFree(E.h_goc);
    if (E.goc_ev) (void)hipEventDestroy(E.goc_ev);
    E.goc_seg.release();
    for (auto& e : E.ks_ev)
        if (e) (void)hipEventDestroy(e);
    if (E.d_tables) (void)hipFree(E.d_tables);
    if (E.d_small) (void)hipFree(E.d_small);
    if (E.d_nraw) (void)hipFree(E.d_nraw);
    if (E.h_small) (void)hipHostFree(E.h_small);
    if (E.h_nraw) (void)hipHostFree(E.h_nraw);
    for (auto& e : E.ev)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : E.tev)
        if (e) (void)hipEventDestroy(e);
    if (E.s && !E.s_external) (void)hipStreamDestroy(E.s);
    if (E.s_mt) (void)hipStreamDestroy(E.s_mt);
    delete h;
}

int sb_debug_successors(int32_t device, const uint64_t* lo, const uint64_t* hi, int64_t n, uint64_t* out_lo,
                        uint64_t* out_hi, uint64_t* out_key, int32_t* out_count) {
    if (!g_tables_ready) {
        set_error("call sb_init_tables first");
        return SB_ERR_NOTABLES;
    }
    if (n <= 0) return SB_OK;
    return guarded([&]() {
        SB_HIP(hipSetDevice(device));
        Tables* dt = upload_tables(0);
        uint64_t *dlo, *dhi, *olo, *ohi, *okey;
        int32_t* ocnt;
        const size_t m = (size_t)n * MAX_CHILDREN;
        SB_HIP(hipMalloc((void**)&dlo, n * 8));
        SB_HIP(hipMalloc((void**)&dhi, n * 8));
        SB_HIP(hipMalloc((void**)&olo, m * 8));
        SB_HIP(hipMalloc((void**)&ohi, m * 8));
        SB_HIP(hipMalloc((void**)&okey, m * 8));
        SB_HIP(hipMalloc((void**)&ocnt, n * 4));
        SB_HIP(hipMemcpy(dlo, lo, n * 8, hipMemcpyHostToDevice));
        SB_HIP(hipMemcpy(dhi, hi, n * 8, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_debug_succ, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, 0, dt, dlo, dhi, n, olo, ohi, okey, ocnt);
        SB_HIP(hipGetLastError());
        SB_HIP(hipMemcpy(out_lo, olo, m * 8, hipMemcpyDeviceToHost));
        SB_HIP(hipMemcpy(out_hi, ohi, m * 8, hipMemcpyDeviceToHost));
        SB_HIP(hipMemcpy(out_key, okey, m * 8, hipMemcpyDeviceToHost));
        SB_HIP(hipMemcpy(out_count, ocnt, n * 4, hipMemcpyDeviceToHost));
        for (void* p : {(void*)dlo, (void*)dhi, (void*)olo, (void*)ohi, (void*)okey, (void*)ocnt, (void*)dt}) SB_HIP(hipFree(p));
        return SB_OK;
    });
}

int sb_debug_mt_words(int32_t device, const uint32_t* mt_state625, int64_t n, uint32_t* out) {
    return sb_debug_mt_words_cfg(device, mt_state625, n, 256, 1, out);
}

int sb_debug_mt_words_cfg(int32_t device, const uint32_t* mt_state625, int64_t n, int32_t producers,
                          int64_t twists, uint32_t* out) {
    if (!mt_state625 || !out || n < 0 || producers < 1 || twists < 1) return SB_ERR_ARG;
    return guarded([&]() {
        SB_HIP(hipSetDevice(device));
        mt_debug_words(mt_state625, n, producers, twists, out);
        return SB_OK;
    });
}

int sb_debug_scores(int32_t device, int32_t heuristic, const uint64_t* lo, const uint64_t* hi, const int32_t* k,
                    int64_t n, double* out) {
    if (!g_tables_ready) {
        set_error("call sb_init_tables first");
        return SB_ERR_NOTABLES;
    }
    if (n <= 0) return SB_OK;
    for (int64_t i = 0; i < n; i++)
        if (k[i] < 1 || k[i] > 100) {
            set_error("sb_debug_scores: k out of 1..100");
            return SB_ERR_ARG;
        }
    return guarded([&]() {
        SB_HIP(hipSetDevice(device));
        Tables* dt = upload_tables(0);
        uint64_t *dlo, *dhi;
        int32_t* dk;
        double* dout;
        SB_HIP(hipMalloc((void**)&dlo, n * 8));
        SB_HIP(hipMalloc((void**)&dhi, n * 8));
        SB_HIP(hipMalloc((void**)&dk, n * 4));
        SB_HIP(hipMalloc((void**)&dout, n * 8));
        SB_HIP(hipMemcpy(dlo, lo, n * 8, hipMemcpyHostToDevice));
        SB_HIP(hipMemcpy(dhi, hi, n * 8, hipMemcpyHostToDevice));
        SB_HIP(hipMemcpy(dk, k, n * 4, hipMemcpyHostToDevice));
        dim3 g((unsigned)((n + 255) / 256));
        switch (heuristic) {
            case 1: hipLaunchKernelGGL(k_debug_scores<1>, g, dim3(256), 0, 0, dt, dlo, dhi, dk, n, dout); break;
            case 2: hipLaunchKernelGGL(k_debug_scores<2>, g, dim3(256), 0, 0, dt, dlo, dhi, dk, n, dout); break;
            case 3: hipLaunchKernelGGL(k_debug_scores<3>, g, dim3(256), 0, 0, dt, dlo, dhi, dk, n, dout); break;
            default: hipLaunchKernelGGL(k_debug_scores<0>, g, dim3(256), 0, 0, dt, dlo, dhi, dk, n, dout); break;
        }
        SB_HIP(hipGetLastError());
        SB_HIP(hipMemcpy(out, dout, n * 8, hipMemcpyDeviceToHost));
        for (void* p : {(void*)dlo, (void*)dhi, (void*)dk, (void*)dout, (void*)dt}) SB_HIP(hipFree(p));
        return SB_OK;
    });
}

int sb_debug_topk(int32_t device, const uint64_t* keys, int64_t n, int64_t keep, uint32_t* out_idx) {
    if (!keys || !out_idx || n < 0 || keep < 0) return SB_ERR_ARG;
    if (n == 0 || keep == 0) return SB_OK;
    return guarded([&]() {
        SB_HIP(hipSetDevice(device));
        hipStream_t st;
        SB_HIP(hipStreamCreate(&st));
        uint64_t* dk;
        uint32_t* di;
        const int64_t m = std::min(n, keep);
        SB_HIP(hipMalloc((void**)&dk, n * 8));
        SB_HIP(hipMalloc((void**)&di, m * 4));
        SB_HIP(hipMemcpy(dk, keys, n * 8, hipMemcpyHostToDevice));
        TopkScratch s;
        topk_stable_desc(dk, n, keep, di, s, st);
        SB_HIP(hipStreamSynchronize(st));
        SB_HIP(hipMemcpy(out_idx, di, m * 4, hipMemcpyDeviceToHost));
        SB_HIP(hipFree(dk));
        SB_HIP(hipFree(di));
        s.release();
        SB_HIP(hipStreamDestroy(st));
        return SB_OK;
    });
}

// the host-scored prune of sb_prune on its own: f64 scores -> order keys (k_order_keys) -> full-key top-k
int sb_debug_topk_scores(int32_t device, const double* scores, int64_t n, int64_t keep, uint32_t* out_idx) {
    if (!scores || !out_idx || n < 0 || keep < 0) return SB_ERR_ARG;
    if (n == 0 || keep == 0) return SB_OK;
    return guarded([&]() {
        SB_HIP(hipSetDevice(device));
        hipStream_t st;
        SB_HIP(hipStreamCreate(&st));
        uint64_t* dk;
        uint32_t* di;
        uint32_t* derr;
        const int64_t m = std::min(n, keep);
        SB_HIP(hipMalloc((void**)&dk, n * 8));
        SB_HIP(hipMalloc((void**)&di, m * 4));
        SB_HIP(hipMalloc((void**)&derr, 4));
        SB_HIP(hipMemset(derr, 0, 4));
        SB_HIP(hipMemcpy(dk, scores, n * 8, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_order_keys, dim3(grid_cap(n, 256, 8192)), dim3(256), 0, st, dk, n, derr);
        TopkScratch s;
        topk_stable_desc(dk, n, keep, di, s, st, false, derr, false, nullptr, /*full_key=*/true);
        SB_HIP(hipStreamSynchronize(st));
        uint32_t err = 0;
        SB_HIP(hipMemcpy(&err, derr, 4, hipMemcpyDeviceToHost));
        SB_HIP(hipMemcpy(out_idx, di, m * 4, hipMemcpyDeviceToHost));
        SB_HIP(hipFree(dk));
        SB_HIP(hipFree(di));
        SB_HIP(hipFree(derr));
        s.release();
        SB_HIP(hipStreamDestroy(st));
        if (err) throw HipError{hipErrorLaunchFailure, "sb_debug_topk_scores: device error word " + std::to_string(err)};
        return SB_OK;
    });
}

}  // extern "C"

#include "sb_dist.inc"
#include "sb_realistic.inc"
