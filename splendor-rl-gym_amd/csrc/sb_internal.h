// sb_internal.h — host-side declarations shared by the engine's translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace sb {

// ---- error plumbing: every HIP call in the library goes through SB_HIP ----
void set_error(const std::string& msg);
struct HipError {
    hipError_t code;
    std::string what;
};
#define SB_HIP(call)                                                                                        \
    do {                                                                                                    \
        hipError_t _e = (call);                                                                             \
        if (_e != hipSuccess)                                                                               \
            throw ::sb::HipError{_e, std::string(#call) + " -> " + hipGetErrorString(_e) + " @" __FILE__ ":" + \
                                         std::to_string(__LINE__)};                                         \
    } while (0)

// ---- device allocation with a diagnosable failure: the message names what was being allocated, the bytes
// requested and the HBM free at that moment (an OOM in one rank of eight sharing a GPU must be
// readable from one run).  SB_DEBUG_HBM_LIMIT=<bytes> (tests) fails every single request above that size the same way.
std::string oom_message(const char* what, size_t bytes, hipError_t code);
void dev_malloc(void** p, size_t bytes, const char* what);

// ---- device buffer helper (grow-only) ----
template <class T>
struct DBuf {
    T* p = nullptr;
    size_t cap = 0;
    void ensure(size_t n, const char* what = "engine buffer") {
        if (n <= cap) return;
        if (p) SB_HIP(hipFree(p));
        p = nullptr;
        cap = 0;
        size_t c = n < 1024 ? 1024 : n + n / 2;   // slack: a growing size reallocates rarely
        dev_malloc((void**)&p, c * sizeof(T), what);
        cap = c;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Bump allocator for the per-turn beams (kept for path reconstruction until sb_destroy): no
// hipMalloc on the step path — hipMalloc/hipFree can serialise against in-flight work.
struct Arena {
    std::vector<void*> blocks;
    char* cur = nullptr;
    size_t left = 0;
    size_t block_bytes = (size_t)256 << 20;
    void reserve(size_t bytes) {   // make sure the next `bytes` come from one block already allocated
        if (bytes <= left) return;
        const size_t b = bytes > block_bytes ? bytes : block_bytes;
        void* p = nullptr;
        dev_malloc(&p, b, "turn arena block");
        blocks.push_back(p);
        cur = (char*)p;
        left = b;
    }
    void* alloc(size_t bytes) {
        bytes = (bytes + 255) & ~(size_t)255;
        if (bytes > left) {
            const size_t b = bytes > block_bytes ? bytes : block_bytes;
            void* p = nullptr;
            dev_malloc(&p, b, "turn arena block");
            blocks.push_back(p);
            cur = (char*)p;
            left = b;
        }
        void* r = cur;
        cur += bytes;
        left -= bytes;
        return r;
    }
    void release() {
        for (void* p : blocks) (void)hipFree(p);
        blocks.clear();
        cur = nullptr;
        left = 0;
    }
};

// ---- scan (sb_scan.hip) ----
struct ScanScratch {
    DBuf<uint32_t> tiles;
};
constexpr int SCAN_TILE = 4096;
// single-workgroup exclusive scan of a short array in place (tile sums); *total_dev gets the sum
void scan_tiles_inplace(uint32_t* tiles, int64_t ntiles, uint32_t* total_dev, hipStream_t st);
// exclusive scan of n u32 values (in may equal out); *total_dev (u32, device) receives the sum
void scan_exclusive_u32(const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total_dev, ScanScratch& s,
                        hipStream_t st);
// the same when the caller's kernel already wrote the SCAN_TILE tile sums into s.tiles (n > 0)
void scan_exclusive_u32_sums(const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total_dev, ScanScratch& s,
                             hipStream_t st);

// ---- stable top-k (sb_sort.hip) ----
struct TopkScratch {
    DBuf<uint64_t> k0, k1;          // keys ping-pong
    DBuf<uint32_t> v0, v1;          // payload ping-pong
    DBuf<uint64_t> ck;              // select candidates (keys)
    DBuf<uint32_t> ci;              // select candidates (indices)
    DBuf<uint64_t> os;              // LSD sort: digit histograms, tickets, look-back granules
    DBuf<uint32_t> tile_a, tile_b;  // partition counts
    DBuf<uint64_t> small;           // select state + histogram
    DBuf<uint32_t> fx_list;         // sort fix-up: flagged positions
    DBuf<uint32_t> fx_mark;         // sort fix-up: run claims (epoch stamps)
    DBuf<uint32_t> fx_list2;        // sort fix-up: runs with too many distinct keys for a wave (k_fx_fix)
    DBuf<uint32_t> os_tcnt;         // LSD sort (two-level passes): per-digit tile counts, then their offsets
    DBuf<uint32_t> osh_part;        // sort digit histograms: one row per k_os_hist block (two-stage flush)
    DBuf<uint32_t> tkh_part;        // select histograms: one row per k_tk_hist block (two-stage flush)
    DBuf<uint64_t> sk;              // select: staged first-partition keys (one TK_TILE region per tile)
    DBuf<uint32_t> si;              // select: staged first-partition payloads
    uint32_t fx_epoch = 0;
    uint32_t os_epoch = 0;          // LSD sort look-back granule epochs (SB_OS_EPOCH)
    uint64_t* h_nc = nullptr;       // pinned: the last select's candidate count (read without a wait: nc_ev)
    hipEvent_t nc_ev = nullptr;
    bool nc_pending = false;
    void release();
};
// Stable descending order of keys[0..n) (ties keep index order), first `keep` indices into out_idx.
// Returns the number written (min(n, keep)).  ms_select/ms_sort get device times if non-null.
// range_ready: the producer of the keys already folded their min/max into the pair returned by
// topk_range_reset (called before it ran on the same stream).  err (device word): bit 4 is set if the
// sort's look-back wait hit its spin bound (reported by check_err_word; never expected).
// fused: the producer also added every key to the first-pass histogram (topk_fused_hist/_base; keys
// are IEEE images of positive doubles), which replaces the generic first select pass when usable.
// payload: out_idx receives payload[i] of the kept positions i instead of i (next_queue's 4-byte
// descriptors: the gather then reads none of them at a random line).
// full_key: sort on every varying key bit (up to 8 passes) instead of the top 40 + the exact fix-up, whose
// runs of equal prefixes hold at most FX_LIST distinct keys (error bit 32 beyond): keys of arbitrary
// distribution (host-scored heuristics, sb_prune) take this path.
int64_t topk_stable_desc(const uint64_t* keys, int64_t n, int64_t keep, uint32_t* out_idx, TopkScratch& s,
                         hipStream_t st, bool range_ready = false, uint32_t* err = nullptr, bool fused = false,
                         const uint32_t* payload = nullptr, bool full_key = false);
// fill_ff (optional): fill_n u32 words set to ~0 by the same launch (the gather's per-pts first-rank table)
// fused first select pass (the producer's histogram): bins of key >> SB_SEL_FSH over a 2048-bin window.  47 (default):
// 1/32-binade bins around the threshold two selects back, then a second pass over all keys before the partition.  42 (A/B,
// rejected): 1/1024-binade bins around the previous threshold and no second pass — but C3's scores are so
// discrete (≈115k distinct values in the kept 4M) that the threshold's bin still holds millions of keys, and
// copying them as candidates costs more than the pass it saves (select 0.578 -> 0.578-0.588 ms; stage 89 -> 130-143
// us, unstage 30 -> 47-76 us: profiles/r4/s2/fsh_ab.txt)
#ifndef SB_SEL_FSH
#define SB_SEL_FSH 47
#endif
unsigned long long* topk_range_reset(TopkScratch& s, hipStream_t st, bool fused = false, bool off_window = false,
                                     uint32_t* fill_ff = nullptr, int fill_n = 256);
unsigned long long* topk_fused_hist(TopkScratch& s);
const uint64_t* topk_fused_base(TopkScratch& s);
// size the scratch for n keys and keep kept (avoids allocation on the step path)
void topk_reserve(TopkScratch& s, int64_t n, int64_t keep);

// ---- MT19937 noise stream (sb_mt.hip) ----
struct HostMT {
    uint32_t mt[624];
    int idx;
    uint32_t next();
};
// P jump-ahead producers; chunk c covers stream words [c*P*L, (c+1)*P*L), L = twists*624
struct MTProducers {
    int P = 0;
    int64_t twists = 0;
    int64_t chunk = 0;
    uint32_t* d_win = nullptr;     // P x 624 segment-start windows
    uint32_t* d_poly = nullptr;    // jump polynomials (doubling tree + chunk stride)
    uint32_t* chunk_poly = nullptr;
    uint32_t* stride_poly = nullptr;   // sharded: jump world * P * L (to this rank's next chunk)
    void init(const uint32_t origin[624], int P, int64_t twists, hipStream_t st);
    void gen_chunk(uint32_t* out, hipStream_t st);   // P*L tempered words
    void gen_chunk_accepted(uint8_t* stage, uint32_t* counts, hipStream_t st);   // accepted values per producer
    void release();
};
struct NoiseStream {
    MTProducers prod;
    DBuf<uint32_t> raw;            // raw tempered words (host-emitted lead block)
    DBuf<uint8_t> stage;           // per-producer accepted values of one chunk
    DBuf<uint8_t> ring;            // accepted randint values 1..100
    uint64_t ring_mask = 0;
    uint64_t produced = 0;         // accepted values written so far (host mirror, valid after sync)
    uint64_t consumed = 0;         // accepted values consumed by emitted states
    uint32_t* d_total = nullptr;   // device counter of accepted values from the last compaction
    uint32_t* h_total = nullptr;   // pinned mirror
    HostMT initial;                // state at sb_create (for sb_get_mt_state replay)
    HostMT replay;                 // replay cursor
    uint64_t replay_draws = 0;
    ScanScratch scan;
    hipEvent_t ev_ready = nullptr;
    bool pending = false;
    bool sharded = false;          // world > 1: values come from noise_shard_fill
    DBuf<uint64_t> segtab;         // sharded fill: first accepted index of every window
    int ck = 1;                    // sharded: twists per checkpoint (sub-segment)
    int nslots = 4;                // sharded: chunk slots of checkpoint windows
    DBuf<uint32_t> ckpt;           // sharded: nslots x P x (twists / ck) windows of 624 words
    hipEvent_t ev_main = nullptr;  // sharded: main-stream point a new chunk waits for (slot reuse)
};
void noise_init(NoiseStream& ns, const uint32_t* state625, uint64_t ring_cap_pow2, int64_t twists, hipStream_t st);
uint64_t noise_chunk_words(const NoiseStream& ns);
// Launch one chunk of generation + compaction on stream st (asynchronous; no-op if one is pending
// or the ring lacks room).
void noise_generate_async(NoiseStream& ns, hipStream_t st);
// Block until the ring holds >= need unconsumed values (generating more if necessary).
void noise_ensure(NoiseStream& ns, uint64_t need, hipStream_t st);
void noise_free(NoiseStream& ns);
// Sharded stream (world > 1): chunks c = rank (mod world) are this rank's.  setup jumps the producers
// to chunk `rank`; chunk() copies the P producer windows of the next owned chunk to d_win_out and
// writes its per-producer accepted counts to d_counts (asynchronously on st); fill() regenerates
// producer segments into the ring.
void noise_shard_setup(NoiseStream& ns, int rank, int world, hipStream_t st);
// next owned chunk into checkpoint slot `slot`: per sub-segment (ck twists) accepted counts to d_counts
// (P x S, producer-major) and the window at its start to the slot; on st_mt after st_main's pending work
void noise_shard_chunk(NoiseStream& ns, int slot, uint32_t* d_counts, hipStream_t st_main, hipStream_t st_mt);
// gather checkpoint windows (index = slot * P * S + sub-segment) into d_out (m x 624)
void noise_shard_pack(NoiseStream& ns, int m, const int64_t* h_idx, uint32_t* d_out, hipStream_t st);
// regenerate m sub-segments from contiguous windows; accepted values with global index in [a, b) go to the ring
struct NoiseRanges {   // sharded fill: accepted-draw index ranges [a, b) placed at ring positions dst + (idx - a)
    uint64_t a[16], b[16], dst[16];
    int n;
};
void noise_shard_fill(NoiseStream& ns, int m, const uint32_t* d_wins, const uint64_t* h_acc0, const NoiseRanges& R,
                      hipStream_t st);
void noise_mt_state(NoiseStream& ns, uint32_t* out625);
// debug: raw device words from P producers of `twists` twists per segment
void mt_debug_words(const uint32_t* state625, int64_t n, int P, int64_t twists, uint32_t* out);

}  // namespace sb
