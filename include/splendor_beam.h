/*
 * splendor_beam.h — C-ABI of the MI355X Splendor beam-search step engine (libsplendor_beam.so).
 *
 * Drop-in boundary for ONE hot path of IamJasonBian/Splendor-RL-Gym: the per-turn state
 * expansion of State.solve (src/solver.py:390-464) — legal-move enumeration (src/buys.py:13-41,
 * src/gems.py:14-113), gem arithmetic (src/gems.py:116-143, src/solver.py:338-355), trail dedup
 * (src/solver.py:425-450), heuristic scoring (src/solver.py:210-305) and the stable top-k prune
 * to beam_width (src/solver.py:452-456).  The reference has no FFI; its boundary is the Python
 * call surface State.solve / HEURISTICS, which the ctypes host layer
 * (splendor-rl-gym_amd/splendor_amd/) keeps.  Each entry point below names the reference
 * interface it replaces.
 *
 * Conventions: plain C types only; every call returns SB_OK (0) or a negative SB_ERR_* code,
 * with a message from sb_last_error() (thread-local).  No exceptions or callbacks cross the ABI.
 * The library owns all device memory and HIP streams; the caller owns every host buffer.
 * One handle is driven by one host thread; calls block until their results are on the host.
 *
 * Packed speedrun state (two u64 words, also used by oracle/ and the host codec):
 *   lo = owned-card bitmask, cards 0..63
 *   hi = bits 0..25 cards 64..89 | bits 26+3i gems of colour i (0..7) | bits 41..48 pts
 *        | bits 49..63 saved
 * State identity = CPython hash((cards, gems)) as an unsigned 64-bit key (src/solver.py:318).
 */
#ifndef SPLENDOR_BEAM_H
#define SPLENDOR_BEAM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SB_OK 0
#define SB_ERR_ARG -1        /* bad argument / handle */
#define SB_ERR_HIP -2        /* HIP runtime error (message names the call) */
#define SB_ERR_STATE -3      /* call not valid in the handle's state (e.g. path before done) */
#define SB_ERR_CAPACITY -4   /* visited set / buffer capacity exceeded */
#define SB_ERR_NOTABLES -5   /* sb_init_tables not called */

#define SB_HEUR_SIMPLE 0     /* simple_heuristic      src/solver.py:210-215 */
#define SB_HEUR_BALANCED 1   /* balanced_heuristic    src/solver.py:218-249 (also 'competitive', :289-296) */
#define SB_HEUR_AGGRESSIVE 2 /* aggressive_heuristic  src/solver.py:252-262 */
#define SB_HEUR_EFFICIENCY 3 /* efficiency_heuristic  src/solver.py:265-286 */
#define SB_HEUR_HOST 15      /* any other HEURISTICS callable (HEURISTICS.md:204-229, src/solver.py:299-305,429):
                                the caller scores next_queue itself (sb_read_next + sb_prune) */

#define SB_N_POW_EXP 11      /* exponents {0.3,0.4,0.5,0.6,0.7,0.8,1.2,2.0,2.5,2.8,3.2} */
#define SB_POW_BASES 256     /* integer bases 0..255 */

typedef struct sb_engine sb_engine;

typedef struct {
    int32_t goal_pts;          /* State.solve(goal_pts)                src/solver.py:392 */
    int32_t use_heuristic;     /* False = pure BFS (no noise, no prune) src/solver.py:394,452-456 */
    int32_t heuristic;         /* SB_HEUR_*; unknown names map to simple on the host (:429) */
    int32_t device;            /* HIP device ordinal */
    int64_t beam_width;        /* State.solve(beam_width)              src/solver.py:396 */
    int32_t visited_log2;      /* log2 initial visited-set capacity (entries, 10..34); 0 = auto from beam_width and
                                  free HBM; grown between turns either way (sb_visited_capacity) */
    int32_t flags;             /* bit 0: collect per-kernel timings; bit 1: sharded (sbd_*) mode even at world_size 1;
                                  bit 2 (test): generic first select pass instead of the one folded into the
                                  emission; bit 3 (test): folded pass with its window forced off the keys
                                  (exercises its fallback); bit 4 (test): grow the visited set at 25% projected
                                  load instead of 60% (exercises rebuilds of large tables); bit 5: sharded record
                                  buffers for 48 raw children per parent instead of the worst case (several
                                  ranks sharing one GPU), overflow fails the step (SB_ERR_CAPACITY); bit 6: reserved (set by
                                  the host when it expands with sbd_expand_parts); bit 7 (test): the key
                                  pass gives every key (with bit 8: every card set) to rank 0 (parts that
                                  send no records; results unchanged); bit 8: card-set ownership of the
                                  sharded trail (sbd_mig_*, world_size > 1); bit 9 (with bit 8): owner
                                  emission (sbd_oe_*); bit 10 (test): the pipelined turn's receive bound starts at
                                  1024 records, so the host grows it (sbd_grow_receive) every turn; bit 11
                                  (world_size > 1, key ownership): global-order claims — the own children become
                                  records to this rank and every record of the turn is claimed in one pass in
                                  global order (sbd_owner_claim_all) */
    /* multi-GPU (config 5): this engine owns global beam ranks [rank_lo, rank_hi) */
    int32_t world_size;        /* 1 for single-GPU */
    int32_t rank;
} sb_config;

typedef struct {
    int64_t n_parents;         /* len(queue) at the start of the step */
    int64_t n_raw;             /* successors generated (State.__iter__ yields) */
    int64_t n_unique;          /* len(next_queue): first occurrences not in trail */
    int64_t n_kept;            /* len(queue) after the prune */
    int32_t done;              /* 1: a goal state was found (or the queue emptied) */
    int32_t turn;              /* turn index the stats belong to */
    int64_t winner_rank;       /* rank of `puzzle` in this turn's queue when done */
    int32_t n_records;         /* max_pts records printed in this turn (src/solver.py:439-442) */
    int32_t record_pts[32];
    int64_t record_rank[32];
    uint64_t noise_draws;      /* randint(1,100) draws consumed so far (= scored states) */
    /* timings (flags bit 0): milliseconds, device-side events around each phase */
    float ms_expand, ms_survive, ms_emit, ms_select, ms_sort, ms_gather, ms_mt, ms_total;
} sb_step_stats;

/* Host-captured exact tables (replace get_deck/get_takes/get_buys and Python's float pow):
 *   deck_rows   90 x 7 int32: cost[5], pt, colour            (src/cardparser.py:17-66, cards.csv)
 *   pow_tables  SB_N_POW_EXP x SB_POW_BASES doubles = float(x) ** e, captured by Python
 *   noise       100 doubles = k * 0.01 for k = 1..100          (src/solver.py:215,247,260,284)
 * The take-pattern table (src/gems.py:14-37) is generated inside the library. */
int sb_init_tables(const int32_t* deck_rows, const double* pow_tables, const double* noise);

/* Replaces State.solve's setup (src/solver.py:425-433): root state + random.getstate().
 * mt_state625 = the 624 MT words + position, exactly as random.getstate()[1]. */
int sb_create(const sb_config* cfg, const uint32_t* mt_state625, uint64_t root_lo, uint64_t root_hi,
              sb_engine** out);

/* One iteration of the `while queue:` loop (src/solver.py:434-457).  The next turn's expansion is
 * launched before returning (it overlaps the caller's work); the stats' device times are filled by
 * sb_turn_times once a turn has completed. */
int sb_step(sb_engine* e, sb_step_stats* out);

/* Host-scored turns (cfg.heuristic == SB_HEUR_HOST, use_heuristic = 1): sb_step runs the goal check, the
 * expansion and the trail dedup, writes next_queue and returns with n_unique set and n_kept = 0 (or done);
 * the caller reads next_queue (sb_read_next: states in next_queue order, the order `sorted` calls its key in,
 * src/solver.py:453), scores every entry with its Python callable and hands the scores to sb_prune, which
 * runs the stable descending top-k (`sorted(..., reverse=True)[:beam_width]`, ties in next_queue order) on
 * the device, writes the next beam and launches the next expansion.  Scores are compared as f64 (-0.0 ==
 * 0.0); a NaN fails the call (SB_ERR_HIP). *n_kept = len(queue) of the next turn.  sb_step is refused
 * (SB_ERR_STATE) while a host-scored turn awaits sb_prune. */
int sb_read_next(sb_engine* e, int64_t start, int64_t n, uint64_t* lo, uint64_t* hi);
int sb_prune(sb_engine* e, const double* scores, int64_t n, int64_t* n_kept);

/* Device phase times (ms) of a completed turn, timing flag set (flags bit 0): expand, count+scan,
 * host gap, emit, top-k, gather, total.  Speedrun handles only; the last 64 turns are kept. */
int sb_turn_times(sb_engine* e, int32_t turn, float* out7);

/* Number of turns stored (turn 0 = root) and the size of one turn's queue. */
int sb_num_turns(sb_engine* e, int32_t* out);
int sb_turn_size(sb_engine* e, int32_t turn, int64_t* out);

/* Copy queue[start:start+n] of a turn to host arrays (any pointer may be NULL).
 * par = rank of the parent in the previous turn (the `trail` link, src/solver.py:449). */
int sb_read_turn(sb_engine* e, int32_t turn, int64_t start, int64_t n, uint64_t* lo, uint64_t* hi,
                 uint32_t* par, uint64_t* key);

/* Root..winner path (src/solver.py:459-464).  *len = number of states written (<= cap). */
int sb_path(sb_engine* e, uint64_t* lo, uint64_t* hi, int32_t cap, int32_t* len);

/* MT19937 state after the draws consumed so far, as random.getstate()[1], so the caller's global
 * `random` ends where the reference's would after solve(). */
int sb_get_mt_state(sb_engine* e, uint32_t* out625);

/* Block until all device work of the handle has finished. */
int sb_sync(sb_engine* e);

/* Lookahead (default on): sb_step launches the next turn's expansion before it returns.  Off: it does
 * not, and the next sb_step launches that expansion itself — a benchmark that times an exact set of
 * turns turns it off for the step before the first timed one and for the last timed one, so the timed
 * region holds the expansions of exactly the turns it counts.  Results do not depend on it. */
int sb_set_lookahead(sb_engine* e, int32_t on);

/* Block until the turns launched so far have finished on the engine stream; the noise generation that
 * runs ahead of need on its own stream (draws for later turns) is not waited for.  sb_sync waits for both. */
int sb_sync_engine(sb_engine* e);

/* Visited-set entries (len(trail)). */
int sb_visited_size(sb_engine* e, uint64_t* out);

/* Visited-set capacity in slots and how often it was rebuilt larger.  The reference's trail is an
 * unbounded dict (src/solver.py:425-426,447-450): before a turn whose worst case (every raw child new)
 * could pass 60% load, the table is rehashed into 2^k times the slots while free HBM allows; results
 * do not depend on the capacity.  Sharded mode: this rank's owner shard. */
int sb_visited_capacity(sb_engine* e, uint64_t* capacity, int32_t* rebuilds);
/* out6 = [slots, rebuilds, rebuilds smaller than the turn's worst case wanted (free HBM ran short), rebuilds wanted and
 * not made, peak load after a turn (keys / slots, ppm), keys] of the visited set (sharded: this rank's owner shard).
 * A shortened or skipped growth raises the load (longer probe chains) without changing a result; the HARD_LOAD (85%)
 * check after a turn is the limit.  SB_DEBUG_VISITED_MAX=<slots> (tests) fails rebuilds above it. */
int sb_visited_stats(sb_engine* e, uint64_t* out6);

void sb_destroy(sb_engine* e);
const char* sb_last_error(void);
int sb_version(void);
/* Identity of the sources the library was built from (sha256 prefix over csrc/ + this header, passed
 * by the build); the ctypes loader compares it with the tree and refuses a stale library. */
const char* sb_build_id(void);

/* ---- kernel-level entry points for parity tests (same device code as sb_step) ---- */
/* Ordered successors of n parents, stride 192 per parent: out_count[i] children for parent i. */
int sb_debug_successors(int32_t device, const uint64_t* lo, const uint64_t* hi, int64_t n,
                        uint64_t* out_lo, uint64_t* out_hi, uint64_t* out_key, int32_t* out_count);
/* n tempered MT19937 words continuing from mt_state625 (device jump-ahead producers: 256 x 1 twist). */
/* one device allocation through the engine's allocator, then freed: on failure (SB_ERR_CAPACITY when out of memory)
 * sb_last_error names what, the bytes requested and the HBM free, as every engine allocation does;
 * SB_DEBUG_HBM_LIMIT=<bytes> in the environment fails any single request above it (tests) */
int sb_debug_alloc(uint64_t bytes);
int sb_debug_mt_words(int32_t device, const uint32_t* mt_state625, int64_t n, uint32_t* out);
/* same with `producers` (power of two) producers of `twists` twists per segment */
int sb_debug_mt_words_cfg(int32_t device, const uint32_t* mt_state625, int64_t n, int32_t producers,
                          int64_t twists, uint32_t* out);
/* Scores of n states with the given randint values k (1..100). */
int sb_debug_scores(int32_t device, int32_t heuristic, const uint64_t* lo, const uint64_t* hi,
                    const int32_t* k, int64_t n, double* out);
/* Stable descending sort of n u64 keys: out_idx = permutation (ties keep input order), first `keep`. */
int sb_debug_topk(int32_t device, const uint64_t* keys, int64_t n, int64_t keep, uint32_t* out_idx);
/* sb_prune's host-scored prune alone: f64 scores (any sign or spacing) -> stable descending order. */
int sb_debug_topk_scores(int32_t device, const double* scores, int64_t n, int64_t keep, uint32_t* out_idx);
/* Diagnostic (profiles/expand_bench.py): device time (ms, averaged over reps) of the expansion's variants on
 * a single-GPU engine's current queue whose expansion is not launched yet (sb_set_lookahead(e, 0) before
 * the last sb_step), each on a copy of the visited set: out_ms[0] k_expand (one GPU), [1] sharded
 * expansion at world 1, [2] at world 8 (rank 0), [3] world 8 owning no child (every key a record),
 * [4] owner claims of all of [3]'s records, [5] [3] and [4] side by side on two streams, [6] raw count +
 * scan, [7] raw children, [8] the sharded key pass at world 8 (rank 0), [9] its count scan + record move
 * [10..13] timing-only variants of [8] (no own claims; also a stand-in key; also no stores; no claims and no
 * stores), [14] k_keys_a owning nothing beside the owner claims of [3]'s records on a second stream
 * (wall), [15] that k_keys_a alone, [16] one rank's pipelined dedup at world 8 (4 parts: key pass + the claims
 * of the records standing in for what the other ranks send) on two streams (wall), [17] the same on one
 * stream, [18] with the key passes on a high-priority stream and the claims on a low-priority one, [19]
 * the device's stream priority levels (out_ms holds 20 floats).  The engine cannot step after this call. */
int sb_debug_expand_bench(sb_engine* e, int32_t reps, float* out_ms);

/* ---- sharded mode (cfg.world_size > 1 or flags bit 1): per-rank step primitives; the exchanges
 * between them are the caller's (splendor_amd/dist.py: torch.distributed / RCCL).  Device pointers
 * are caller-owned buffers on the engine's device.  The engine's work is ordered on its stream
 * (sbd_set_stream); calls that return host values wait for it. ---- */
/* local first rank per pts of this rank's queue slice (0xFFFFFFFF = none); after sbd_expand_launch it
 * waits only for the table's copy, which was enqueued ahead of the expansion */
int sbd_goal_table(sb_engine* e, uint32_t* first256);
/* expand the local slice, in two calls.  sbd_expand_launch enqueues the expansion and returns without
 * waiting (the caller launches it as soon as the slice exists, before its goal check): the successors
 * this rank owns (owner = fmix64(key) >> 40 mod world) are claimed in its shard of the visited set, every
 * other successor becomes a record (key).  sbd_expand_counts waits for it and stably partitions the
 * records by owner, cut into nchunk (<= 16) exchange chunks of whole 4096-record tiles:
 * chunk_owner_counts[nchunk][world] = records per chunk and owner, *n_raw = successors generated. */
int sbd_expand_launch(sb_engine* e, int32_t world);
int sbd_expand_counts(sb_engine* e, int32_t nchunk, int64_t* chunk_owner_counts, int64_t* n_raw);
/* Pipelined expansion for world > 1 (sb_keypass.inc): the slice's successors in nparts (<= 16) exchange parts
 * of consecutive parents, all enqueued without a host wait.  Each part: successors hashed, the ones this rank
 * owns claimed in its shard, every other one ranked among its owner's records; a per-part event.  n_global =
 * the turn's parents over all ranks (bounds what this rank can receive).  The raw count is read with
 * sbd_raw_total after the caller's next wait.  Then per part: sbd_part_counts waits for it and gives its
 * records per owner (and the answers this rank may receive this turn, the bound for sbd_owner_begin);
 * sbd_part_pack writes them to the caller's buffer in owner groups, (parent, ordinal) order within each, on
 * the claim stream; send_base = the part's first index in the turn's concatenated send buffers (the layout
 * the answers must come back in for sbd_apply).  Received records claim with answer indices in arrival
 * order (sbd_owner_claim, on the claim stream, beside the later parts' kernels); sbd_owner_total sets the
 * turn's received count before sbd_owner_finish. */
/* bounds (nullable): nparts + 1 local parent indices, part j = parents [bounds[j], bounds[j+1]) — block-cyclic slices,
 * where part j of rank r is block j * world + r of the global queue; null: parts of equal 64-parent chunk counts */
int sbd_expand_parts(sb_engine* e, int32_t world, int32_t nparts, int64_t n_global, const int64_t* bounds);
int sbd_part_counts(sb_engine* e, int32_t part, int64_t* owner_counts, int64_t* recv_capacity);
int sbd_part_pack(sb_engine* e, int32_t part, uint64_t* d_key, int64_t send_base);
/* global-order claims (flags bit 11): sbd_expand_parts packs every part right behind its key pass into the engine's
 * send buffer (part j's owner groups at its first raw slot = the earlier parts' records); sbd_part_pack then only
 * registers send_base (d_key must be null) and the caller sends views of *d_ptr (*cap u64, valid until the next
 * expansion).  Claim segments may read this rank's own records there (p_start with bit 63 set). */
int sbd_send_buffer(sb_engine* e, void** d_ptr, int64_t* cap);
int sbd_set_claim_stream(sb_engine* e, void* stream);
int sbd_owner_total(sb_engine* e, int64_t n_total);
/* the turn's received records will exceed the receive bound sbd_part_counts reported (an estimate from the raw
 * ratio so far): drain this rank's streams and grow the lost bits (and the card-set answer tags) to hold n_needed,
 * contents kept; *new_cap = the new bound.  The caller grows its answer buffer the same way. */
int sbd_grow_receive(sb_engine* e, int64_t n_needed, int64_t* new_cap);
/* world 1 (no records, no exchange to size): go on without waiting for the expansion; *n_raw is read by
 * sbd_raw_total after the caller's next wait on the engine stream (sbd_apply's count). */
int sbd_expand_defer(sb_engine* e);
int sbd_raw_total(sb_engine* e, int64_t* n_raw);
/* the record keys grouped by owner, (parent, ordinal) order inside a group (d_tag unused: tags are
 * implicit in the order) */
int sbd_pack(sb_engine* e, uint64_t* d_key, uint64_t* d_tag);
/* owner side, per turn: begin(n_total records this owner receives; src_base[q] = answer index of source
 * q's first record, nsrc = world), one claim per received chunk (in any order: tags carry the global
 * order), finish.  A chunk holds nseg source segments: source q's records at [seg_start[q],
 * seg_start[q+1]) (seg_start[0] = 0), answer indices seg_base[q].. (source rank major, then parent
 * order).  d_ret[answer index] = 1 for a first occurrence, final after sbd_owner_finish.  The children a
 * rank owns itself never become records: sbd_expand claims them in its shard. */
int sbd_owner_begin(sb_engine* e, int64_t n_total, int32_t nsrc, const int64_t* src_base);
int sbd_owner_claim(sb_engine* e, const uint64_t* d_key, int64_t n, int32_t nseg, const int64_t* seg_start,
                    const int64_t* seg_base, uint8_t* d_ret);
int sbd_owner_finish(sb_engine* e, uint8_t* d_ret);
/* global-order claims (flags bit 11): after every part has arrived, the turn's n_total records in one pass, in
 * virtual (source rank, part, record) order — the global (parent rank, ordinal) order; segment k = virtual records
 * [v_start[k], v_start[k+1]) (the last to n_total) found at d_key + p_start[k].  d_ret[v] = 1 for a claim that inserted
 * or took its key — NOT final in this mode: a record displaced by a later claim keeps 1 and only its lost bit (engine
 * state) says so.  The answers are final only as packed by sbd_pack_bits_segs, which folds the lost bits in;
 * sbd_owner_finish does nothing here and sbd_pack_bits refuses the mode (SB_ERR_STATE).  The own children are records
 * to this rank itself (sbd_part_counts / sbd_part_pack include them). */
int sbd_owner_claim_all(sb_engine* e, const uint64_t* d_key, int64_t n_total, int32_t nseg, const int64_t* v_start,
                        const int64_t* p_start, uint8_t* d_ret);
/* global-order claims of one exchange part as soon as it has arrived (block-cyclic slices, or world 1: part j of every
 * source is one contiguous range of the global order, after every earlier part): virtual records [v_begin, v_end) in
 * nseg <= 64 segments (v_start[0] = v_begin ascending, record v at d_key + p_start[k] + v - v_start[k]), tag turn | v,
 * d_ret[v]; on the claim stream, after the caller's wait for the part's transfer; part < 16 selects its ticket word.
 * d_ret is final for a part once every later part's claims have run (a later record may displace; sbd_pack_bits_segs
 * drops the displaced answers). */
int sbd_owner_claim_part(sb_engine* e, int32_t part, const uint64_t* d_key, int64_t v_begin, int64_t v_end, int32_t nseg,
                         const int64_t* v_start, const int64_t* p_start, uint8_t* d_ret);
/* answers over the wire as bits: dst[i] = bit k set iff src[8i + k] != 0 (n bytes -> ceil(n/8));
 * unpack is the inverse (n answer bytes from ceil(n/8) packed bytes).  Both on the engine stream. */
int sbd_pack_bits(sb_engine* e, const uint8_t* d_src, int64_t n, uint8_t* d_dst);
int sbd_unpack_bits(sb_engine* e, const uint8_t* d_src, int64_t n, uint8_t* d_dst);
/* the same over nseg segments in one launch (device bases + host tables of offsets; len = answer bytes):
 * pack: bytes d_src[src_off[s], + len[s]) -> bits d_dst[dst_off[s], + ceil(len[s]/8)); unpack the inverse. */
int sbd_pack_bits_segs(sb_engine* e, const uint8_t* d_src, int32_t nseg, const int64_t* src_off, const int64_t* len,
                       uint8_t* d_dst, const int64_t* dst_off);
int sbd_unpack_bits_segs(sb_engine* e, const uint8_t* d_src, int32_t nseg, const int64_t* src_off, const int64_t* len,
                         uint8_t* d_dst, const int64_t* dst_off);
/* apply the answers (in pack order): this rank's next_queue entries as an int64 at n_unique_dev (device),
 * without waiting (the caller all-gathers it on the engine stream); sbd_apply_finish(that value) then
 * checks the step's error word and updates the host state. */
int sbd_apply(sb_engine* e, const uint8_t* d_back, void* n_unique_dev);
int sbd_apply_finish(sb_engine* e, int64_t n_unique_local);
/* states + scores of the local survivors; next_queue positions k_off.., n_total draws consumed */
int sbd_emit(sb_engine* e, uint64_t k_off, uint64_t n_total, int64_t goff);
/* Sharded noise stream (heuristic, sharded mode): rank r generates MT19937 chunks c = r (mod world),
 * each P producer segments of `twists` twists, in count-only mode with a checkpoint every ck twists.
 * sbd_noise_info: [P, twists, accepted values in the lead block, consumed, ck, S = twists/ck sub-segments
 * per producer, checkpoint slots, 0].  sbd_noise_chunk: the rank's next owned chunk into checkpoint slot
 * `slot` (windows kept on this device) and its accepted count per sub-segment (P x S u32, producer-major,
 * device buffer counts_out), launched asynchronously after the stream's earlier work (sbd_noise_sync
 * waits).  sbd_noise_pack: copy m checkpoint windows (index = slot * P * S + sub-segment) into wins_out
 * (m x 624 u32) for the all_to_all to the ranks that consume them.  sbd_noise_fill: regenerate m
 * sub-segments from contiguous windows (acc0 = global index of each one's first accepted draw) and keep
 * the accepted values with global index in [a, b) for this rank's emission. */
/* Run the engine's step work on the caller's stream (e.g. torch.cuda.current_stream(), which the RCCL
 * collectives use): exchanges and kernels are then ordered without host synchronisation. */
int sbd_set_stream(sb_engine* e, void* stream);

int sbd_noise_info(sb_engine* e, uint64_t* out8);
int sbd_noise_chunk(sb_engine* e, int32_t slot, void* counts_out);          /* device buffer; asynchronous */
int sbd_noise_sync(sb_engine* e);                                          /* wait for sbd_noise_chunk */
int sbd_noise_pack(sb_engine* e, int32_t m, const int64_t* idx, void* wins_out);
int sbd_noise_fill(sb_engine* e, int32_t m, const void* wins, const uint64_t* acc0, uint64_t a, uint64_t b);
/* block-cyclic slices: the accepted draws of nr <= 16 ranges [a[k], b[k]) (this rank's blocks of the next_queue), range k
 * kept at ring position dst[k] + (index - a[k]) (the emission reads local position k at consumed + k_off + k) */
int sbd_noise_fill_ranges(sb_engine* e, int32_t m, const void* wins, const uint64_t* acc0, int32_t nr, const uint64_t* a,
                          const uint64_t* b, const uint64_t* dst);

/* Joint select on the device (dist.py _multiselect), no host round trip: sbd_key_range writes this
 * rank's score-key range of the turn to range_dev as two int64 for one all_reduce(MIN) by the caller
 * (kmin ^ 2^63, ~(kmax ^ 2^63)); sbd_sel_begin = select state for npos (<= 64) positions (1-based ranks
 * in score-descending order) below the bits common to the reduced range; per pass: sbd_sel_hist
 * (npos x 1024 int64 buffer: a histogram of the next digit — 10 bits while at most 16 prefixes are live, else 8 —
 * per distinct prefix into hist_dev, over the keys
 * (src 0) or the candidates (src 1); hist_dev must be zero on entry: fresh, or as the previous
 * sbd_sel_pick left it), an all_reduce(SUM) of hist_dev by the caller on the same stream,
 * sbd_sel_pick; passes after the last digit are no-ops, so the caller runs a fixed 7 (ceil(64/10)), 8 when
 * npos > 16 (8-bit digits).
 * After the first pass sbd_sel_compact keeps the keys of the chosen buckets as candidates.
 * sbd_sel_eq: count of keys equal to position 0's key (int64 at eq_dev) for the all_gather of the
 * keep boundary's ties. */
int sbd_key_range(sb_engine* e, void* range_dev);
int sbd_sel_begin(sb_engine* e, int32_t npos, const int64_t* positions, const void* range_dev);
/* the same with positions nexact.. as block boundaries (block-cyclic slices): each stops refining once its bucket holds at
 * most fmax keys over all ranks — its boundary is then the bucket's lowest key (a block ends between scores, any
 * boundary keeps the global order) — so the later passes resolve the keep boundary alone */
int sbd_sel_begin_approx(sb_engine* e, int32_t npos, const int64_t* positions, const void* range_dev, int32_t nexact,
                         int64_t fmax);
int sbd_sel_hist(sb_engine* e, int32_t src, void* hist_dev);
int sbd_sel_pick(sb_engine* e, void* hist_dev);   /* also clears hist_dev for the next pass */
int sbd_sel_compact(sb_engine* e);
int sbd_sel_eq(sb_engine* e, void* eq_dev);
/* kept = key > T or (key == T and global tie index < its position) [if has_top; T = position 0's key,
 * eq_all_dev = every rank's tie count]; destination range = #{j : key < split_j} (splits = the next
 * nsplit positions' keys); dest_counts_dev = int64[world] records per destination, on the device (no wait) */
int sbd_partition(sb_engine* e, int32_t has_top, const void* eq_all_dev, int32_t rank, int32_t nsplit, int32_t world,
                  void* dest_counts_dev);
int sbd_partition_bfs(sb_engine* e, uint64_t k_off, uint64_t n_total, int32_t world, void* dest_counts_dev);
/* ---- block-cyclic slices (key ownership, per-part claims): rank r's slice is nblk blocks, block j = global block
 * j * world + r (the next beam dealt so, every rank holds parents of every score level and each exchange part is one
 * range of the global order).  sbd_block_counts (after sbd_apply): survivors per local block (bounds = nblk + 1 local
 * parents) to out_dev (nblk int64).  sbd_sel_eq_blocks: the keep boundary's ties per local block (qstart = nblk + 1
 * local next_queue starts) to eq_dev (nblk int64), and the per-tile offsets the partition reads.
 * sbd_partition_blocks: kept test with this rank's quota from every rank's per-block ties (eq_all_dev: world x nblk,
 * rank-major; ties kept in global (block, rank) order), the select's positions 1 .. world * nblk - 1 as the next
 * beam's block boundaries; digit = destination rank * nblk + its block; dest_counts_dev = world * nblk int64.
 * sbd_dest_subcounts: the kept records per (local block, digit), nblk x D int64 (the receiver's ordering). */
int sbd_block_counts(sb_engine* e, int32_t nblk, const int64_t* bounds, void* out_dev);
int sbd_sel_eq_blocks(sb_engine* e, int32_t nblk, const int64_t* qstart, void* eq_dev);
int sbd_partition_blocks(sb_engine* e, int32_t has_top, const void* eq_all_dev, int32_t rank, int32_t world, int32_t nblk,
                         void* dest_counts_dev, const int64_t* qstart, void* sub_dev);   /* qstart / sub_dev (nullable):
                         sbd_dest_subcounts' counts written on the way (nblk x world * nblk int64) */
int sbd_dest_subcounts(sb_engine* e, int32_t nblk, const int64_t* qstart, int32_t D, void* out_dev);
/* kept records grouped by destination, next_queue order inside a group, one all_to_all buffer of at least the
 * kept count (the local next_queue size always suffices, so it can be enqueued before the counts reach the host).
 * 3 x u64 per record (state lo, state hi, global parent rank | noise draw << 32: the receiver re-scores it);
 * with owner emission (flags bit 9) the third word is global parent rank (25 bits) | draw << 25 | position << 32.
 * rec20 != 0 (without owner emission; the caller's choice, the same on every rank, when every global parent rank of
 * the turn is < 2^25): 20-byte records, five u32 (lo, hi, parent (25 bits) | draw << 25) — 17% fewer bytes on the
 * rebalance's wire */
int sbd_pack_kept(sb_engine* e, uint64_t* d_rec, int32_t rec20);
/* grouped kept records (round 5; key ownership with descriptor emission, global parent ranks < 2^25): a source's
 * kept children of one parent bound for one destination travel as a group — a 20-byte row (parent lo, hi, global
 * rank) and a u16 per child (move | draw << 8 | opens its group << 15).  Destination d's segment of
 * d_buf: its rows, then its child entries padded to 4 bytes (5 G_d + ceil(C_d / 2) u32).  cap_u32 >= 22 bytes per
 * local survivor / 4 (+ 2 world + 2).  d_counts2 (device, 2 x world int64): (C_d, G_d) pairs for the count exchange.
 * Replaces sbd_pack_kept(rec20) on the rebalance's wire; the receiver calls sbd_unpack_kept, then sbd_receive. */
int sbd_pack_kept_grouped(sb_engine* e, uint32_t* d_buf, int64_t cap_u32, int64_t* d_counts2);
/* receive side of the grouped records: nseg source segments of d_buf (host arrays: u32 base, groups, children of
 * each, in source order) expanded into the 20-byte records sbd_receive takes (d_rec: sum(children) x 5 u32, the
 * sources' segments concatenated in order).  Error word bit 256 if a segment's group starts do not match its rows. */
int sbd_unpack_kept(sb_engine* e, const uint32_t* d_buf, int32_t nseg, const int64_t* seg_base, const int64_t* seg_groups,
                    const int64_t* seg_children, uint32_t* d_rec, int32_t nperm, const int64_t* perm, int32_t npm,
                    const int64_t* pmap);
/* (block-cyclic slices: perm = nperm (source child, destination record) run starts — the children of each (source,
 * destination part, source block) run written in (destination part, source block, source) order, the global
 * next_queue order within a block; pmap = npm (sender-side parent number, global rank) run starts, the senders'
 * rank-major numbering mapped to the global queue.  Both nullable with n = 0.) */
/* the new slice: n received records in the form sbd_pack_kept wrote (global next_queue order, or with owner
 * emission source segments in position order), stable-sorted by score if heur */
int sbd_receive(sb_engine* e, const uint64_t* d_rec, int64_t n, int32_t heur);
int sbd_mark_done(sb_engine* e, int64_t winner_rank_local);

/* ---- card-set ownership of the sharded trail (flags bit 8, world_size > 1; csrc/sb_mig.inc).  Replaces the
 * key-owner dedup of one step (src/solver.py:446-450 over the global queue): the trail is sharded by the
 * state's card set, every parent is expanded on the rank owning its card set, so its takes (same cards) are
 * claimed there and only buys to other card-set owners become records; tags carry the global parent rank.
 *   range side:  sbd_mig_launch (after the slice arrives, no wait: owner digits and raw child counts, the
 *                partition counts; the goal table copied ahead), sbd_mig_counts (waits: the slice's parents,
 *                then its raw children, per owner: 2 x world values), sbd_mig_pack (the slice as (lo, hi,
 *                global rank) rows grouped by owner, n x 5 u32), all_to_all by the caller
 *   expand side: sbd_mig_expand (the received rows, source-major, become the expand list; key pass in nparts
 *                parts), then per part sbd_part_counts / sbd_part_pack (12-byte records: three u32, the key and
 *                global parent rank << 7 | move) / all_to_all / sbd_mig_claim on the owner (answer indices
 *                ans_base..), sbd_owner_total + sbd_owner_finish, answer bits back, sbd_mig_apply (the expand
 *                list's survivors as one bit per raw child in move order, source q's parents in a byte-aligned
 *                segment of a zeroed stream), all_to_all back
 *   range side:  sbd_mig_place (the bits into slice order: masks, counts, offsets; unique count on the
 *                device), then sbd_apply_finish / sbd_emit / ... as in the key-owner protocol. */
int sbd_mig_launch(sb_engine* e, int32_t world);
int sbd_mig_counts(sb_engine* e, int64_t* counts);
int sbd_mig_pack(sb_engine* e, int64_t goff, uint32_t* d_rows);
int sbd_mig_expand(sb_engine* e, int32_t world, int32_t nparts, int64_t n_global, const uint32_t* d_rows, int64_t n_exp);
int sbd_mig_claim(sb_engine* e, const uint32_t* d_rec, int64_t m, int64_t ans_base, uint8_t* d_ret);
int sbd_mig_apply(sb_engine* e, const uint8_t* d_back, uint8_t* d_bits, int32_t nseg, const int64_t* seg_start,
                  const int64_t* seg_byte);
int sbd_mig_place(sb_engine* e, const uint8_t* d_bits, int32_t nown, const int64_t* group_start,
                  const int64_t* byte_base, void* n_unique_dev);
/* ---- owner emission (flags bit 9 with bit 8; csrc/sb_oe.inc): the survivors are emitted on the expanding
 * (card-set owner) ranks, whose parents span every score level, so the kept records leave every rank evenly.
 *   range side:  after sbd_mig_place / sbd_apply_finish, sbd_oe_pack (each row's global next_queue offset and
 *                its survivors' noise draws, rows' order; the noise bytes per owner on the host — waits; consumes
 *                the turn's draws), all_to_all of both by the caller
 *   expand side: sbd_mig_apply keeps the expand list's masks; sbd_oe_counts (survivors per source segment, host —
 *                waits), sbd_oe_emit (the emission over the expand list: states, keys, global parent ranks,
 *                next_queue positions), then the joint select as usual; at the keep boundary sbd_oe_ties +
 *                sbd_oe_tie_read (this rank's tie positions; the caller gathers every rank's and takes the
 *                need-th smallest, pstar), sbd_oe_partition (kept: key > T or key == T and position <= pstar) or
 *                sbd_oe_partition_bfs, sbd_pack_kept (the par word carries the position << 32)
 *   receive:     sbd_receive orders the records by (score desc, position asc) */
int sbd_oe_pack(sb_engine* e, uint64_t k_off, uint64_t n_total, uint32_t* d_rgoff, uint8_t* d_rnoise, int32_t nown,
                const int64_t* group_start, int64_t* nb_out);
int sbd_oe_counts(sb_engine* e, int32_t nseg, const int64_t* seg_start, int64_t* out);
int sbd_oe_emit(sb_engine* e, const uint32_t* d_xgoff, const uint8_t* d_xnoise);
int sbd_oe_ties(sb_engine* e, int64_t* count, int64_t* need);
int sbd_oe_tie_read(sb_engine* e, int64_t* pos, int64_t count);
int sbd_oe_partition(sb_engine* e, int32_t has_top, int64_t pstar, int32_t nsplit, int32_t world, void* dest_counts_dev);
int sbd_oe_partition_bfs(sb_engine* e, uint64_t n_total, int32_t world, void* dest_counts_dev);
/* receive side: the next sbd_receive's records arrive as nseg source segments (seg_start[0..nseg], each segment in
 * next_queue position order); sbd_receive merges them by position, then orders them stably by score */
int sbd_oe_segments(sb_engine* e, int32_t nseg, const int64_t* seg_start);
/* test hook: the receive merge alone (host positions, nseg ascending segments; out_idx[rank] = record) */
int sb_debug_oe_merge(int32_t device, const uint32_t* pos, int64_t m, int32_t nseg, const int64_t* seg_start,
                      uint32_t* out_idx);
/* flags bit 0: device time (ms) of the last pipelined expansion's key kernels (k_keys_a / k_mkeys_a, summed
 * over its parts; waits for them) — the bench's roofline of the dominant world > 1 kernel */
int sbd_keypass_ms(sb_engine* e, float* ms);

/* ---- realistic multi-player mode (MultiPlayerState, src/solver.py:471-860; config C4) ----
 * params = {players (2..4), target_points, len tier1, len tier2, len tier3, infinite_resources (0/1:
 * GameConfig.infinite_resources, src/solver.py:33; 1 = speedrun takes, unlimited pool kept in w[11])};
 * tiers = 3 x 40 int32
 * card orders of the tiers (visible first 4, then the deck, src/solver.py:94-119); root_w = the
 * 12-word packed root (oracle/csrc/oracle.c realistic section).  sb_destroy / sb_get_mt_state /
 * sb_num_turns / sb_turn_size / sb_sync / sb_visited_size accept realistic handles. */
int sbr_create(const sb_config* cfg, const int32_t* params, const int32_t* tiers, const uint32_t* mt_state625,
               const uint64_t* root_w, sb_engine** out);
/* one iteration of MultiPlayerState.solve's loop (src/solver.py:820-852) */
int sbr_step(sb_engine* e, sb_step_stats* out);
int sbr_read_turn(sb_engine* e, int32_t turn, int64_t start, int64_t n, uint64_t* w, uint32_t* par, uint64_t* key);
int sbr_path(sb_engine* e, uint64_t* w, int32_t cap, int32_t* len);

#ifdef __cplusplus
}
#endif
#endif /* SPLENDOR_BEAM_H */
