// owgs_internal.h -- device-side data layout shared by owgs_kernels.hip and owgs_host.cpp.
//
// HBM layout of one controller shard (one owgs_ctx), all struct-of-arrays:
//   permits[n_slots]        i32  ForcibleSemaphore state of NestedSemaphore #i (indexed by invoker id, SCPB:413)
//   usable[(n_ids+31)/32]   u32  bitmap: invoker id is Healthy (InvokerState.isUsable, ISUP:54-59)   [identity pools]
//   pool_words[nm + nb]     i32  pool position -> id if usable, -1 unusable, -2 usable but id outside invokerSlots
//                                 (the reference throws when probing it)                           [explicit pools]
//   hlist[hm + hb]          i32  usable ids of each pool in pool order (healthyInvokers, SCPB:418)
//   act_meta[n_actions]     u32x2 per action: {home | step << 15 | pool << 30 | cursor_ok << 31,
//                                 mem | maxConcurrent << 17 | throw << 29 | empty << 30}   (SCPB:262-268)
//   act_slot[n_actions]     i32  slot-key id (fullyQualifiedName(true) interned, the NestedSemaphore map key)
//   ct_keys/ct_vals[CTC]    u32  NestedSemaphore concurrency maps of all invokers: one open-addressing table keyed by
//                                 (invoker id, slot key) = (inv + 1) | slot << 15, value c | operationCount << 12.
//                                 Key 0 = empty, key 0xFFFFFFFF = deleted.  Loaded into LDS by every kernel that
//                                 touches it and written back at its end.
//
// Per-replay scratch (built by the pre-pass kernels from the stream, consumed by the engine):
//   rec[n_act]              u32x4 per activation (see OWGS_REC_*): static walk/limit fields of its action plus the
//                                 chunk-local ranks (occurrence of its action among earlier lanes of its chunk, the
//                                 next lane of the same action, the nearest earlier lane of the same slot key with a
//                                 different action).  Inside a chunk the records are dealt by class: maxConcurrent
//                                 == 1 lanes first, then the concurrent ones (stream order inside a class), so each
//                                 engine wave runs one speculation path.
//   lix[n_chunks][OWGS_WL]  u32  stream lane (index in the chunk) of each record position | the first lane of its
//                                 action << 16 (the lane that holds the action's chunk cursor word)
//   gcur[n_actions]         u32  walk cursor of each action (first walk step that may still fit) | batch tag << 15,
//                                 written by the engine, gathered into LDS a chunk ahead by the I/O wave
//   relx[n_act]             i32  position of the activation's release record, -1 never released: inside its batch's
//                                 range rel_off[b] .. rel_off[b+1], maxConcurrent == 1 releases first (relcnt[2b]
//                                 of them), concurrent ones after (order inside a class is free)
//   rel_rec[n_rel]          u32x2 written by the engine when the released activation is decided: {inv | mem << 15,
//                                 slot | maxConcurrent << 17}; inv 0x7FFF = no ActivationEntry (CLB:278-279).  Batch b
//                                 applies rel_rec[rel_off[b] .. rel_off[b+1]) before its publishes.
#pragma once
#include <stdint.h>

// --------------------------------------------------------------------------------------------- engine geometry
#ifndef OWGS_EW
#define OWGS_EW 7                      // engine waves (+ the I/O wave: two waves per SIMD, 256 VGPRs each)
#endif
#ifndef OWGS_LPW
#define OWGS_LPW 64                    // activations per engine wave (64 vs 56: headline 31.5 vs 32.2 ms, same box;
#endif                                 // 56 vs 48: 32.4 vs 33.5; the other configs run narrower chunks)
#define OWGS_ENT (OWGS_EW * 64)        // engine threads
#define OWGS_WL (OWGS_EW * OWGS_LPW)   // chunk width: activations resolved together (one per engine lane)
#define OWGS_NT (OWGS_ENT + 64)        // threads: engine waves + one I/O wave
#ifndef OWGS_NBK_LOG2
#define OWGS_NBK_LOG2 10  // (11: no faster on the BASELINE configs, 8 KB more LDS, ~1.9k fewer invokers)
#endif
#define OWGS_NBK (1 << OWGS_NBK_LOG2)  // "first lane of its invoker" buckets (hashed; collisions are conservative)
#ifndef OWGS_CTC
#define OWGS_CTC 4096                  // concurrency-table capacity (entries, power of two)
#endif
#define OWGS_LDS_BYTES (160 * 1024)

// --------------------------------------------------------------------------------------------- action meta
#define OWGS_AM_POS_MASK 0x7FFFu       // home / step (pool positions < 32768)
#define OWGS_AM_POOL (1u << 30)
#define OWGS_AM_COK (1u << 31)         // walk cursor exact: maxConcurrent == 1 or the slot key has one walk
#define OWGS_AM_MEM_MASK 0x1FFFFu      // memory limit MB < 131072
#define OWGS_AM_MAXC_SHIFT 17
#define OWGS_AM_MAXC_MASK 0xFFFu       // maxConcurrent <= 4095
#define OWGS_AM_THROW (1u << 29)       // home/step index negative (Int.MinValue hash): schedule() throws
#define OWGS_AM_EMPTY (1u << 30)       // pool empty: None
#define OWGS_AM_VALID (1u << 31)       // (rec only) lane holds an activation

// rec.z = action (17 bits, 0x1FFFF none) | occ << 17 (10 bits) | pk1 low 5 bits << 27
// rec.w = slot (17 bits) | next << 17 (10 bits, 0x3FF none) | pk1 high 5 bits << 27
// (the 10-bit "ext" field split over z/w holds pk1 for maxConcurrent > 1 lanes and the hot-action slot otherwise)
// (chunk-lane fields are 10 bits: OWGS_WL <= 512)
#define OWGS_REC_NOACT 0x1FFFFu
#define OWGS_RMASK 0x3FFu
#define OWGS_REC_NONEXT OWGS_RMASK
#define OWGS_REC_NOHOT 0x3FF           // ext field of a maxConcurrent==1 lane: hot-action slot or none

// --------------------------------------------------------------------------------------------- concurrency map
#define OWGS_CT_SLOT_SHIFT 15
#define OWGS_CT_C_BITS 12
#define OWGS_CT_C_MASK 0xFFFu
#define OWGS_CT_TOMB 0xFFFFFFFFu
#define OWGS_MAX_SLOTS_CT 32767        // invoker ids representable in the key
#define OWGS_MAX_SLOTKEYS 131070       // fqn@version keys representable in the key (131071 would alias the tombstone)
#define OWGS_MAX_CONC 4095             // maxConcurrent representable (c < maxConcurrent)
#define OWGS_MAX_OPS 524287          // operationCount is a signed 20-bit field (watched pairs can count below 0)
#define OWGS_MAX_MEM_MB 131071

#define OWGS_NONE_V (-1)
#define OWGS_THROW_V (-2)
#define OWGS_REL_NOSUCH_BIT 1
#define OWGS_REL_OVERFLOW_BIT 2
#define OWGS_REL_NOENTRY_BIT 4
#define OWGS_RR_NOINV 0x7FFFu

#define OWGS_PW_UNUSABLE (-1)
#define OWGS_PW_BADID (-2)

// device error word bits
#define OWGS_ERR_CTAB_FULL 1
#define OWGS_ERR_BAD_STREAM 2          // replay: a release without a matching acquire, or a permit overflow
#define OWGS_ERR_OPS 4
#define OWGS_ERR_INTERNAL 8             // engine invariant violated (a pass without progress)
#define OWGS_ERR_PERMITS 16             // slot permits outside [-2^29, 2^29) MB (the LDS encoding's range)
#define OWGS_ERR_GEOM 32                // the launch's geometry tag is not the engine object's (nothing was touched)
#define OWGS_ERR_RELRISK 64             // owgs_process_batch: the call's releases could push a slot's permits out of the
                                        // LDS range; the engine returned before touching anything (the host reruns the
                                        // call through the ordered release kernels)

// LDS permits of identity pools carry the usable flag: an unusable invoker's permits are stored + OWGS_PENC, so one
// LDS read gives both (usable permits < OWGS_PLIM <= unusable ones); HBM holds the plain values
#define OWGS_PLIM (1 << 29)
#define OWGS_PENC (1 << 30)

// stats slots
#define OWGS_ST_PASSES 0
#define OWGS_ST_PROBES 1
#define OWGS_ST_FALLBACKS 2
#define OWGS_ST_LONG 3
#define OWGS_ST_CHUNKS 4
#define OWGS_ST_STOPS 5
#define OWGS_NSTATS 48  // 0-7 counters, 8-15 profile-build phase cycles, 16-31 profile-build walk counters,
                        // 40-42 profile-build kernel cycles (state load, batches, write-back); 46-47 (host-side, large-
                        // state contexts) decisions kept from the group speculation / decided alone

#define OWGS_MULTI_MAX 8  // controller shards per owgs_engine_multi_kernel launch (kernarg: 8 x args)
#define OWGS_MULTI_DEV_MAX 64  // owgs_engine_multi_dev_kernel: argument blocks in HBM

// HBM overflow of the concurrency table: (invoker, fqn) keys that do not fit in the LDS-sized primary table (the
// reference map is an unbounded TrieMap, NestedSemaphore.scala:30).  Open addressing over cap entries (power of two),
// {key, value} as in the primary; key 0 = empty, OWGS_CT_TOMB = deleted.  A key lives in at most one of the two
// tables; lookups fall through to the overflow only while it holds entries (cnt[0] > 0).  Every access goes through
// L2 (device-scope atomics or L1-bypassing loads).
#define OWGS_CT_LDS_FILL (OWGS_CTC - 256)  // primary entries (live + deleted) beyond which new keys go to the overflow
struct OwgsOvf {
    uint2* t;            // [cap]
    int32_t cap;         // 0: no overflow table
    int32_t* cnt;        // [0] non-empty entries (live + deleted)
    uint32_t* rc;        // [cap] engine release phase: release count << 12 | maxConcurrent (zero between batches)
    int32_t* touched;    // [cap] engine release phase: overflow entries released in the current batch
    int32_t* n_touched;  // [1]
};

// Watched (invoker, fqn) pairs after a slot-state reset (owgs_watch.hip): d[p] = in-flight
// activations of p minus the operationCount of p's entry; W = {p : d[p] > 0}.  Z[p] = the reference holds the empty
// entry a failed concurrent try creates (NestedSemaphore.scala:61-62) while the engine's table has none.
struct OwgsWatch {
    uint32_t* keys;   // [cap] ct_key(invoker, slot); 0 empty, OWGS_CT_TOMB deleted
    uint32_t* vals;   // [cap] d | Z << 31
    int32_t cap;      // 0: no watched pairs (every kernel skips the watch paths)
    int32_t* cnt;     // [1] live entries
    int32_t* wkey;    // [OWGS_MAX_SLOTKEYS + 1] live entries per fqn@version key
};
#define OWGS_W_Z 0x80000000u

struct OwgsEngineArgs {
    int32_t* permits;
    int32_t n_slots;
    int32_t pool_mode;           // 0: identity pools (usable bitmap), 1: explicit pool words
    const uint32_t* usable;      // identity: bitmap over ids [0, n_ids)
    int32_t n_ids;               // identity: blackbox pool position p -> id n_ids - nb + p
    const int32_t* pool_words;   // explicit: [nm + nb]
    int32_t nm, nb;
    const int32_t* hlist;
    int32_t hm, hb;
    int32_t shortcut_ok;         // bit0 managed, bit1 blackbox: pool has no usable out-of-range id
    uint32_t* ct_keys;           // [OWGS_CTC] HBM image of the concurrency table
    uint32_t* ct_vals;
    uint32_t* ct_tmp;            // [2 * max(OWGS_CTC, ovf.cap)] scratch for the table rebuild
    OwgsOvf ovf;
    int32_t n_actions;           // per-action LDS words (walk cursor + chunk rank base)
    // stream
    int32_t n_batches;
    const int64_t* acq_off;      // [n_batches + 1]
    int64_t n_act;               // acq_off[n_batches]
    const int64_t* rel_off;      // [n_batches + 1] or null (no releases)
    const uint4* rec;            // [n_act] pre-pass records, each chunk's lanes dealt by class (see lix)
    const uint32_t* lix;         // [n_chunks][OWGS_WL] stream lane | first lane of its action << 16, per record position
    uint32_t* gcur;              // [max(n_actions, 1)] walk cursor of each action: batch tag << 15 | step
    int32_t cur_tag0;            // batch b of this launch tags its cursors (cur_tag0 + b + 1) & 0x1FFFF
    const int32_t* relpos;       // [n_act] relx (see above), or null: no releases
    const int32_t* relcnt;       // [2 * n_batches] per batch: maxConcurrent == 1 records, concurrent records
    uint2* rel_rec;              // [n_rel] release records, in rel_aid order (written when the activation is decided)
    const int32_t* rel_src;      // explicit releases (owgs_process_batch): record position -> the caller's release
                                 // index (flags go to rel_flags[rel_src[p]]); null for a stream's own releases
    unsigned long long seq_base;
    const unsigned long long* seq; // optional explicit seq per activation
    int32_t* out_inv;
    uint8_t* out_flags;
    uint8_t* rel_flags;
    unsigned long long rng_seed;
    unsigned long long* stats;   // this launch's counters (zero when it starts)
    unsigned long long* stats_next;  // the next launch's counter block: zeroed at the end of this one (no fill launch)
    int32_t* err;
    int32_t opts;                // diagnostics (env OWGS_OPTS): bit0 = no hot-action rank tables
    int32_t cw;                  // chunk width of this replay (<= OWGS_WL)
    unsigned long long* trace;   // diagnostic build only (-DOWGS_TRACE): [waves][OWGS_TRACE_CAP] barrier timeline
    int32_t feat;                // engine code paths this launch needs (OWGS_F_*): picks the compiled specialisation
    uint32_t geom;               // OWGS_GEOM_TAG of the geometry the host sized this launch's buffers for
    unsigned long long* rel_bound;  // owgs_process_batch: per slot, the memory the call's releases can return at most
                                    // (staged by owgs_stage_releases_kernel; the engine checks and zeroes it), or null
    // identity pools, owgs_replay_device_group: the usable bitmap batch b applies before its releases (updateInvokers
    // with a new health vector, SCPB:512-551) at hwords + b * hstride, or null
    const uint32_t* hwords;
    int32_t hstride;
    // pinned host words the launch's last step stores into (null: none), so that the caller reads them after its
    // stream synchronisation without a copy: the context's error word after this launch, and the overflow table's
    // entry count (its bound for the next call's sizing)
    int32_t* err_host;
    int32_t* ovf_host;
    // the primary table's entries right after its last rebuild, kept across launches (null: 0 at every launch): a
    // launch rebuilds the table once its entries grew by OWGS_CTC / 8 since (a shim call per launch would otherwise
    // rebuild in every call once the table is half full)
    int32_t* ct_clast;
    // owgs_process_batch: as its last step the launch copies out_copy_n16 x 16 bytes of its outputs (decisions, flags,
    // release flags: HBM) to the caller's pinned block, so no copy is queued behind it (0: none)
    const uint4* out_copy_src;
    uint4* out_copy_dst;
    int32_t out_copy_n16;
};
// Geometry/ABI tag.  The host and an engine object must agree on the chunk width (the stride of lix, the 10-bit lane
// fields of the records), the primary table's capacity and the argument block's layout; the host builds the tag of the
// geometry it sized its buffers for, and every engine object's launch wrappers (and the kernels themselves, before
// their first barrier or wait) compare it with their own: a mismatch is refused (OWGS_ERR_GEOM) instead of running
// with out-of-bounds chunk tables.
#define OWGS_GEOM_TAG(wl)                                                                             \
    (0x50000000u | ((uint32_t)(wl) & 0x3FFu) | (((uint32_t)sizeof(OwgsEngineArgs) & 0x3FFu) << 10) | \
     ((uint32_t)__builtin_ctz(OWGS_CTC) << 20))
// Engine specialisations.  The engine body is compiled once per feature set, and the host launches the smallest one
// that covers the context and the call, so a stream without concurrent actions on identity pools runs a kernel with
// none of the NestedSemaphore map, explicit-pool or explicit-sequence code in it (fewer instructions per pass, fewer
// registers, a loop body that stays in the instruction cache).
#define OWGS_F_CONC 1  // maxConcurrent > 1 actions: the concurrency map (primary + overflow), container scans
#define OWGS_F_GEN 2   // explicit pool words (non-identity pools) or explicit per-activation sequence numbers
#define OWGS_F_ALL 3

// generateHash(namespace, action) for n actions: out[i] = abs(h(ns_i) ^ h(path_i)), Int.MinValue kept (SCPB:370-372).
// If raw != 0, out[i] = h(ns_i) only (String.hashCode of the first string set).
struct OwgsHashArgs {
    const char* ns_bytes;
    const int32_t* ns_off;
    const char* path_bytes;
    const int32_t* path_off;
    int32_t n;
    int32_t raw;
    int32_t* out;
};

struct OwgsPrepArgs {
    const int32_t* hash;
    const int32_t* mem;
    const int32_t* maxc;
    const uint8_t* bb;
    const uint8_t* cursor_ok;
    int32_t n;
    int32_t nm, nb;
    const int32_t* msteps;
    int32_t n_msteps;
    const int32_t* bsteps;
    int32_t n_bsteps;
    uint2* act_meta;
};

// chunk-local pre-pass: one workgroup of OWGS_WL threads per chunk
struct OwgsRelposArgs {
    const int64_t* rel_aid;      // [n_rel]
    int64_t n_rel, n_act;
    const int64_t* rel_off;      // [n_batches + 1]
    int32_t n_batches;
    const int32_t* act;          // [n_act] action per activation
    const uint2* act_meta;       // [n_actions]
    int32_t* relx;               // out [n_act] (memset -1)
    int32_t* relcnt;             // out [2 * n_batches] (memset 0)
    int32_t* err;
    // a group of batches replayed in its own launch (owgs_replay_device_group): a release of an activation decided by
    // an EARLIER launch (aid < decided_below) gets its record written here from that decision, not by the engine
    int64_t decided_below;
    const int32_t* out_inv;
    const int32_t* act_slot;
    uint2* rel_rec;
};

struct OwgsPrepassArgs {
    int32_t n_batches;
    const int64_t* acq_off;
    const int32_t* cstart;       // [n_batches + 1] first chunk of each batch (owgs_chunks_kernel), or null: each
                                 // workgroup walks the few batches' chunk counts itself
    const int32_t* act;          // [n_act] action per activation, or null: per-activation meta in xmeta/xslot
    const uint2* act_meta;       // [n_actions]
    const int32_t* act_slot;     // [n_actions]
    const uint2* xmeta;          // explicit walks: [n_act]
    const int32_t* xslot;        // explicit walks: [n_act]
    uint4* rec;                  // out [n_act]: chunk lanes in class order (maxConcurrent == 1 first)
    uint32_t* lix;               // out [n_chunks][OWGS_WL]: stream lane | first lane of its action << 16
    int32_t cw;                  // chunk width (<= OWGS_WL)
    int32_t deal;                // lane dealing strategy (diagnostics, env OWGS_DEAL; 0 = default)
    uint32_t geom;               // OWGS_GEOM_TAG of the host's geometry (checked like the engine's)
};

// ordered explicit releases (owgs_release_batch): one wave, releases in stream order
struct OwgsReleaseArgs {
    int32_t* permits;
    int32_t n_slots;
    uint32_t* ct_keys;
    uint32_t* ct_vals;
    int32_t n;
    const int32_t* inv;
    const int32_t* mem;
    const int32_t* maxc;
    const int32_t* slot;
    uint8_t* flags;
    int32_t* err;
    OwgsOvf ovf;
    // scratch of the parallel front end (owgs_launch_release_seq): per-invoker upper bound of the memory returned,
    // overflow-risk word, selection of the releases the ordered kernel still has to apply
    unsigned long long* bound;  // [n_slots]
    int32_t* risk;
    uint8_t* sel_flag;          // [n]
    int32_t* sel_idx;           // [n]
    int32_t* sel_cnt;
    void* temp;
    size_t temp_bytes;
    // concurrent releases grouped by NestedSemaphore entry (no-risk path): entry key and release index per release,
    // sorted copies, and each entry's [begin, end) in the sorted order
    uint32_t* ckey;      // [n]
    int32_t* cval;       // [n]
    uint32_t* ckey_s;    // [n]
    int32_t* cval_s;     // [n]
    int32_t* cbeg;       // [OWGS_CTC]
    int32_t* cend;       // [OWGS_CTC]
    OwgsWatch w;         // watched pairs (w.cap == 0: none); their releases take the ordered kernel
};

// Resident engine (owgs_resident.hip): owgs_process_batch's small calls served by one workgroup that keeps the slot
// state in LDS between calls, fed through a control block in pinned, coherent host memory.  Word indices of ctl:
#define OWGS_RES_BELL 0     // host: call number (counts up from the launch's last_call), -1 = write back and exit
#define OWGS_RES_DONE 16    // device: call number of the last call served (written after its outputs and result)
#define OWGS_RES_STATE 32   // device: 1 = image loaded, 2 = written back and exiting
#define OWGS_RES_RESULT 48  // device: the last call's outcome (0, OWGS_RES_BAIL_*) | its device error bits << 8
#define OWGS_RES_USED 49    // device: primary-table entries (live + deleted) after the last call
#define OWGS_RES_GEN 50     // device: the walk-cursor generation reached (the host's next launch starts past it)
#define OWGS_RES_TOMBS 51   // device: deleted primary-table entries after the last call
#define OWGS_RES_WHY 52     // device: why the engine exited (0 the stop word, 1 idle, 2 its lifetime)
#define OWGS_RES_WLIVE 53   // device: watched pairs left after the last call (when the launch has any)
#define OWGS_RES_PROF 96    // device: the last call's counters (OWGS_RES_NPROF words: walk rounds, decisions,
                            // staging / release / publish cycles, overflow lookups, cursor hits, U shortcuts,
                            // decisions of the grouped walks)
#define OWGS_RES_NPROF 21  // (+ validation passes, decisions decided alone, their cycles, speculation and
                           // validation cycles: validation includes the decisions decided alone; speculation's
                           // rank matching, plain walks, concurrent walks; validation's entry inserts; the
                           // releases' concurrent part; chunks whose concurrent decisions were speculated ahead;
                           // the helper wave's concurrent walks)
#define OWGS_RES_HDR 64     // host: the call -- n_runs, n_rel, n_pub, has_seq, seq_base lo, hi, then byte offsets in
                            // the input block of pub_off, the release invokers, the release actions, seq (u64), the
                            // block's length, the memory the releases return at most (lo, hi), and the byte
                            // offset of the publish words.  The block: rel_off i32[n_runs + 1] | pub_off |
                            // publish words u32[n_pub] (action | rank << 17 | shared << 23) | release invokers
                            // i32[n_rel] | release actions i32[n_rel] | seq u64[n_pub], 16-byte aligned parts (the
                            // engine gathers each record's action meta and slot key from HBM; stream mode's header
                            // names its record arrays in LDS instead: see spec_replay).
                            // Outputs (block `out`): out_inv i32[n_pub] | out_flags u8[n_pub] | rel_flags u8[n_rel]
#define OWGS_RES_NHDR 16
#define OWGS_RES_CALL_LIMIT 0x7FFFFF00ll     // the bell stays below this (a negative bell is the stop word)
#define OWGS_RES_GEN_LIMIT 0xFFFFFF00ull     // the walk-cursor generation stays below this (compared by equality)
#define OWGS_RES_CTL_WORDS 128
#define OWGS_RES_BAIL_RELRISK 1  // a release could leave the LDS permit range: nothing applied, the host reruns the
                                 // call through the ordered release kernels
#define OWGS_RES_BAIL_STAGE 2    // the call does not fit the staging area (the host sized it: not expected)
struct OwgsResArgs {
    int32_t* permits;
    int32_t n_slots;
    const uint32_t* usable;      // identity pools only
    int32_t n_ids, nm, nb;
    uint32_t* ct_keys;
    uint32_t* ct_vals;
    uint32_t* ct_tmp;            // [2 * OWGS_CTC] scratch of the primary table's cleanup
    OwgsOvf ovf;
    const uint2* act_meta;
    const int32_t* act_slot;
    int32_t n_actions;
    unsigned long long rng_seed;
    int32_t* err;
    int32_t* ctl;                // [OWGS_RES_CTL_WORDS] pinned, coherent
    const int32_t* in;           // pinned inputs of a call
    char* out;                   // pinned outputs of a call
    int32_t stage_bytes;         // LDS bytes for a call's staged inputs
    int32_t last_call;           // the bell's value at launch
    uint2* cur;                  // [n_actions] walk cursor of each action: {generation, first walk step that may fit}
    uint32_t gen_base;           // first cursor generation of this launch (above every generation stored in cur)
    long long idle_ticks;        // s_memrealtime ticks (100 MHz) without a call before the engine writes back and exits
    long long life_ticks;        // ... and ticks after its launch, checked between calls (0: no bound)
    int32_t spec;                // walk steps of each publish's speculative walk (0: decisions one at a time only)
    int32_t cspec;               // ... of a concurrent publish's (0: max(4, spec / 4))
    int32_t cspec_pre;           // ... of the next chunk's concurrent publishes, speculated ahead (0: as cspec)
    int32_t hsplit;              // wave 1 speculates the concurrent decisions of a chunk while wave 0 walks the others
    int32_t prespec;             // (hsplit == 1) wave 1 speculates the concurrent decisions of a run's next chunk too
    // watched pairs after a reset (w.cap == 0: none): their releases in queue order with the
    // empty-entry rule, and the Z marks of the walks that tried and failed at them, inside the engine.  The host indexes
    // W by fqn@version key at launch: w_sidx (open addressing, w_scap a power of two) {slot + 1, first, count, primary
    // action} -> w_list[first .. first + count) {W index, walk step of the pair's invoker in the primary action's walk
    // (0x7FFFFFFF: not in its pool)}, by step
    OwgsWatch w;
    const uint4* w_sidx;
    int32_t w_scap;
    const uint2* w_list;
    // stream mode (owgs_replay_device through this engine): no doorbell, the stream's batches from HBM
    int32_t smode;
    int32_t s_nb;
    long long s_nact;            // activations in the stream (a release must name one of them)
    const int64_t* s_acq_off;    // [s_nb + 1]
    const int32_t* s_act;        // [n_activations] action handle of each activation
    const int64_t* s_rel_off;    // [s_nb + 1] or null
    const int64_t* s_rel_aid;    // released activations (decided by an earlier batch)
    unsigned long long s_seq_base;
    int32_t* s_out_inv;
    uint8_t* s_out_fl;
    uint8_t* s_rel_fl;           // or null
    unsigned long long* s_stats; // [OWGS_RES_NPROF] summed counters, or null
    uint32_t* s_claim;           // one bit per activation, zeroed: a second release of one is refused (or null)
};

// Large-state engine (owgs_seq.hip): contexts beyond the on-chip image (owgs_limits) or with maxConcurrent beyond
// OWGS_MAX_CONC.  Permits in HBM, one HBM map keyed by the full (invoker, fqn@version) pair, 32-bit walk positions.
#define OWGS_SEQ_MAX_WORDS 16383  // usable-bitmap words of the large-state engine (524,256 invoker ids; pools up to 524,287 positions, owgs_coprime_max)
struct OwgsSeqArgs {
    int32_t* permits;
    int32_t n_slots;
    const uint32_t* usable;       // identity pools: bitmap over ids [0, n_ids)
    int32_t n_ids, nm, nb;
    const int32_t* msteps;        // pairwiseCoprimeNumbersUntil of each pool (SCPB:379-384)
    int32_t n_msteps;
    const int32_t* bsteps;
    int32_t n_bsteps;
    const int32_t* act_hash;      // generateHash (SCPB:370-372) per action handle
    const int32_t* act_mem;
    const int32_t* act_maxc;
    const int32_t* act_slot;
    const uint8_t* act_bb;
    uint4* cur;                   // [n_actions] walk cursor {generation, first step that may still fit, its pool
                                  //   position, 0} (maxConcurrent == 1 actions)
    int32_t n_actions;
    uint32_t gen0;                // this call's first cursor generation (release runs count up from it)
    uint4* map;                   // [map_cap] {invoker + 1 (0 empty, ~0 deleted), slot, free slots, operationCount}
    int32_t map_cap;              // a power of two
    int32_t* map_filled;          // non-empty entries (live + deleted)
    int32_t n_runs;
    const int64_t* rel_off;       // [n_runs + 1] releases of each run (indices into the release arrays)
    const int64_t* pub_off;       // [n_runs + 1] publishes of each run (indices into pub_act / out_*)
    const int64_t* rel_aid;       // releases by activation (stream replays): invoker dec_inv[aid], action dec_act[aid]
    const int32_t* dec_inv;
    const int32_t* dec_act;
    const int32_t* rel_inv;       // explicit releases (rel_aid null): invoker and action handle
    const int32_t* rel_act;
    const int32_t* rel_mem;       // or, for the completion path's records (rel_act null): memory, maxConcurrent and
    const int32_t* rel_maxc;      //   fqn@version key of each release
    const int32_t* rel_slot;
    uint8_t* rel_flags;           // or null
    const int32_t* pub_act;
    const unsigned long long* seq;  // or null: seq_base + index
    unsigned long long seq_base;
    int32_t* out_inv;
    uint8_t* out_flags;
    unsigned long long rng_seed;
    int32_t* state;               // [5] {stopped for a map growth, run, phase, index lo, hi} -- resumed when resume != 0
    int32_t resume;
    int32_t* err;
};

// owgs_process_batch: the caller's releases (invoker, action handle) of each run as engine release records
struct OwgsStageArgs {
    int32_t n_runs;
    const int64_t* rel_off;     // [n_runs + 1]
    const int32_t* rel_inv;
    const int32_t* rel_act;
    const int32_t* act_mem;
    const int32_t* act_maxc;
    const int32_t* act_slot;
    int32_t n_slots;
    uint2* rel_rec;             // out [n_rel]: per run maxConcurrent == 1 (and no-op) records first, concurrent after
    int32_t* rel_src;           // out [n_rel]: record position -> release index
    int32_t* relcnt;            // out [2 n_runs]: records of the first class, of the second
    uint8_t* rel_flags;         // out [n_rel]: OWGS_REL_NOENTRY_BIT for invoker < 0, else 0 (the engine adds NoSuch)
    // span mode (owgs_replay_device_span, one run): rel_off is null, release i names activation rel_aid[i] of the
    // caller's stream, whose invoker and action are dec_inv[...] / dec_act[...]; span_off receives the engine's
    // offsets {0, span_npub} (publishes) and {0, n_rel} (releases)
    const int64_t* rel_aid;
    const int32_t* dec_inv;
    const int32_t* dec_act;
    int64_t span_nrel, span_npub;
    int64_t* span_off;
    int32_t* tile_cnt;          // span mode, more than OWGS_STAGE_TILE releases: first-class records per tile (scratch)
    unsigned long long* bound;  // or null: per slot, the memory of every release naming it (zero before the call)
};
#define OWGS_STAGE_TILE 1024

// watch kernels (owgs_watch.hip)
struct OwgsWRebuildArgs {   // at a reset: the new W from the table's entries and the old W
    const uint32_t* ct_keys;
    const uint32_t* ct_vals;
    OwgsOvf ovf;
    OwgsWatch old_w;
    OwgsWatch new_w;
};
struct OwgsWUpdateArgs {    // after a publish run: Z of the watched pairs that are absent from the table
    int32_t n;              // decisions
    const int32_t* act;     // registered actions (or null: explicit walks in xmeta / xslot)
    const uint2* act_meta;
    const int32_t* act_slot;
    const uint2* xmeta;
    const int32_t* xslot;
    const int32_t* out_inv;
    const uint8_t* out_flags;
    int32_t pool_mode, n_ids, nm, nb;
    const uint32_t* usable;     // identity pools
    const int32_t* pool_words;  // [nm + nb]
    const uint32_t* ct_keys;    // HBM image of the primary table (written back by the engine)
    OwgsOvf ovf;
    OwgsWatch w;
    int32_t* D;             // [n_actions] deepest failed step + 1 per action in this run (zero between runs)
    int32_t* L;             // [n] actions listed in D
    uint4* L2;              // [n] {meta.x, slot, depth, 0} per listed walk
    int32_t* Lcnt;          // [2] listed actions, listed walks
};

struct OwgsLookupArgs {
    const uint32_t* ct_keys;
    const uint32_t* ct_vals;
    OwgsOvf ovf;
    const int32_t* inv;
    const int32_t* slot;
    int32_t n;
    int2* out;
};

// --------------------------------------------------------------------------------------------- completion acks
// (owgs_acks.hip; outcome codes = OWGS_ACK_* in include/owgs.h)
#ifndef OWGS_ACK_FAIL
#define OWGS_ACK_FAIL 0
#define OWGS_ACK_JVM 1
#define OWGS_ACK_UNSUPPORTED 2
#define OWGS_ACK_RELEASED 3
#define OWGS_ACK_HEALTH 4
#define OWGS_ACK_NOENTRY 5
#define OWGS_ACK_FORCED_NOENTRY 6
#endif
#define OWGS_ACK_COMPLETION 3       // parsed CompletionMessage (before resolution into RELEASED / HEALTH / NOENTRY)

struct OwgsAckParseArgs {
    const uint8_t* bytes;        // messages, padded by >= 16 readable bytes
    const int64_t* off;          // [n + 1]
    int32_t n;
    long long health_start_ms;   // TransactionId.invokerHealth's start (TransactionId.scala:225)
    const uint8_t* forced;       // null for raw acks
    ulonglong2* key;             // out: activation id (128 bits)
    int32_t* inst;               // out: invoker instance (BigDecimal.intValue)
    uint8_t* info;               // out: kind | isSystemError << 4 | health tid << 5 | forced << 6
};

// activationSlots (CLB:60): open addressing over cap (power of two) slots
struct OwgsActTable {
    unsigned long long* tw;      // 0 empty, 1 ready, 2 deleted, 1 << 63 | batch index = claimed by an insert batch
    ulonglong2* tk;              // activation id
    int2* tv;                    // {action handle, caller ticket}
    int32_t* owner;              // lowest batch index of a slot's inserts / removals (INT_MAX between calls)
    long long cap;
};

struct OwgsAckCompleteArgs {
    const ulonglong2* key;
    const uint8_t* info;
    const int32_t* inst;
    int32_t n;
    int32_t* slot;               // scratch [n]
    const int32_t* act_mem;
    const int32_t* act_maxc;
    const int32_t* act_slot;
    int32_t n_slots;
    int32_t *r_inv, *r_mem, *r_maxc, *r_slot;   // release records (owgs_release_seq_kernel input)
    uint8_t* out_kind;
    int32_t* out_ticket;
    unsigned long long* counters;               // [0] entries inserted, [1] entries removed
};

// ActivationMessage serialisation + topic fan-out (owgs_msgs.hip); every pointer is device memory
struct OwgsMsgArgs {
    int32_t n;
    const int32_t* invoker;
    const int32_t* tmpl;
    const char* ta;
    const int64_t* ta_off;
    const char* tb;
    const int64_t* tb_off;
    int32_t n_templates;
    const char* rci;
    int32_t rci_len;
    const ulonglong2* aid;
    const char* tid;
    const int64_t* tid_off;
    const int64_t* tid_start;
    const uint8_t* flags;
    const char* content;
    const int64_t* content_off;
    const ulonglong2* cause;
    const char* trace;
    const int64_t* trace_off;
    int32_t n_topics;
    // scratch and outputs
    uint32_t* key;
    int64_t* len;
    int32_t* bad;          // bit0 invoker/template out of range, bit1 malformed UTF-8 transaction id, bit2 overflow
    int32_t* order;        // [n] activation index of each output message (first m valid)
    int64_t* out_off;      // [n + 1] byte offsets (out_off[m] = out_off[n] = total)
    int32_t* topic_start;  // [n_topics + 1]
    char* out;
    int64_t cap;
};
