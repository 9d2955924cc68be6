// owgs_internal.h -- device-side data layout shared by owgs_kernels.hip and owgs_host.cpp.
//
// HBM layout of one controller shard (one owgs_ctx), all struct-of-arrays:
//   permits[n_slots]        i32  ForcibleSemaphore state of NestedSemaphore #i (indexed by invoker id, SCPB:413)
//   pool_words[nm + nb]     i32  managed pool positions [0,nm) then blackbox [nm,nm+nb): id if usable, -1 unusable,
//                                 -2 usable but id outside invokerSlots (the reference throws when probing it)
//   hlist[hm + hb]          i32  usable ids of each pool in pool order (healthyInvokers, SCPB:418)
//   act_info[n_actions]     i4   {home, step, mem_mb, meta}; meta = maxConcurrent | pool<<24 | throw<<25 | empty<<26
//   act_slot[n_actions]     i32  slot-key id (fullyQualifiedName(true) interned)
//   act_hash[n_actions]     i32  generateHash(namespace, fqn(false))
//   ctab[cap]               u64  NestedSemaphore concurrency maps of all invokers: one open-addressing table keyed by
//                                 (invoker id, slot key), value {permits c, operationCount} packed in one 8-byte entry
//                                 (one load per probe).  operationCount 0 means "absent" (the reference removes the
//                                 entry, NS:109-111).
#pragma once
#include <stdint.h>

#define OWGS_META_MAXC_MASK 0x00FFFFFF
#define OWGS_META_POOL_SHIFT 24
#define OWGS_META_THROW (1u << 25)
#define OWGS_META_EMPTY (1u << 26)
#define OWGS_META_CURSOR (1u << 27)  // walk cursor valid: maxConcurrent == 1 or the fqn is invoked on one walk only

// concurrency-map entry (8 bytes): key32 << 32 | val32, key32 = (invoker+1) | slot << 15, val32 = c | ops << 12
#define OWGS_CT_SLOT_SHIFT 15
#define OWGS_CT_C_BITS 12
#define OWGS_CT_C_MASK 0xFFFu
#define OWGS_MAX_SLOTS_CT 32767      // invoker ids representable in key32
#define OWGS_MAX_SLOTKEYS 131071     // fqn@version keys representable in key32
#define OWGS_MAX_CONC 4095           // maxConcurrent representable in val32 (c < maxConcurrent)
#define OWGS_MAX_OPS 1048575

#define OWGS_NONE_V (-1)
#define OWGS_THROW_V (-2)
#define OWGS_REL_NOSUCH_BIT 1
#define OWGS_REL_OVERFLOW_BIT 2
#define OWGS_REL_NOENTRY_BIT 4

#define OWGS_PW_UNUSABLE (-1)
#define OWGS_PW_BADID (-2)

#define OWGS_STAMP_BUCKETS 1024
#define OWGS_LDS_BYTES (160 * 1024)
#define OWGS_ENGINE_WAVES 1

struct OwgsEngineArgs {
    int32_t* permits;
    int32_t n_slots;
    const int32_t* pool_words;
    int32_t nm, nb;
    const int32_t* hlist;
    int32_t hm, hb;
    int32_t shortcut_ok; // bit0 managed, bit1 blackbox: pool has no usable out-of-range id
    const int4* act_info;
    const int32_t* act_slot;
    unsigned long long* ctab;
    uint32_t ctab_mask;
    int32_t n_cursors;  // actions with an LDS walk cursor (0 = cursors off)
    // stream
    int32_t n_batches;
    const int64_t* acq_off;
    const int32_t* act;
    const int64_t* rel_off;
    const int64_t* rel_aid;
    const int32_t* rel_inv; // explicit-release mode (owgs_release_batch): invoker per release, action in rel_act
    const int32_t* rel_act;
    unsigned long long seq_base;
    const unsigned long long* seq; // optional explicit seq per activation
    // dense per-activation / per-release records built by owgs_gather_kernel (or by the host for explicit walks)
    const int4* info;   // [n_act] {home, step, mem, meta}
    const int2* aux;    // [n_act] {slot key, action handle or -1}
    const int4* rinfo;  // [n_rel] {aid (or invoker if rel_inv), mem, meta, slot key}
    int32_t* out_inv;
    uint8_t* out_flags;
    uint8_t* rel_flags;
    unsigned long long rng_seed;
    unsigned long long* stats; // [0] iterations [1] probes [2] fallbacks [3] long walks [4] groups
    int32_t* err;              // device error word (table full, ...)
};

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

struct OwgsGatherArgs {
    const int32_t* act;
    int64_t n_act;
    const int4* act_info;
    const int32_t* act_slot;
    int4* info;
    int2* aux;
    const int64_t* rel_aid;
    const int32_t* rel_inv;
    const int32_t* rel_act;
    int64_t n_rel;
    int4* rinfo;
};

struct OwgsLookupArgs {
    const unsigned long long* ctab;
    uint32_t ctab_mask;
    const int32_t* inv;
    const int32_t* slot;
    int32_t n;
    int2* out;
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
    int4* act_info;
};
