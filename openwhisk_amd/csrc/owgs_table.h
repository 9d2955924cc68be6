// owgs_table.h -- device helpers for the NestedSemaphore concurrency map (an open-addressing table keyed by
// (invoker, fqn@version), owgs_internal.h) and for the watched-pair table of a reset (owgs_watch.hip).  Shared by the
// engine, the release kernels and the watch kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "owgs_internal.h"

__device__ __forceinline__ uint32_t ct_hash(uint32_t k) {
    k ^= k >> 16;
    k *= 0x7feb352dU;
    k ^= k >> 15;
    k *= 0x846ca68bU;
    k ^= k >> 16;
    return k;
}
__device__ __forceinline__ uint32_t ct_key(int inv, int slot) {
    return (uint32_t)(inv + 1) | ((uint32_t)slot << OWGS_CT_SLOT_SHIFT);
}
// Concurrency table (LDS or HBM image): linear probing from a 4-entry-aligned home, so the engine reads a key's
// first 4 candidate entries with two ds_read_b128 (bucketized linear probing).  Deleted entries are skipped, an empty
// entry ends the chain.
#define CT_BLK 4
__device__ __forceinline__ uint32_t ct_home(uint32_t key) {
    return (ct_hash(key) & (OWGS_CTC / CT_BLK - 1)) * CT_BLK;
}
__device__ __forceinline__ int ct_find(const uint32_t* ctk, uint32_t key) {
    uint32_t h = ct_home(key);
    for (int p = 0; p < OWGS_CTC; ++p) {
        const uint32_t k = ctk[h];
        if (k == key) return (int)h;
        if (k == 0) return -1;
        h = (h + 1) & (OWGS_CTC - 1);
    }
    return -1;
}
// insert a key known to be absent: claim the first empty or deleted entry of its chain (concurrent inserters of
// different keys race by CAS)
__device__ __forceinline__ int ct_insert(uint32_t* ctk, uint32_t key, int* fresh) {
    uint32_t h = ct_home(key);
    for (int p = 0; p < OWGS_CTC;) {
        const uint32_t k = ctk[h];
        if (k == 0 || k == OWGS_CT_TOMB) {
            if (atomicCAS(&ctk[h], k, key) == k) {
                *fresh = k == 0;
                return (int)h;
            }
            continue;  // lost the race: re-read this entry
        }
        h = (h + 1) & (OWGS_CTC - 1);
        ++p;
    }
    return -1;
}

// ------------------------------------------------------------------------------------------------ overflow table
__device__ __forceinline__ uint2 ovf_ld(const uint2* t, int i) {
    const unsigned long long v = __hip_atomic_load((const unsigned long long*)&t[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
}
__device__ __forceinline__ void ovf_st(uint2* t, int i, uint32_t k, uint32_t v) {
    __hip_atomic_store((unsigned long long*)&t[i], (unsigned long long)k | ((unsigned long long)v << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ovf_st_val(uint2* t, int i, uint32_t v) {
    __hip_atomic_store(&t[i].y, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// index of key in the overflow (or -1), *val its value (0 if absent); linear probing from its hash, an empty entry
// ends the chain
__device__ __forceinline__ int ovf_find(const OwgsOvf& O, uint32_t key, uint32_t* val) {
    *val = 0u;
    if (O.cap <= 0) return -1;
    const uint32_t m = (uint32_t)O.cap - 1u;
    uint32_t h = ct_hash(key) & m;
    for (int p = 0; p < O.cap; ++p) {
        const uint2 e = ovf_ld(O.t, (int)h);
        if (e.x == key) {
            *val = e.y;
            return (int)h;
        }
        if (e.x == 0u) return -1;
        h = (h + 1u) & m;
    }
    return -1;
}
// insert a key absent from both tables into the first empty or deleted entry of its chain (CAS on the key word)
__device__ __forceinline__ int ovf_insert(const OwgsOvf& O, uint32_t key, uint32_t val) {
    if (O.cap <= 0) return -1;
    const uint32_t m = (uint32_t)O.cap - 1u;
    uint32_t h = ct_hash(key) & m;
    for (int p = 0; p < O.cap;) {
        const uint32_t k = ovf_ld(O.t, (int)h).x;
        if (k == 0u || k == OWGS_CT_TOMB) {
            if (atomicCAS(&O.t[h].x, k, key) == k) {
                ovf_st_val(O.t, (int)h, val);
                return (int)h;
            }
            continue;  // lost the entry: re-read it
        }
        h = (h + 1u) & m;
        ++p;
    }
    return -1;
}

// signed operationCount of an entry value (c | ops << 12, ops a 20-bit two's complement field: entries the
// reference creates empty on a failed try can count below zero, ResizableSemaphore.scala:99-108)
__device__ __forceinline__ int ct_ops(uint32_t v) { return (int)v >> OWGS_CT_C_BITS; }
__device__ __forceinline__ uint32_t ct_val(int c, int ops) {
    return (uint32_t)c | ((uint32_t)ops << OWGS_CT_C_BITS);
}

// ------------------------------------------------------------------------------------------------ watched pairs
// W: key = ct_key(invoker, slot), value = d | Z << 31 (owgs_internal.h OwgsWatch); linear probing from the key's hash
__device__ __forceinline__ int w_find(const OwgsWatch& W, uint32_t key) {
    if (W.cap <= 0) return -1;
    const uint32_t m = (uint32_t)W.cap - 1u;
    uint32_t h = ct_hash(key) & m;
    for (int p = 0; p < W.cap; ++p) {
        const uint32_t k = __hip_atomic_load(&W.keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == key) return (int)h;
        if (k == 0u) return -1;
        h = (h + 1u) & m;
    }
    return -1;
}
// insert a key absent from the table (the rebuild inserts distinct keys into an empty table)
__device__ __forceinline__ int w_insert(const OwgsWatch& W, uint32_t key, uint32_t val) {
    const uint32_t m = (uint32_t)W.cap - 1u;
    uint32_t h = ct_hash(key) & m;
    for (int p = 0; p < W.cap; ++p, h = (h + 1u) & m) {
        if (atomicCAS(&W.keys[h], 0u, key) == 0u) {
            __hip_atomic_store(&W.vals[h], val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return (int)h;
        }
    }
    return -1;
}
