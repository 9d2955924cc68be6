// owgs_kernels.hip -- CDNA4 (gfx950) kernels of the batched invoker scheduler.
//
// Kernels
//   owgs_hash_kernel      generateHash(namespace, action) (SCPB:370-372): java.lang.String.hashCode of both strings,
//                         one wave per action; lane i sums c[i+64k] * 31^(L-1-i-64k) (mod 2^32), the wave reduces.
//   owgs_prepare_kernel   per action: home = hash % n, step = stepSizes(hash % k), limits -> act_meta (SCPB:262-268).
//   owgs_chunks_kernel    first chunk of every batch (chunks = OWGS_WL consecutive publishes of one batch).
//   owgs_prepass_kernel   one workgroup per chunk: per-activation engine record = action meta + chunk-local ranks.
//   owgs_relpos_kernel    release bookkeeping: each released activation learns the position of its release record.
//   owgs_engine_kernel    the hot path: releases (SCPB:327-331 -> NS:98-113) and schedule() (SCPB:398-436 with
//                         NS:32-91) for a whole stream of batches, replaying the reference's SEQUENTIAL semantics.
//   owgs_relflags_kernel  per-release flags after the replay (no ActivationEntry, CLB:278-279).
//   owgs_release_seq_kernel  explicit releases in stream order (owgs_release_batch).
//
// Engine.  One workgroup owns one controller shard: OWGS_EW engine waves + one I/O wave.  Slot
// permits, pool usability, the concurrency maps and one word per action (walk cursor + chunk rank base) live in LDS
// for the whole stream.  Activations are resolved OWGS_WL at a time (one per engine lane, in stream order) by
// speculation + conservative validation + prefix commit:
//   * memory permits never increase inside a batch (releases are applied at batch boundaries), so a walk step that is
//     infeasible at the chunk frontier f stays infeasible: the per-action cursor (first step that may still be
//     feasible) only moves forward inside a batch;
//   * PACKING: lane i of action a with rank r (earlier uncommitted lanes of a in the chunk) speculates the step at
//     which the capacity along a's walk (floor(permits / mem) invocations per invoker, + the concurrency slots for
//     maxConcurrent > 1) first exceeds r, i.e. where it lands if the r earlier lanes of a land where they speculate;
//   * every lane adds its memory consumption to a (hashed) bucket of its target invoker; a lane is KNOWN to fit when
//     it is the first lane of its bucket or the bucket total fits the invoker's permits (a sound upper bound of the
//     consumption by earlier lanes), or it is a forced acquire;
//   * lanes [f, l) commit, l = first lane not known to fit; the frontier lane f is always exact, so each pass
//     commits at least one lane; the next pass re-speculates [l, chunk end) against the updated state.
// The I/O wave streams the next chunk's records from HBM into an LDS double buffer; the engine waves only store to
// HBM (decisions, release records), so no engine-wave load ever waits behind its own stores.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <atomic>

#include "owgs_internal.h"
#include "owgs_table.h"

// Engine geometry variants (owgs_engine_narrow.hip): the same source compiled again with narrower chunks inside its own
// namespace, exporting only the geometry-dependent entry points (engine, pre-pass, LDS layout) under a suffix.
#ifdef OWGS_VARIANT_NS
#define OWGS_SHARED 0
namespace OWGS_VARIANT_NS {
#else
#define OWGS_SHARED 1
#endif
#ifndef OWGS_GEOM
#define OWGS_GEOM(name) name
#endif

typedef unsigned long long u64;

#define K_NONE 0
#define K_THROW 1
#define K_TARGET 2
#define K_FALLBACK 3
#define K_LONG 4
#define K_HOT 5  // resolved from the hot-action rank table after the pass barrier
#define K_CSCAN 6  // concurrent action, mem > every usable permit count: resolved from the key's open containers
#ifndef OWGS_REL_RQ
#define OWGS_REL_RQ 4  // release sweep: 16-byte reads in flight per thread, concurrent records
#endif
#ifndef OWGS_REL_RQ1
#define OWGS_REL_RQ1 8  // maxConcurrent == 1 records
#endif
#ifndef OWGS_OVF
#define OWGS_OVF 1  // 0: measurement variant without the overflow table's fall-through paths
#endif
#ifndef OWGS_HOT_ROT
#define OWGS_HOT_ROT 0  // engine wave (w + OWGS_HOT_ROT) % OWGS_EW walks hot slots w + 1, w + 1 + 8, .. (load balance)
#endif
#ifndef OWGS_HOT_IO
#define OWGS_HOT_IO 1  // the I/O wave takes a share of the hot-action walks
#endif
#ifndef OWGS_QUEUE_IO
#define OWGS_QUEUE_IO 1  // ... and pops queued long walks when the queue is shared
#endif
#ifndef OWGS_CSCAN_MIN_N
#define OWGS_CSCAN_MIN_N (OWGS_CTC / 2)  // pools at most this large walk instead of scanning the table
#endif
#ifndef OWGS_EXT
#define OWGS_EXT 1  // stopping maxConcurrent == 1 lanes are re-decided exactly inside the pass (see the commit phase)
#endif
#ifndef EXT_MAX
#define EXT_MAX 48  // re-decisions per pass
#endif
#ifndef EXT_ROUNDS
#define EXT_ROUNDS 8  // walk rounds (128 steps each) a re-decision may take; a longer walk waits for the next pass
#endif
#ifndef OWGS_PRE
#define OWGS_PRE 0  // stopping lanes walk their own re-decision in validate, in parallel (see the commit phase)
#endif
#ifndef PRE_G
#define PRE_G 6  // 4-step groups such a walk may take (beyond them the I/O wave walks it)
#endif
// the pre-walk's record of the invokers it skipped: one bit of a 64-bit signature per invoker
__device__ __forceinline__ uint32_t pre_bit(int x) { return ((uint32_t)x * 0x9E3779B1u) >> 26; }
// fxa[li] (per lane of the pass, stream order): x = action | not known to fit << 24 | exempt << 25 | re-decidable << 26
// | re-decided << 27 | kind << 28 | clash << 30; y = target (0xFFFF none) | walk step << 16 (after a re-decision: the
// new ones); z = the action's meta.x (home | step << 15 | pool); w = mem | took memory << 31
#define FX_NOT 0xFFFFu
#define FX_NF (1u << 24)
#define FX_EXEMPT (1u << 25)
#define FX_OK (1u << 26)
#define FX_DONE (1u << 27)
#define FX_CLASH (1u << 30)  // a lane after the pass limit that targets a re-decided lane's invoker or shares its action
#ifndef OWGS_CSCAN_ON
#define OWGS_CSCAN_ON 1
#endif

#ifndef KPROBE
#define KPROBE 16  // walk steps a maxConcurrent==1 lane probes on its own before the wave-cooperative walk (x4)
#endif
#ifndef KPROBE_G
#define KPROBE_G 4  // same for the general path (concurrency lookups per step)
#endif
#ifndef FGRP
#define FGRP 4  // walk steps per group of the maxConcurrent == 1 fast path (their reads issue together)
#endif
#define CAPMAX 1024  // capacities are clamped: a lane's rank is < OWGS_WL
#ifndef LW_Q
#define LW_Q 2  // walk steps each lane probes per round of a wave-cooperative long walk (2 vs 4: 35.4 vs 36.1 ms
                // headline, 130 vs 137 ms configs[1], 222 vs 229 ms C5 shard 0 of 8; round 2)
#endif

// diagnostic build (-DOWGS_PROFILE, libowgs_prof.so): s_memtime cycle accounting per engine phase into stats[8..15]
#if defined(OWGS_PROFILE) || defined(OWGS_TRACE) || defined(OWGS_EXT_PROF)
// a timestamp the compiler can neither merge with another nor move out of its branch
__device__ __forceinline__ unsigned long long memtime_pinned() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#endif
#ifdef OWGS_PROFILE
#define PT_DECL                 \
    u64 pt_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; \
    u64 pw_c[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; \
    u64 pt_x[3] = {0, 0, 0};                  \
    u64 pt_y[2] = {0, 0};                     \
    u64 sc_prof_q = 0;                        \
    u64 pt_t = memtime_pinned(); \
    int pt_on = 1;
#define PT(k)                                        \
    {                                                \
        const u64 _t = memtime_pinned();             \
        if (pt_on) pt_acc[k] += _t - pt_t;           \
        pt_t = _t;                                   \
    }
#else
#define PT_DECL
#define PT(k)
#endif

// LDS scalars
#define SC_LMIN 0   // [2] first lane not known to fit (pass parity)
#define SC_IRR 2    // explicit releases (owgs_process_batch): an entry got more releases than its operationCount
#define SC_RRISK 3  // owgs_process_batch: some slot could leave the permit range through the call's releases
#define SC_U0 4     // upper bound of usable permits, managed pool
#define SC_U1 5     // blackbox pool
#define SC_USED 6   // non-empty concurrency-table entries (live + deleted)
#define SC_NLIVE 7  // table rebuild: live entries
#define SC_NHOT 8   // multi-lane actions of the current chunk (hot slots claimed)
#define SC_CBWD 9   // 1 + the chunk that moved a concurrent action's HBM walk cursor backward (forced acquire)
#define SC_OVF 13   // overflow-table entries (live + deleted), mirror of A.ovf.cnt[0]
#define SC_CLAST 12  // primary entries (live) right after the last table rebuild
#define SC_LQN 10   // long walks queued in this pass
#define SC_LQH 11   // next queued long walk to take
#define SC_LFIN 14  // pass limit after the in-pass re-decisions (OWGS_EXT)
#define SC_NEXT 15  // re-decisions in this pass
// [2][CFT_N] per pass parity and hashed fqn@version key: the first lane of the pass with a concurrent forced acquire
// of that key (its new container's free slots can only change the walks of lanes with the same key, NS:57-82)
#define SC_CFT (16 + 10 * OWGS_EW)
#ifndef CFT_LOG2
#define CFT_LOG2 6
#endif
#define CFT_N (1 << CFT_LOG2)
#define SC_N (SC_CFT + 2 * CFT_N)

// hot actions: every action with >= HOT_MIN lanes in a chunk gets a slot (assigned by the pre-pass; a concurrent
// action only when no lane of the chunk shares its fqn@version with another action); per pass one wave walks its
// capacity prefix once and writes the target of each rank 0..HOT_RANKS-1 into the slot's table, so the action's
// lanes do not walk one by one.  The rec "ext" field holds the slot (maxConcurrent == 1: slot or OWGS_REC_NOHOT;
// maxConcurrent > 1: pk1 + 1 <= OWGS_WL, or HOT_CONC + slot)
#ifndef NHOT
#define NHOT 16
#endif
#define HOT_RANKS 64
#ifndef HOT_MIN
#define HOT_MIN 6
#endif
#define HOT_CONC 0x3E0
#ifndef HOT_CONC_ON
#define HOT_CONC_ON 0  // concurrent hot tables: measured slower (their walks re-run every pass), kept as an option
#endif
static_assert(OWGS_WL < HOT_CONC, "pk1 and the concurrent hot marker share the 10-bit ext field");
#define OWGS_WROWS ((OWGS_WL + 63) / 64)  // wave rows the I/O wave stages per chunk
// a chunk of len lanes is spread evenly over the engine waves: wave w holds record positions
// [wave_off(len, w), wave_off(len, w) + wave_cap(len, w)) in its lanes 0.. (positions stay dense below len)
__host__ __device__ inline int wave_cap(int len, int w) {
    const int b = len / OWGS_EW, r = len % OWGS_EW;
    return min(OWGS_LPW, b + (w < r ? 1 : 0));
}
__host__ __device__ inline int wave_off(int len, int w) {
    const int b = len / OWGS_EW, r = len % OWGS_EW;
    return w * b + min(w, r);
}

// ------------------------------------------------------------------------------------------------ helpers
__device__ __forceinline__ u64 splitmix64(u64 x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

// Counter RNG replacing ThreadLocalRandom.nextInt(|H|) (SCPB:421); identical to oracle/owsched_oracle.c
__device__ __forceinline__ uint32_t rng_index(u64 seed, u64 seq, uint32_t n) {
    u64 u = splitmix64(seed ^ (seq * 0x9E3779B97F4A7C15ULL)) >> 32;
    return (uint32_t)((u * (u64)n) >> 32);
}

__device__ __forceinline__ int ffs64(u64 m) { return __ffsll((long long)m) - 1; }

// DPP (GFX9 row_shr / row_bcast) wave64 scans: no LDS round trip
template <int CTRL, int ROWM>
__device__ __forceinline__ int dpp_add_src(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWM, 0xf, true);  // out-of-row / masked lanes read 0
}
__device__ __forceinline__ int wave_incl_scan(int v) {
    v += dpp_add_src<0x111, 0xf>(v);  // row_shr:1
    v += dpp_add_src<0x112, 0xf>(v);  // row_shr:2
    v += dpp_add_src<0x114, 0xf>(v);  // row_shr:4
    v += dpp_add_src<0x118, 0xf>(v);  // row_shr:8
    v += dpp_add_src<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
    v += dpp_add_src<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
    return v;
}
template <int CTRL, int ROWM>
__device__ __forceinline__ int dpp_keep(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWM, 0xf, false);  // invalid source lanes keep `old`
}
__device__ __forceinline__ int wave_incl_max(int v) {
    const int I = (int)0x80000000;
    v = max(v, dpp_keep<0x111, 0xf>(I, v));
    v = max(v, dpp_keep<0x112, 0xf>(I, v));
    v = max(v, dpp_keep<0x114, 0xf>(I, v));
    v = max(v, dpp_keep<0x118, 0xf>(I, v));
    v = max(v, dpp_keep<0x142, 0xa>(I, v));
    v = max(v, dpp_keep<0x143, 0xc>(I, v));
    return v;
}
__device__ __forceinline__ int wave_max(int v) {
    const int I = (int)0x80000000;
    v = max(v, dpp_keep<0x111, 0xf>(I, v));
    v = max(v, dpp_keep<0x112, 0xf>(I, v));
    v = max(v, dpp_keep<0x114, 0xf>(I, v));
    v = max(v, dpp_keep<0x118, 0xf>(I, v));
    v = max(v, dpp_keep<0x142, 0xa>(I, v));
    v = max(v, dpp_keep<0x143, 0xc>(I, v));
    return __builtin_amdgcn_readlane(v, 63);
}

// interleaved {key, value} table (engine LDS).  One aligned block of 4 entries: 1 = key found (*val, *idx),
// 0 = an empty entry ends the chain, 2 = the chain continues in the next block.
__device__ __forceinline__ int ct_block(uint4 e01, uint4 e23, uint32_t key, uint32_t h, uint32_t* val, int* idx) {
    // branch-free: a key of the chain always sits before the chain's first empty entry
    const bool h0 = e01.x == key, h1 = e01.z == key, h2 = e23.x == key, h3 = e23.z == key;
    const bool z = e01.x == 0u || e01.z == 0u || e23.x == 0u || e23.z == 0u;
    const bool hit = h0 || h1 || h2 || h3;
    const uint32_t v = h0 ? e01.y : h1 ? e01.w : h2 ? e23.y : e23.w;
    const int k = h0 ? 0 : h1 ? 1 : h2 ? 2 : 3;
    *val = hit ? v : 0u;
    *idx = hit ? (int)h + k : -1;
    return hit ? 1 : (z ? 0 : 2);
}
// lookup from block h (a home, or the block after one that did not end the chain); index or -1, *val (0 if absent)
__device__ __forceinline__ int ct_findv_from(const uint2* ct, uint32_t key, uint32_t h, uint32_t* val) {
    int idx = -1;
    *val = 0u;
    for (int p = 0; p < OWGS_CTC / CT_BLK; ++p) {
        const uint4 e01 = *(const uint4*)&ct[h];
        const uint4 e23 = *(const uint4*)&ct[h + 2];
        const int st = ct_block(e01, e23, key, h, val, &idx);
        if (st != 2) return st == 1 ? idx : -1;
        h = (h + CT_BLK) & (OWGS_CTC - 1);
    }
    *val = 0u;
    return -1;
}
__device__ __forceinline__ int ct_findv(const uint2* ct, uint32_t key, uint32_t* val) {
    return ct_findv_from(ct, key, ct_home(key), val);
}
// find-or-insert with block reads: the key's index, inserting it into the first deleted or empty entry of its chain
// when absent (concurrent inserters of different keys race by CAS and rescan); *fresh = a new entry took an empty one
__device__ __forceinline__ int ct_upsertv(uint2* ct, uint32_t key, int* fresh) {
    *fresh = 0;
    for (int attempt = 0; attempt < OWGS_CTC; ++attempt) {
        uint32_t h = ct_home(key);
        int freei = -1;
        uint32_t freek = 0;
        bool ended = false;
        for (int p = 0; p < OWGS_CTC / CT_BLK && !ended; ++p) {
            const uint4 e01 = *(const uint4*)&ct[h];
            const uint4 e23 = *(const uint4*)&ct[h + 2];
            const uint32_t ks[4] = {e01.x, e01.z, e23.x, e23.z};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (ended) break;
                if (ks[q] == key) return (int)h + q;
                if (ks[q] == 0u || ks[q] == OWGS_CT_TOMB) {
                    if (freei < 0) {
                        freei = (int)h + q;
                        freek = ks[q];
                    }
                    if (ks[q] == 0u) ended = true;  // the key is absent
                }
            }
            h = (h + CT_BLK) & (OWGS_CTC - 1);
        }
        if (freei < 0) return -1;  // full
        if (atomicCAS((uint32_t*)&ct[freei], freek, key) == freek) {
            *fresh = freek == 0u;
            return freei;
        }
        // lost the entry to another inserter: rescan (the key may have been inserted by nobody else: it is this
        // lane's group)
    }
    return -1;
}
__device__ __forceinline__ int ct_insertv(uint2* ct, uint32_t key, int* fresh) {
    uint32_t h = ct_home(key);
    for (int p = 0; p < OWGS_CTC;) {
        const uint32_t k = ct[h].x;
        if (k == 0 || k == OWGS_CT_TOMB) {
            if (atomicCAS((uint32_t*)&ct[h], k, key) == k) {
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

// engine lookups over both tables: index < OWGS_CTC = primary (LDS), OWGS_CTC + j = overflow entry j
__device__ __forceinline__ int ct_find2(const uint2* ct, const OwgsOvf& O, bool ovf_on, uint32_t key,
                                        uint32_t* val) {
    int i = ct_findv(ct, key, val);
    if (i < 0 && ovf_on) {
        const int j = ovf_find(O, key, val);
        i = j >= 0 ? OWGS_CTC + j : -1;
    }
    return i;
}
// resolve a lookup whose first primary block was read already: st = ct_block's result (1 hit, 0 absent from the
// primary, 2 chain continues)
__device__ __forceinline__ int ct_resolve2(const uint2* ct, const OwgsOvf& O, bool ovf_on, int st, uint32_t key,
                                           uint32_t h, uint32_t* val, int ci) {
    if (st == 2) ci = ct_findv_from(ct, key, (h + CT_BLK) & (OWGS_CTC - 1), val);
    if (ci < 0 && ovf_on) {
        const int j = ovf_find(O, key, val);
        ci = j >= 0 ? OWGS_CTC + j : -1;
    }
    return ci;
}

// min(floor(pv / m), CAPMAX) for pv >= 0, 0 when pv < m; float reciprocal + one correction (pv / m < 2^10)
__device__ __forceinline__ int cap_of(int pv, int m, float rm) {
    if (pv < m) return 0;
    if (pv >= m * CAPMAX) return CAPMAX;
    int q = (int)((float)pv * rm);
    const int r = pv - q * m;
    if (r < 0) --q;
    else if (r >= m) ++q;
    return q;
}

// x mod n for 0 <= x < 2^31, 1 <= n < 2^15 without an integer division: float reciprocal, then exact correction
__device__ __forceinline__ int mod_fast(int x, int n, float rn) {
    const int q = (int)((float)x * rn);  // |q - x / n| <= 2 for x < 2^31, n < 2^15
    int r = x - q * n;
    r += r < 0 ? n : 0;
    r += r < 0 ? n : 0;
    r -= r >= n ? n : 0;
    r -= r >= n ? n : 0;
    return r;
}

// branch-free cap_of (float reciprocal + one correction); pv may be negative (forced acquires)
__device__ __forceinline__ int cap_bf(int pv, int m, float rm) {
    int q = (int)((float)max(pv, 0) * rm);
    const int r = pv - q * m;
    q += r >= m ? 1 : 0;
    q -= r < 0 ? 1 : 0;
    q = min(q, CAPMAX);
    return pv >= m ? q : 0;
}

// LDS-DMA (global_load_lds): each lane's 16 (4) bytes land at lds_dst + 16 (4) * lane.  M0 is compiler-reserved:
// saved and restored inside the statement (cdna_hip_programming.md section 5.7).  The issuing wave must wait
// vmcnt before a barrier that publishes the bytes.
__device__ __forceinline__ void lds_dma16(const void* gsrc, uint32_t lds_dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
}
__device__ __forceinline__ void lds_dma4(const void* gsrc, uint32_t lds_dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
}

// same, L1 bypassed (sc1): the walk cursors are re-read while this CU's engine waves store them
__device__ __forceinline__ void lds_dma4_l2(const void* gsrc, uint32_t lds_dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off sc1\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
}

// ------------------------------------------------------------------------------------------------ LDS layout
#define OWGS_NSTG 3  // chunk staging buffers
struct OwgsLayout {
    uint32_t P, pool, pc, ccw, ct, stgA, stgX, stgL, stgC, fst, spt, hdir, htab, hscr, bhead, nextl, spc, cdirty, skey, lq, fxa, rc, sc,
        uni, uni_bytes, total;
};

__host__ __device__ inline OwgsLayout owgs_layout(int n_slots, int pool_mode, int n_ids, int nm, int nb, int n_actions) {
    OwgsLayout L;
    uint32_t o = 0;
#define OWGS_AL(x) (((uint32_t)(x) + 15u) & ~15u)
    const uint32_t words = (uint32_t)(n_ids + 31) / 32;
    L.P = o;
    o += OWGS_AL(4u * (uint32_t)n_slots);
    L.pool = o;
    o += pool_mode ? OWGS_AL(2u * (uint32_t)(nm + nb)) : OWGS_AL(4u * words);
    L.pc = o;  // identity pools: usable ids before each bitmap word (rank/select for the fallback)
    o += pool_mode ? 0u : OWGS_AL(4u * (words + 1));
    (void)n_actions;  // per-action state lives in HBM (walk cursors: A.gcur)
    L.ccw = o;        // per chunk: walk cursor + committed lanes of each action, at its first lane
    o += 4u * OWGS_WL;
    L.ct = o;
    o += 8u * OWGS_CTC;
    L.stgA = o;  // records, lane indices and release slots of 3 chunks (g, g+1 staged, g+2 streaming in)
    o += OWGS_NSTG * OWGS_WL * 16u;
    L.stgX = o;
    o += OWGS_NSTG * OWGS_WL * 4u;
    L.stgL = o;
    o += OWGS_NSTG * OWGS_WL * 4u;
    L.stgC = o;  // HBM walk cursors of chunks g and g+1, gathered by the I/O wave
    o += 2u * OWGS_WL * 4u;
    L.sc = o;
    o += 4u * SC_N;
    // phase union: acquire phase {fst, spt, hot directory, hot rank tables, hot scratch} / release phase {rc}
    L.uni = o;
    L.fst = o;
    L.spt = o + 4u * OWGS_NBK;
    L.hdir = L.spt + 4u * OWGS_WL;                  // NHOT x {action, meta.x, meta.y, slot}, NHOT x max occ, NHOT x flag
    L.htab = L.hdir + 24u * NHOT;                   // NHOT x HOT_RANKS x {id | kind << 15 | ks << 18, step}
    L.hscr = L.htab + 8u * NHOT * HOT_RANKS;        // (OWGS_EW + 1) x 64 rank marks (the I/O wave walks hot slots too)
    L.bhead = L.hscr + 4u * 64 * (OWGS_EW + 1);     // per pass: lanes of each bucket (list head, lane + 1)
    L.nextl = L.bhead + 4u * OWGS_NBK;              // next lane of the bucket list (lane + 1, 0 = end)
    L.spc = L.nextl + 4u * OWGS_WL;                 // memory each lane tentatively takes at its target
    L.cdirty = L.spc + 4u * OWGS_WL;                // [2][OWGS_WL] pass parity x first lane of an action: re-speculated
    L.skey = L.cdirty + 8u * OWGS_WL;               // per lane {slot key, action} (shared-key check)
    L.lq = L.skey + 8u * OWGS_WL;                   // long-walk queue: {record | rank, step, position, cum} / result
    L.fxa = L.lq + 16u * OWGS_WL;                  // per lane: validation summary / in-pass re-decision (OWGS_EXT)
    L.rc = o;
    const uint32_t ua = (L.fxa - o) + 16u * OWGS_WL, ur = 4u * OWGS_CTC;
    L.uni_bytes = ua > ur ? ua : ur;
    o += L.uni_bytes;
    L.total = o;
#undef OWGS_AL
    return L;
}

extern "C" size_t OWGS_GEOM(owgs_engine_lds_bytes)(int n_slots, int pool_mode, int n_ids, int nm, int nb, int n_actions) {
    return owgs_layout(n_slots, pool_mode, n_ids, nm, nb, n_actions).total;
}

// ------------------------------------------------------------------------------------------------ hashing
__device__ __forceinline__ uint32_t pow31(uint32_t k) {
    uint32_t r = 1, b = 31;
    while (k) {
        if (k & 1) r *= b;
        b *= b;
        k >>= 1;
    }
    return r;
}

__device__ __forceinline__ uint32_t wave_java_hash(const char* bytes, int b, int e, int lane) {
    const int L = e - b;
    uint32_t acc = 0;
    for (int i = lane; i < L; i += 64) acc += (uint32_t)(uint8_t)bytes[b + i] * pow31((uint32_t)(L - 1 - i));
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) acc += (uint32_t)__shfl_xor((int)acc, d, 64);
    return acc;
}

__global__ __launch_bounds__(256) void owgs_hash_kernel(OwgsHashArgs a) {
    const int w = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int lane = threadIdx.x & 63;
    if (w >= a.n) return;
    const uint32_t h1 = wave_java_hash(a.ns_bytes, a.ns_off[w], a.ns_off[w + 1], lane);
    int32_t out;
    if (a.raw) {
        out = (int32_t)h1;
    } else {
        const uint32_t h2 = wave_java_hash(a.path_bytes, a.path_off[w], a.path_off[w + 1], lane);
        const int32_t x = (int32_t)(h1 ^ h2);
        out = x < 0 ? (int32_t)(0u - (uint32_t)x) : x;  // Int.abs: MinValue stays MinValue
    }
    if (lane == 0) a.out[w] = out;
}

__global__ __launch_bounds__(256) void owgs_lookup_kernel(OwgsLookupArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t key = ct_key(a.inv[i], a.slot[i]);
    const int ix = ct_find(a.ct_keys, key);
    uint32_t v = ix >= 0 ? a.ct_vals[ix] : 0u;
    const bool found = ix >= 0 || (a.ovf.cap > 0 && *a.ovf.cnt > 0 && ovf_find(a.ovf, key, &v) >= 0);
    a.out[i] = found ? make_int2((int)(v & OWGS_CT_C_MASK), ct_ops(v)) : make_int2(-1, 0);  // x = -1: absent
}

// home/step selection (SCPB:266-268) -> packed action meta
__global__ __launch_bounds__(256) void owgs_prepare_kernel(OwgsPrepArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const int pool = a.bb[i] ? 1 : 0;
    const int n = pool ? a.nb : a.nm;
    const int k = pool ? a.n_bsteps : a.n_msteps;
    const int32_t* steps = pool ? a.bsteps : a.msteps;
    uint32_t y = (uint32_t)a.mem[i] | ((uint32_t)a.maxc[i] << OWGS_AM_MAXC_SHIFT);
    int home = 0, step = 0;
    if (n <= 0) {
        y |= OWGS_AM_EMPTY;
    } else if (k <= 0) {
        y |= OWGS_AM_THROW;
    } else {
        const int h = a.hash[i];
        home = h % n;
        const int si = h % k;
        if (si < 0 || home < 0) y |= OWGS_AM_THROW;  // Vector.apply(negative) throws (SCPB:268 / 411)
        else step = steps[si] % n;                    // same walk; lets the engine advance with one conditional subtract
    }
    uint32_t x = (uint32_t)home | ((uint32_t)step << 15) | (pool ? OWGS_AM_POOL : 0u);
    if (a.cursor_ok[i]) x |= OWGS_AM_COK;
    a.act_meta[i] = make_uint2(x, y);
}

// ------------------------------------------------------------------------------------------------ pre-pass
// first chunk of each batch: cstart[b] = sum over b' < b of ceil(n_b' / cw), cw = the replay's chunk width
__global__ __launch_bounds__(64) void owgs_chunks_kernel(const int64_t* acq_off, int32_t n_batches, int32_t cw,
                                                         int32_t* cstart) {
    if (threadIdx.x != 0) return;
    int32_t c = 0;
    for (int b = 0; b < n_batches; ++b) {
        cstart[b] = c;
        const int64_t n = acq_off[b + 1] - acq_off[b];
        c += (int32_t)((n + cw - 1) / cw);
    }
    cstart[n_batches] = c;
}

// one workgroup per chunk: occ (earlier lanes of the same action), next lane of the same action, nearest earlier
// lane with the same slot key and a different action (shared fqn@version), packed with the action meta.
// Lanes are grouped by action and by slot key through two small LDS hash tables; each group is identified by its
// first lane and holds a bit mask of its lanes, so every rank above is a popcount or a bit search over OWGS_WL bits
// (the all-pairs scans this replaces cost O(chunk) per lane: 70 us for one full chunk, the pre-pass latency of a
// small shim call).
#define PP_HT (2 * OWGS_WL)  // hash slots per table (load <= 1/2)
__device__ __forceinline__ uint32_t pp_hash(int32_t k) { return ((uint32_t)k * 2654435761u) >> 16; }
// first lane of the group of key k: the entry's key by CAS, then the group's first lane by atomicMin (two phases with
// a barrier between, done by the caller); returns the table slot
__device__ __forceinline__ int pp_insert(int32_t* hk, int32_t k) {
    uint32_t h = pp_hash(k) % PP_HT;
    for (;;) {
        const int32_t prev = atomicCAS(&hk[h], (int32_t)0x80000000, k);
        if (prev == (int32_t)0x80000000 || prev == k) return (int)h;
        h = h + 1 == PP_HT ? 0 : h + 1;
    }
}

__global__ __launch_bounds__(OWGS_WL) void owgs_prepass_kernel(OwgsPrepassArgs A) {
    constexpr int NWR = (OWGS_WL + 63) / 64;
    if (A.geom != OWGS_GEOM_TAG(OWGS_WL)) return;  // (uniform) another geometry's buffers: write nothing
    __shared__ __align__(16) int32_t s_a[OWGS_WL], s_s[OWGS_WL], s_p[OWGS_WL];
    __shared__ int32_t hk_a[PP_HT], hl_a[PP_HT], hk_s[PP_HT], hl_s[PP_HT];
    __shared__ unsigned long long m_a[OWGS_WL][NWR], m_s[OWGS_WL][NWR];  // lane masks, by the group's first lane
    __shared__ int32_t sh_a[OWGS_WL];  // per action group: some lane has a shared-key lane before it (pk1 != 0)
    const int g = blockIdx.x;
    int b = -1, gb = 0;  // the chunk's batch and that batch's first chunk
    if (A.cstart) {
        if (g >= A.cstart[A.n_batches]) return;
        int lo = 0, hi = A.n_batches - 1;  // last batch with cstart[b] <= g
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (A.cstart[mid] <= g) lo = mid;
            else hi = mid - 1;
        }
        b = lo;
        gb = A.cstart[b];
    } else {  // a few batches (a shim call's runs): their chunk counts walked here, no chunk-table launch before
        for (int bb = 0; bb < A.n_batches; ++bb) {
            const int nc = (int)((A.acq_off[bb + 1] - A.acq_off[bb] + A.cw - 1) / A.cw);
            if (g < gb + nc) {
                b = bb;
                break;
            }
            gb += nc;
        }
        if (b < 0) return;
    }
    const int64_t c0 = A.acq_off[b] + (int64_t)(g - gb) * A.cw;
    const int len = (int)min((int64_t)A.cw, A.acq_off[b + 1] - c0);
    const int t = threadIdx.x;
    uint2 meta = make_uint2(0, 0);
    int a = -1, slot = 0;
    if (t < len) {
        if (A.act) {
            a = A.act[c0 + t];
            meta = A.act_meta[a];
            slot = A.act_slot[a];
        } else {
            meta = A.xmeta[c0 + t];
            slot = A.xslot[c0 + t];
        }
    }
    const int aid = (A.act && t < len) ? a : -1 - t;  // explicit walks: every lane is its own walk
    s_a[t] = aid;
    s_s[t] = slot;
    for (int i = t; i < PP_HT; i += OWGS_WL) {
        hk_a[i] = hk_s[i] = (int32_t)0x80000000;
        hl_a[i] = hl_s[i] = OWGS_WL;
    }
    for (int i = t; i < OWGS_WL * NWR; i += OWGS_WL) {
        (&m_a[0][0])[i] = 0ull;
        (&m_s[0][0])[i] = 0ull;
    }
    sh_a[t] = 0;
    __syncthreads();
    int ha = 0, hs_ = 0;
    if (t < len) {
        ha = pp_insert(hk_a, aid);
        hs_ = pp_insert(hk_s, slot);
    }
    __syncthreads();
    if (t < len) {
        atomicMin(&hl_a[ha], t);
        atomicMin(&hl_s[hs_], t);
    }
    __syncthreads();
    const int lead = t < len ? hl_a[ha] : t;  // first lane of the chunk with this lane's action
    const int slead = t < len ? hl_s[hs_] : t;
    const unsigned long long bit = 1ull << (t & 63);
    if (t < len) {
        atomicOr(&m_a[lead][t >> 6], bit);
        atomicOr(&m_s[slead][t >> 6], bit);
    }
    __syncthreads();
    int occ = 0, next = (int)OWGS_REC_NONEXT, pk1 = 0, cnt = 0;
    if (t < len) {
        const int tw = t >> 6;
        const unsigned long long below = bit - 1ull;
#pragma unroll
        for (int w = 0; w < NWR; ++w) {
            const unsigned long long ma = m_a[lead][w];
            // lanes with the same slot key under another action (the same action implies the same key)
            const unsigned long long mo = m_s[slead][w] & ~ma;
            cnt += __popcll(ma);
            if (w < tw) {
                occ += __popcll(ma);
                if (mo) pk1 = 64 * w + 63 - __builtin_clzll(mo) + 1;
            } else if (w == tw) {
                occ += __popcll(ma & below);
                const unsigned long long mb = mo & below;
                if (mb) pk1 = 64 * w + 63 - __builtin_clzll(mb) + 1;
                const unsigned long long ab = ma & ~(below | bit);
                if (ab) next = 64 * w + __builtin_ctzll(ab);
            } else if (next == (int)OWGS_REC_NONEXT && ma) {
                next = 64 * w + __builtin_ctzll(ma);
            }
        }
    }
    // hot actions (>= HOT_MIN lanes in the chunk; concurrent ones only without a shared-key lane): slots in order of
    // their first lane
    const int mc = (int)((meta.y >> OWGS_AM_MAXC_SHIFT) & OWGS_AM_MAXC_MASK);
    s_p[t] = pk1;
    if (t < len && pk1 != 0) sh_a[lead] = 1;  // (a plain store: every writer writes 1)
    __syncthreads();
    const bool shared = t < len && mc > 1 && sh_a[lead] != 0;
    const bool q = t < len && A.act && cnt >= HOT_MIN && !shared && !(meta.y & (OWGS_AM_THROW | OWGS_AM_EMPTY)) &&
                   (mc == 1 || HOT_CONC_ON);
    // qualifying leaders as a lane mask: an action's hot slot = the qualifying leaders before its first lane
    __shared__ unsigned long long m_q[NWR];
    {
        const unsigned long long mq = __ballot(q && occ == 0);
        if ((t & 63) == 0) m_q[t >> 6] = mq;
    }
    __syncthreads();
    int hs = OWGS_REC_NOHOT;
    if (q) {
        int k = 0;
#pragma unroll
        for (int w = 0; w < NWR; ++w) {
            if (w < (lead >> 6)) k += __popcll(m_q[w]);
            else if (w == (lead >> 6)) k += __popcll(m_q[w] & ((1ull << (lead & 63)) - 1ull));
        }
        if (k < NHOT) hs = k;
    }
    // record position by class: 0 = walks of maxConcurrent == 1 actions, 1 = no walk of its own (hot-table rank,
    // throwing index, empty pool), 2 = concurrent walks; stream order inside a class.  A wave then mostly runs one
    // speculation path, and the class-1 lanes sit between the two walking classes.
    const int cls = (hs != OWGS_REC_NOHOT || (meta.y & (OWGS_AM_THROW | OWGS_AM_EMPTY))) ? 1 : (mc > 1 ? 2 : 0);
    s_p[t] = t < len ? cls : 3;
    // class masks (one ballot per wave and class): thread 0's dealing below walks set bits in registers instead of
    // re-reading every lane's class from LDS in each of its loops
    __shared__ unsigned long long s_m[3][(OWGS_WL + 63) / 64];
    __shared__ int s_cnt[OWGS_EW], s_cap[OWGS_EW];
    {
        const unsigned long long m0 = __ballot(t < len && cls == 0), m1 = __ballot(t < len && cls == 1),
                                 m2 = __ballot(t < len && cls == 2);
        if ((t & 63) == 0) {
            s_m[0][t >> 6] = m0;
            s_m[1][t >> 6] = m1;
            s_m[2][t >> 6] = m2;
        }
    }
    __syncthreads();
    // Mode 1 (large pools) in parallel: concurrent lanes round-robin over the fewest back waves that hold them,
    // walkers round-robin over the front waves, walk-free lanes into the free slots from wave 0 up.  Every thread
    // places its own lane from its class rank; this is exactly what the serial dealing below does whenever no wave
    // fills up before its last round-robin turn (checked here; otherwise, and for the other modes, thread 0 deals).
    bool dealt = false;
    if (A.deal == 1) {
        constexpr int NWR = (OWGS_WL + 63) / 64;
        int nc[3] = {0, 0, 0};
#pragma unroll
        for (int c = 0; c < 3; ++c)
            for (int r = 0; r < NWR; ++r) nc[c] += __popcll(s_m[c][r]);
        int nwv = 0;
        for (int w = 0; w < OWGS_EW; ++w) nwv += wave_cap(len, w) > 0;
        int f2 = 0, acc2 = 0;
        while (f2 < nwv && acc2 < nc[2]) acc2 += wave_cap(len, nwv - 1 - f2++);
        const int sp0 = nwv - f2, lo2 = nwv - f2;
        // lanes of a class dealt round-robin from wave lo over span waves: wave lo + i gets ceil((n - i) / span)
        auto rr_count = [](int n, int i, int span) { return (span > 0 && n > i) ? (n - i - 1) / span + 1 : 0; };
        bool ok = sp0 >= 1;
        int used[OWGS_EW];
#pragma unroll
        for (int w = 0; w < OWGS_EW; ++w) {
            used[w] = w < sp0 ? rr_count(nc[0], w, sp0) : (w < nwv ? rr_count(nc[2], w - lo2, f2) : 0);
            ok = ok && used[w] <= wave_cap(len, w);
        }
        if (ok) {
            dealt = true;
            if (t < len) {
                const int c = cls;
                const int row = t >> 6;
                int k = 0;  // class rank: lanes of class c before t
                for (int r = 0; r < row; ++r) k += __popcll(s_m[c][r]);
                const unsigned long long below = s_m[c][row] & ((1ull << (t & 63)) - 1ull);
                k += __popcll(below);
                int w = 0, slot = 0;
                if (c == 0) {
                    w = k % sp0;
                    slot = k / sp0;
                } else if (c == 2) {
                    w = lo2 + k % f2;
                    slot = k / f2;
                } else {  // the k-th free slot in wave order
                    int pre = 0;
#pragma unroll
                    for (int v = 0; v < OWGS_EW; ++v) {
                        const int fr = wave_cap(len, v) - used[v];
                        if (k >= pre && k < pre + fr) {
                            w = v;
                            slot = used[v] + (k - pre);
                        }
                        pre += fr;
                    }
                }
                s_s[t] = wave_off(len, w) + slot;
            }
        }
    }
    if (t == 0 && !dealt) {
        constexpr int NWR = (OWGS_WL + 63) / 64;
        // f(j) for every lane j of class c, in stream order (masks and the per-wave counters below live in LDS:
        // indexed by runtime values, a thread-private array would sit in scratch memory)
        auto each = [&](int c, auto&& f) {
            for (int r = 0; r < NWR; ++r)
                for (unsigned long long m = s_m[c][r]; m; m &= m - 1) f(r * 64 + __builtin_ctzll(m));
        };
        // the maxConcurrent == 1 walkers fill the first waves; the concurrent lanes are spread round-robin over the
        // remaining waves and the lanes without a walk fill the gaps (from the last wave down), so the waves that
        // run the concurrent path hold fewer of them (a wave takes as long as its slowest lane).  Wave w holds
        // positions [wave_off(len, w), + wave_cap(len, w)): the chunk spread evenly, positions dense below len.
        int* cnt = s_cnt;
        int* cap = s_cap;
        int n0 = 0, nwv = 0;
        for (int w = 0; w < OWGS_EW; ++w) {
            cnt[w] = 0;
            cap[w] = wave_cap(len, w);
            nwv += cap[w] > 0;
        }
        int n1 = 0, n2 = 0;
        for (int r = 0; r < NWR; ++r) {
            n0 += __popcll(s_m[0][r]);
            n1 += __popcll(s_m[1][r]);
            n2 += __popcll(s_m[2][r]);
        }
        // place the class-c lanes round-robin over waves [wlo, whi) (skipping full ones), spilling anywhere
        auto deal = [&](int c, int wlo, int whi) {
            int rr = 0;
            const int span = max(whi - wlo, 1);
            each(c, [&](int j) {
                int w = -1;
                for (int k = 0; k < span && w < 0; ++k, ++rr) {
                    const int cw_ = wlo + (rr % span);
                    if (cw_ < nwv && cnt[cw_] < cap[cw_]) w = cw_;
                }
                for (int q = nwv - 1; q >= 0 && w < 0; --q)
                    if (cnt[q] < cap[q]) w = q;
                s_s[j] = wave_off(len, w) + cnt[w]++;
            });
        };
        auto fill = [&](int c, bool from_back) {  // contiguous, first free slot
            each(c, [&](int j) {
                int w = from_back ? nwv - 1 : 0;
                if (from_back) while (cnt[w] == cap[w]) --w;
                else while (cnt[w] == cap[w]) ++w;
                s_s[j] = wave_off(len, w) + cnt[w]++;
            });
        };
        int f0 = 0, acc0 = 0;  // waves the maxConcurrent == 1 walkers fill
        while (f0 < nwv && acc0 < n0) acc0 += cap[f0++];
        // the host picks the strategy per replay (owgs_host.cpp, chunk_width): 1 for large pools, 2 for small ones
        const int mode = A.deal;
        if (mode == 1) {  // walkers and walk-free lanes share the front waves; concurrent lanes packed at the back
            int f2 = 0, acc2 = 0;
            while (f2 < nwv && acc2 < n2) acc2 += cap[nwv - 1 - f2++];
            deal(2, nwv - f2, nwv);
            deal(0, 0, max(nwv - f2, 1));
            fill(1, false);
        } else if (mode == 2) {  // every class spread over every wave
            deal(2, 0, nwv);
            deal(0, 0, nwv);
            fill(1, false);
        } else if (mode == 4 || mode == 5) {  // concurrent lanes over (2|3) x the waves they need, then walkers
            int f2 = 0, acc2 = 0;
            while (f2 < nwv && acc2 < n2) acc2 += cap[nwv - 1 - f2++];
            const int k2 = min(nwv, (mode == 4 ? 2 : 3) * f2);
            deal(2, nwv - k2, nwv);
            deal(0, 0, nwv);
            fill(1, false);
        } else if (mode == 3) {  // concurrent lanes spread over every wave, walkers from the front
            deal(2, 0, nwv);
            fill(0, false);
            fill(1, false);
        } else {
            fill(0, false);
            deal(2, f0, nwv);
            fill(1, true);
        }
        (void)n1;
    }
    __syncthreads();
    if (t >= len) return;
    const int pos = s_s[t];
    const int ext = mc > 1 ? (hs != OWGS_REC_NOHOT ? HOT_CONC + hs : pk1) : hs;  // 10 bits
    const uint32_t an = A.act ? (uint32_t)a : OWGS_REC_NOACT;
    uint4 r;
    r.x = meta.x;
    r.y = meta.y | OWGS_AM_VALID;
    r.z = an | ((uint32_t)occ << 17) | ((uint32_t)(ext & 31) << 27);
    r.w = (uint32_t)slot | ((uint32_t)next << 17) | ((uint32_t)(ext >> 5) << 27);
    A.rec[c0 + pos] = r;
    A.lix[(int64_t)g * OWGS_WL + pos] = (uint32_t)t | ((uint32_t)lead << 16);
}

// Release bookkeeping: relx[aid] = the position of the activation's release record, inside its release batch's range
// (rel_aid is grouped by release batch, so the engine reads batch b's records rel_rec[rel_off[b] .. rel_off[b+1])
// contiguously).  An
// activation released twice, or a release id outside the stream, is a malformed stream (the reference's
// activationSlots.remove would find no entry the second time, CLB:278-279; replays take CommonLoadBalancer's streams).
// Inside batch b's range the records are placed by class: releases of maxConcurrent == 1 actions from the front
// (relcnt[b] of them), concurrent ones from the back, so the engine's sweep runs the plain permit return over the first
// part without the concurrency-map path (order inside a batch is free: permit sums commute, and a concurrent release's
// effect depends only on its rank among the releases of its entry).  One atomic per wave and (batch, class).
#define RP_T 1024  // releases per workgroup
#define RP_W 8     // batches from the workgroup's first whose counts are aggregated in LDS (later ones: per wave)
__global__ __launch_bounds__(RP_T) void owgs_relpos_kernel(OwgsRelposArgs R) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    // the batch of each release: one search per workgroup (last batch with rel_off[b] <= first release), then a short
    // forward scan per thread (a search again past 16 steps: runs of empty batches)
    __shared__ int s_b0;
    __shared__ int s_cnt[RP_W][2], s_base[RP_W][2];
    auto last_le = [&](int64_t x) {
        int lo = 0, hi = R.n_batches - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (R.rel_off[mid] <= x) lo = mid;
            else hi = mid - 1;
        }
        return lo;
    };
    if (threadIdx.x == 0) s_b0 = last_le(min((int64_t)blockIdx.x * blockDim.x, R.n_rel - 1));
    if (threadIdx.x < 2 * RP_W) (&s_cnt[0][0])[threadIdx.x] = 0;
    __syncthreads();
    const int bw = s_b0;
    bool live = r < R.n_rel;
    int64_t aid = -1;
    int b = 0, cls = 0;
    if (live) {
        aid = R.rel_aid[r];
        if (aid < 0 || aid >= R.n_act) {
            atomicOr(R.err, OWGS_ERR_BAD_STREAM);
            live = false;
        } else {
            b = bw;
            int k = 0;
            while (k < 16 && b + 1 < R.n_batches && R.rel_off[b + 1] <= r) {
                ++b;
                ++k;
            }
            if (k == 16) b = last_le(r);
            const uint2 m = R.act_meta[R.act[aid]];
            cls = ((m.y >> OWGS_AM_MAXC_SHIFT) & OWGS_AM_MAXC_MASK) > 1 ? 1 : 0;
        }
    }
    // ranks per (batch, class): a wave's group takes its offset from an LDS counter (batches bw .. bw + RP_W - 1), then
    // one global atomic per workgroup and (batch, class) gives the group's base; later batches: a global atomic per wave
    int64_t pos = -1;
    int off = 0;
    bool local = false;
    for (u64 todo = __ballot(live); todo;) {
        const int ld = (int)__builtin_ctzll(todo);
        const int b0 = __builtin_amdgcn_readlane(b, ld);
        const bool win = b0 - bw < RP_W;
        const bool sel = live && b == b0;
        const u64 m0 = __ballot(sel && cls == 0), m1 = __ballot(sel && cls == 1);
        int base0 = 0, base1 = 0;
        if (lane == ld) {
            if (win) {
                if (m0) base0 = atomicAdd(&s_cnt[b0 - bw][0], __popcll(m0));
                if (m1) base1 = atomicAdd(&s_cnt[b0 - bw][1], __popcll(m1));
            } else {
                if (m0) base0 = atomicAdd(&R.relcnt[2 * b0], __popcll(m0));
                if (m1) base1 = atomicAdd(&R.relcnt[2 * b0 + 1], __popcll(m1));
            }
        }
        base0 = __shfl(base0, ld, 64);
        base1 = __shfl(base1, ld, 64);
        if (sel) {
            const u64 mm = cls ? m1 : m0;
            const int rk = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
            if (win) {
                local = true;
                off = (cls ? base1 : base0) + rk;
            } else {
                pos = cls ? R.rel_off[b0 + 1] - 1 - (base1 + rk) : R.rel_off[b0] + base0 + rk;
            }
        }
        todo &= ~(m0 | m1);
    }
    __syncthreads();
    if (threadIdx.x < 2 * RP_W) {
        const int i = threadIdx.x >> 1, c = threadIdx.x & 1, n = s_cnt[i][c];
        s_base[i][c] = n ? atomicAdd(&R.relcnt[2 * (bw + i) + c], n) : 0;
    }
    __syncthreads();
    if (local) {
        const int base = s_base[b - bw][cls] + off;
        pos = cls ? R.rel_off[b + 1] - 1 - base : R.rel_off[b] + base;
    }
    if (live && aid < R.decided_below) {
        // decided by an earlier launch: the record from that decision (the engine writes the others when it decides)
        const int a = R.act[aid];
        const uint2 m = R.act_meta[a];
        const int x = R.out_inv[aid];
        const uint32_t inv15 = x >= 0 ? (uint32_t)x : OWGS_RR_NOINV;
        R.rel_rec[pos] = make_uint2(inv15 | ((m.y & OWGS_AM_MEM_MASK) << 15),
                                    (uint32_t)R.act_slot[a] | (((m.y >> OWGS_AM_MAXC_SHIFT) & OWGS_AM_MAXC_MASK) << 17));
        return;
    }
    if (live && atomicCAS(&R.relx[aid], -1, (int32_t)pos) != -1) atomicOr(R.err, OWGS_ERR_BAD_STREAM);
}

// per-release flags after a replay: the activation was never scheduled -> no ActivationEntry (CLB:278-279)
__global__ __launch_bounds__(256) void owgs_relflags_kernel(const int64_t* rel_aid, int64_t n_rel,
                                                           const int32_t* out_inv, uint8_t* rel_flags) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rel) return;
    if (out_inv[rel_aid[r]] < 0) rel_flags[r] |= (uint8_t)OWGS_REL_NOENTRY_BIT;
}

// ------------------------------------------------------------------------------------------------ engine
struct EngineCtx {
    const int32_t* P;
    const uint32_t* ub;
    const int16_t* pw;
    const uint32_t* pc;
    int pool_mode, n_ids, nm, nb;
};

// pool position -> invoker id (>= 0, usable), OWGS_PW_UNUSABLE or OWGS_PW_BADID, and the id's permits (one LDS read
// for identity pools: the usable flag is folded into the permits)
__device__ __forceinline__ int pool_probe(const EngineCtx& E, int pool, int pos, int* pv) {
    if (E.pool_mode == 0) {
        const int id = pool ? E.n_ids - E.nb + pos : pos;
        const int v = E.P[id];
        *pv = v;
        return v < OWGS_PLIM ? id : OWGS_PW_UNUSABLE;
    }
    const int id = (int)E.pw[pool ? E.nm + pos : pos];
    *pv = id >= 0 ? E.P[id] : 0;
    return id;
}

// usable ids of the identity pool [lo, lo + n) before id x
__device__ __forceinline__ int usable_before(const EngineCtx& E, int x) {
    const int w = x >> 5, b = x & 31;
    const uint32_t m = b ? (E.ub[w] & ((1u << b) - 1u)) : 0u;
    return (int)E.pc[w] + __popc(m);
}

// position of the need-th set bit (0-based) of m, need < popc(m): halving by popcounts, no loop over the bits
__device__ __forceinline__ int select_in_word(uint32_t m, int need) {
    int pos = 0;
#pragma unroll
    for (int w = 16; w >= 1; w >>= 1) {
        const int c = __popc(m & ((1u << w) - 1u));
        const bool up = need >= c;
        need -= up ? c : 0;
        m = up ? m >> w : m;
        pos += up ? w : 0;
    }
    return pos;
}

// k-th usable id (0-based) at or after id lo (identity pools): binary search over the word prefix counts
__device__ __forceinline__ int select_usable(const EngineCtx& E, int lo, int k) {
    const int target = usable_before(E, lo) + k;  // global rank of the wanted id
    int a = lo >> 5, z = (E.n_ids - 1) >> 5;       // last word w with pc[w] <= target
    while (a < z) {
        const int mid = (a + z + 1) >> 1;
        if ((int)E.pc[mid] <= target) a = mid;
        else z = mid - 1;
    }
    const uint32_t m = E.ub[a];
    const int need = target - (int)E.pc[a];
    if (need < 0 || need >= __popc(m)) return -1;  // (the host's healthy counts disagree with the bitmap)
    return (a << 5) + select_in_word(m, need);
}

// k-th usable id of a pool whose ids [lo, lo + n) are all usable (fast path), else select_usable
__device__ __forceinline__ int select_pool(const EngineCtx& E, int lo, int k, bool all_usable) {
    return all_usable ? lo + k : select_usable(E, lo, k);
}

// Workgroup barrier that orders LDS only: a plain __syncthreads() also waits for every outstanding global store of
// the wave (vmcnt(0)), which would drain the engine's decision stores and the I/O wave's prefetch at every pass.
__device__ __forceinline__ void lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// diagnostic build (-DOWGS_TRACE): every wave logs {barrier id, arrival, departure} of the pass-loop barriers into
// A.trace[wave][OWGS_TRACE_CAP] (u64 pairs), for a timeline of which wave arrives last at each barrier
#ifndef OWGS_TRACE_CAP
#define OWGS_TRACE_CAP 16384
#endif
#ifdef OWGS_TRACE
#define LDS_SYNC_T(id)                                                                               \
    {                                                                                                \
        const u64 ta_ = memtime_pinned();                                                            \
        lds_sync();                                                                                  \
        const u64 td_ = memtime_pinned();                                                            \
        if (lane == 0 && tr_n < OWGS_TRACE_CAP) {                                                    \
            A.trace[2 * ((size_t)wave * OWGS_TRACE_CAP + tr_n)] = ((u64)(id) << 56) | (ta_ & ((1ull << 56) - 1)); \
            A.trace[2 * ((size_t)wave * OWGS_TRACE_CAP + tr_n) + 1] = td_;                           \
        }                                                                                            \
        ++tr_n;                                                                                      \
    }
#define TRACE_MARK(id)                                                                               \
    {                                                                                                \
        const u64 tm_ = memtime_pinned();                                                            \
        if (lane == 0 && tr_n < OWGS_TRACE_CAP) {                                                    \
            A.trace[2 * ((size_t)wave * OWGS_TRACE_CAP + tr_n)] = ((u64)(id) << 56) | (tm_ & ((1ull << 56) - 1)); \
            A.trace[2 * ((size_t)wave * OWGS_TRACE_CAP + tr_n) + 1] = tm_;                           \
        }                                                                                            \
        ++tr_n;                                                                                      \
    }
#else
#define LDS_SYNC_T(id) lds_sync()
#define TRACE_MARK(id)
#endif

template <int FEAT>
__device__ __forceinline__ void owgs_engine_body(const OwgsEngineArgs& A) {
    // specialisation (OWGS_F_*): without F_CONC every lane is maxConcurrent == 1 (a record saying otherwise is a broken
    // stream) and the map code is gone; without F_GEN pools are identity pools and sequence numbers implicit
    constexpr bool kConc = (FEAT & OWGS_F_CONC) != 0;
    constexpr bool kGen = (FEAT & OWGS_F_GEN) != 0;
    const int pool_mode = kGen ? A.pool_mode : 0;
    const unsigned long long* const seqp = kGen ? A.seq : nullptr;
    auto conc_of = [&](uint32_t y) -> int {  // maxConcurrent field of a record's meta.y, as this specialisation sees it
        return kConc ? (int)((y >> OWGS_AM_MAXC_SHIFT) & OWGS_AM_MAXC_MASK) : 1;
    };
    // (uniform) a launch prepared for another geometry: its chunk tables have another stride -- refuse it before the
    // first barrier or wait of any wave
    // the caller's pinned words (err_host, ovf_host) on an early exit: the error word, the overflow count unchanged
    auto tail_early = [&](int e) {
        atomicOr(A.err, e);
        if (A.err_host) *A.err_host = __hip_atomic_load(A.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) | e;
        if (A.ovf_host) *A.ovf_host = A.ovf.cap > 0 ? __hip_atomic_load(A.ovf.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    };
    if (A.geom != OWGS_GEOM_TAG(OWGS_WL)) {
        if (threadIdx.x == 0) tail_early(OWGS_ERR_GEOM);
        if (A.stats_next && threadIdx.x < OWGS_NSTATS) A.stats_next[threadIdx.x] = 0ull;
        return;
    }
#ifdef OWGS_PROFILE
    const u64 tk0 = memtime_pinned();  // kernel-level cycles: state load, batches, write-back (stats[40..42])
#endif
    extern __shared__ uint4 lds_raw[];
    char* L = (char*)lds_raw;
    const OwgsLayout Y = owgs_layout(A.n_slots, pool_mode, A.n_ids, A.nm, A.nb, A.n_actions);
    int32_t* P = (int32_t*)(L + Y.P);
    uint32_t* ub = (uint32_t*)(L + Y.pool);
    int16_t* pw = (int16_t*)(L + Y.pool);
    uint32_t* pc = (uint32_t*)(L + Y.pc);
    uint32_t* ccw = (uint32_t*)(L + Y.ccw);
    const uint32_t* stgC = (const uint32_t*)(L + Y.stgC);
    uint2* ct = (uint2*)(L + Y.ct);  // interleaved {key, value}
    uint4* stgA = (uint4*)(L + Y.stgA);
    int32_t* stgX = (int32_t*)(L + Y.stgX);
    uint32_t* fst = (uint32_t*)(L + Y.fst);
    int32_t* spt = (int32_t*)(L + Y.spt);
    uint32_t* bhead = (uint32_t*)(L + Y.bhead);
    int32_t* nextl = (int32_t*)(L + Y.nextl);
    int32_t* spc = (int32_t*)(L + Y.spc);
    int32_t* cdirty = (int32_t*)(L + Y.cdirty);
    uint2* skey = (uint2*)(L + Y.skey);
    uint4* lq = (uint4*)(L + Y.lq);
    uint4* fxa = (uint4*)(L + Y.fxa);
    uint4* hdir = (uint4*)(L + Y.hdir);
    int32_t* hocc = (int32_t*)(L + Y.hdir + 16u * NHOT);
    int32_t* hflag = (int32_t*)(L + Y.hdir + 20u * NHOT);
    uint2* htab = (uint2*)(L + Y.htab);
    int32_t* hscr = (int32_t*)(L + Y.hscr);
    const uint32_t* stgL = (const uint32_t*)(L + Y.stgL);
    uint32_t* rc = (uint32_t*)(L + Y.rc);
    int32_t* sc = (int32_t*)(L + Y.sc);
#ifdef OWGS_PROFILE
    int* spw = sc + 16;
    int* pfw = sc + 16 + 4 * OWGS_EW;  // per-wave speculation timings (SC_N leaves room in every build)
#endif

    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const bool io = wave >= OWGS_EW;
    const int n_slots = A.n_slots, nm = A.nm, nb = A.nb;
    const int words = (A.n_ids + 31) >> 5;

    // ---------------------------------------------------------------- state -> LDS
    uint32_t err = 0;
    constexpr int LB = 8;  // loads in flight per thread (the state load is latency-bound)
    if (tid < SC_N)
        sc[tid] = (tid == SC_IRR || tid == SC_RRISK) ? 0
                                                     : ((tid < 4 || tid >= SC_CFT) ? OWGS_WL : (tid < 6 ? (int)0x80000000 : 0));
    if (A.rel_bound) lds_sync();  // (SC_RRISK is set below)
    bool rrisk = false;    // (owgs_process_batch) a slot the call's releases could push out of the LDS range
    // permits four slots per 16-byte load, with their usable word and (owgs_process_batch) their release bounds, all
    // issued before any is used: one round trip per 10,240 slots (the headline's state in one)
    constexpr int LB4 = 5;
    const int n4 = n_slots >> 2;
    auto slot_in = [&](int i, int v, uint32_t u, unsigned long long bnd) {
        if (v < -OWGS_PLIM || v >= OWGS_PLIM) err |= OWGS_ERR_PERMITS;
        const bool unusable = pool_mode == 0 && i < A.n_ids && !((u >> (i & 31)) & 1u);
        if (bnd) rrisk = rrisk || (long long)v + (long long)bnd >= (long long)OWGS_PLIM;
        return unusable ? v + OWGS_PENC : v;
    };
    for (int j0 = 0; j0 < n4; j0 += OWGS_NT * LB4) {
        int4 v[LB4];
        uint32_t u[LB4];
        ulonglong2 r0[LB4], r1[LB4];
#pragma unroll
        for (int k = 0; k < LB4; ++k) {
            const int j = j0 + k * OWGS_NT + tid;
            v[k] = j < n4 ? ((const int4*)A.permits)[j] : make_int4(0, 0, 0, 0);
            u[k] = (pool_mode == 0 && j < n4 && 4 * j < A.n_ids) ? A.usable[j >> 3] : ~0u;
            r0[k] = r1[k] = make_ulonglong2(0ull, 0ull);
            if (A.rel_bound && j < n4) {
                r0[k] = ((const ulonglong2*)A.rel_bound)[2 * j];
                r1[k] = ((const ulonglong2*)A.rel_bound)[2 * j + 1];
            }
        }
#pragma unroll
        for (int k = 0; k < LB4; ++k) {
            const int j = j0 + k * OWGS_NT + tid;
            if (j >= n4) continue;
            const int i = 4 * j;
            ((int4*)P)[j] = make_int4(slot_in(i, v[k].x, u[k], r0[k].x), slot_in(i + 1, v[k].y, u[k], r0[k].y),
                                      slot_in(i + 2, v[k].z, u[k], r1[k].x), slot_in(i + 3, v[k].w, u[k], r1[k].y));
            if (A.rel_bound && (r0[k].x | r0[k].y | r1[k].x | r1[k].y)) {
                ((ulonglong2*)A.rel_bound)[2 * j] = make_ulonglong2(0ull, 0ull);
                ((ulonglong2*)A.rel_bound)[2 * j + 1] = make_ulonglong2(0ull, 0ull);
            }
        }
    }
    for (int i = 4 * n4 + tid; i < n_slots; i += OWGS_NT) {  // (the last n_slots % 4 slots)
        const unsigned long long bnd = A.rel_bound ? A.rel_bound[i] : 0ull;
        P[i] = slot_in(i, A.permits[i], (pool_mode == 0 && i < A.n_ids) ? A.usable[i >> 5] : ~0u, bnd);
        if (bnd) A.rel_bound[i] = 0ull;
    }
    if (rrisk) sc[SC_RRISK] = 1;
    if (pool_mode == 0) {
        for (int i = tid; i < words; i += OWGS_NT) ub[i] = A.usable[i];
    } else {
        for (int i = tid; i < nm + nb; i += OWGS_NT) pw[i] = (int16_t)A.pool_words[i];
    }
    lds_sync();
    // releases that could leave the range: nothing has been written yet -- the host replays the call through the
    // ordered release kernels (which flag ForcibleSemaphore's overflow Error per release, FS:48-50)
    if (A.rel_bound && sc[SC_RRISK]) {  // (uniform)
        if (tid == 0) tail_early(OWGS_ERR_RELRISK);
        if (A.stats_next && tid < OWGS_NSTATS) A.stats_next[tid] = 0ull;
        return;
    }
    {
        int used = 0;
        for (int i0 = 0; i0 < OWGS_CTC; i0 += OWGS_NT * LB) {
            uint32_t kk[LB], vv[LB];
#pragma unroll
            for (int k = 0; k < LB; ++k) {
                const int i = i0 + k * OWGS_NT + tid;
                kk[k] = i < OWGS_CTC ? A.ct_keys[i] : 0u;
                vv[k] = i < OWGS_CTC ? A.ct_vals[i] : 0u;
            }
#pragma unroll
            for (int k = 0; k < LB; ++k) {
                const int i = i0 + k * OWGS_NT + tid;
                if (i >= OWGS_CTC) continue;
                ct[i] = make_uint2(kk[k], vv[k]);
                used += kk[k] != 0;
            }
        }
        if (used) atomicAdd(&sc[SC_USED], used);
        if (tid == 0 && A.ovf.cap > 0) sc[SC_OVF] = __hip_atomic_load(A.ovf.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (int i = tid; i < (int)(Y.uni_bytes / 4); i += OWGS_NT) ((uint32_t*)(L + Y.uni))[i] = 0u;
    lds_sync();
    // the table's fill after its last rebuild (an earlier launch's; fewer entries now: rebuilt elsewhere since)
    if (tid == 0 && A.ct_clast) sc[SC_CLAST] = min(*A.ct_clast, sc[SC_USED]);
    if (pool_mode == 0 && wave == 0) {  // prefix counts of the usable bitmap
        int carry = 0;
        for (int w0 = 0; w0 <= words; w0 += 64) {
            const int w = w0 + lane;
            const int c = w < words ? __popc(ub[w]) : 0;
            const int inc = wave_incl_scan(c);
            if (w <= words) pc[w] = (uint32_t)(carry + inc - c);
            carry += __builtin_amdgcn_readlane(inc, 63);
        }
    }
    EngineCtx E;
    E.P = P;
    E.ub = ub;
    E.pw = pw;
    E.pc = pc;
    E.pool_mode = pool_mode;
    E.n_ids = A.n_ids;
    E.nm = nm;
    E.nb = nb;

    uint32_t st_pass = 0, st_probe = 0, st_fb = 0, st_long = 0, st_chunk = 0, st_stop = 0, st_gprobe = 0, st_glane = 0;
    uint32_t st_ext = 0, st_pre = 0;  // in-pass re-decisions (I/O wave), of them from the lane's own pre-walk
#ifdef OWGS_EXT_PROF
    u64 xp_cyc = 0, xp_rounds = 0, xp_scans = 0, xp_ph[4] = {0, 0, 0, 0};
#endif
#ifdef OWGS_TRACE
    int tr_n = 0;
#endif
    PT_DECL

    // ---------------------------------------------------------------- I/O wave: chunk prefetch pipeline
    // While the engine resolves chunk g, the I/O wave streams the records of chunk g+2 from HBM straight into
    // stgA/stgX/stgL[(g+2)%3] by LDS-DMA (global_load_lds: no registers, nothing for the engine waves to wait on),
    // gathers the HBM walk cursors of chunk g+1's actions (staged a chunk earlier) into stgC[(g+1)&1], and drains both
    // (vmcnt(0)) before the last barrier of chunk g.
    int io_b = 0;
    int64_t io_c0 = 0;
    const uint32_t stgA_lds = (uint32_t)(size_t)stgA, stgX_lds = (uint32_t)(size_t)stgX, stgL_lds = (uint32_t)(size_t)stgL,
                   stgC_lds = (uint32_t)(size_t)stgC;
    // cursor words of the actions of the chunk staged in stgA[sb] (lanes past its end gather a valid dummy word)
    auto io_gather = [&](int sb, int cb) {
#pragma unroll
        for (int k = 0; k < OWGS_WROWS; ++k) {
            const uint32_t m0 = __builtin_amdgcn_readfirstlane(stgC_lds + (uint32_t)(cb * OWGS_WL + 64 * k) * 4u);
            if (64 * k + lane < OWGS_WL) {
                const uint32_t a = stgA[sb * OWGS_WL + 64 * k + lane].z & OWGS_REC_NOACT;
                const int ai = (int)a < A.n_actions ? (int)a : 0;
                lds_dma4_l2(&A.gcur[ai], m0);
            }
        }
    };
    // advance (io_b, io_c0) to the next chunk; returns false at the end of the stream
    auto io_locate = [&](int& bb, int64_t& c0) -> bool {
        while (bb < A.n_batches && c0 >= A.acq_off[bb + 1]) {
            ++bb;
            if (bb < A.n_batches) c0 = A.acq_off[bb];
        }
        return bb < A.n_batches;
    };
    // lanes past the end of the stream re-read its last record: the engine ignores lanes >= the chunk length
    auto io_dma = [&](int64_t c0, int buf, int gc) {
        const int64_t last = A.n_act - 1;
        const uint32_t* lx = A.lix + (int64_t)gc * OWGS_WL;
#pragma unroll
        for (int k = 0; k < OWGS_WROWS; ++k) {  // (a partial last row: its lanes past OWGS_WL stay idle)
            const uint32_t mL = __builtin_amdgcn_readfirstlane(stgL_lds + (uint32_t)(buf * OWGS_WL + 64 * k) * 4u);
            const uint32_t mA = __builtin_amdgcn_readfirstlane(stgA_lds + (uint32_t)(buf * OWGS_WL + 64 * k) * 16u);
            const uint32_t mX = __builtin_amdgcn_readfirstlane(stgX_lds + (uint32_t)(buf * OWGS_WL + 64 * k) * 4u);
            if (64 * k + lane < OWGS_WL) {
                lds_dma4(&lx[lane + 64 * k], mL);
                int64_t i = c0 + lane + 64 * k;
                i = i < last ? i : last;
                lds_dma16(&A.rec[i], mA);
                if (A.relpos) lds_dma4(&A.relpos[i], mX);
            }
        }
    };
    if (io) {
        if (A.n_batches > 0) io_c0 = A.acq_off[0];
        for (int k = 0; k < 2; ++k)
            if (io_locate(io_b, io_c0)) {
                io_dma(io_c0, k, k);
                io_c0 += A.cw;
            }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        io_gather(0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lds_sync();
#ifdef OWGS_PROFILE
    const u64 tk1 = memtime_pinned();
#endif
    // healthy invokers per pool (|H| of the overload fallback, SCPB:417-424): identity pools count them from the
    // usable bitmap (owgs_update_health_device updates only the bitmap there); other pools take the host's counts
    int hm_e = A.hm, hb_e = A.hb;
    auto rank = [&](int x) {  // usable ids below x (identity pools)
        return x <= 0 ? 0 : (int)pc[x >> 5] + ((x & 31) ? __popc(ub[x >> 5] & ((1u << (x & 31)) - 1u)) : 0);
    };
    if (pool_mode == 0) {
        hm_e = rank(nm);
        hb_e = rank(A.n_ids) - rank(A.n_ids - nb);
    }
    // pools whose ids are all usable: the fallback's k-th healthy invoker is arithmetic (no rank/select reads)
    bool full_m = pool_mode == 0 && hm_e == nm, full_b = pool_mode == 0 && hb_e == nb;

    int g = 0;    // global chunk index
    int par = 0;  // pass parity (double-buffered LDS scalars)
    for (int b = 0; b < A.n_batches; ++b) {
        const int64_t a_beg = A.acq_off[b], a_end = A.acq_off[b + 1];
        if (A.hwords && pool_mode == 0) {
            // ============================================================ health of batch b (updateInvokers,
            // SCPB:512-551: the status vector only; slots and pools unchanged): the usable bitmap, the usable flag folded
            // into each changed invoker's permits, the bitmap's prefix counts and each pool's healthy count.  (The walk
            // cursors are per batch, the bound U is recomputed below from the new bitmap.)
            const uint32_t* hw = A.hwords + (int64_t)b * A.hstride;
            lds_sync();  // (the previous batch's readers of the bitmap are done)
            for (int w = tid; w < words; w += OWGS_NT) {
                const uint32_t nw = hw[w], ow = ub[w];
                for (uint32_t ch = nw ^ ow; ch; ch &= ch - 1u) {
                    const int bit = __builtin_ctz(ch), i = (w << 5) + bit;
                    if (i < A.n_ids && i < n_slots) P[i] += ((nw >> bit) & 1u) ? -OWGS_PENC : OWGS_PENC;
                }
                ub[w] = nw;
            }
            lds_sync();
            if (wave == 0) {  // prefix counts of the usable bitmap
                int carry = 0;
                for (int w0 = 0; w0 <= words; w0 += 64) {
                    const int w = w0 + lane;
                    const int c = w < words ? __popc(ub[w]) : 0;
                    const int inc = wave_incl_scan(c);
                    if (w <= words) pc[w] = (uint32_t)(carry + inc - c);
                    carry += __builtin_amdgcn_readlane(inc, 63);
                }
            }
            lds_sync();
            hm_e = rank(nm);
            hb_e = rank(A.n_ids) - rank(A.n_ids - nb);
            full_m = hm_e == nm;
            full_b = hb_e == nb;
        }

        // ============================================================ releases of batch b (SCPB:327-331)
#ifdef OWGS_PROFILE
        const u64 tb0 = memtime_pinned();
#endif
        if (A.rel_off) {
            // the engine's own stores (decisions, aggregated releases, release records) of earlier batches land;
            // the release counters share LDS with the publish-phase scratch: clear them
            if (!io) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            for (int ix = tid; ix < OWGS_CTC; ix += OWGS_NT) rc[ix] = 0u;
            lds_sync();
            const bool rel_ovf = kConc && OWGS_OVF && sc[SC_OVF] > 0;  // overflow table in use (uniform)
            if (!io) {
                // the release records of batch b (rel_rec[rel_off[b] .. rel_off[b+1]), written when the released
                // activations were decided): maxConcurrent == 1 -> ForcibleSemaphore.release (FS:117-120), summed
                // per invoker with LDS atomics (the sum of releases is order-free); concurrent ->
                // RS.release(1, true) per release (NS:98-113): the count per entry decides the final state, each
                // release's memory return depends only on its rank (c0 + q + 1) % R == 0
                // (this CU may hold lines of these records in its L1 from an earlier batch's read of the
                // neighbouring records: invalidate it once, then the records stream through it)
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                const int64_t cb = A.rel_off[b], ce = A.rel_off[b + 1];
                const int64_t cm = cb + A.relcnt[2 * b];  // [cb, cm): maxConcurrent == 1, [cm, ce): concurrent
                // maxConcurrent == 1: 16-byte reads (two records), OWGS_REL_RQ1 of them in flight per thread (the
                // sweep is latency-bound), a permit add per record
                {
                    constexpr int RQ = OWGS_REL_RQ1;
                    const int64_t pb = cb >> 1, pe = (cm + 1) >> 1;
                    for (int64_t p0 = pb + tid; p0 < pe; p0 += RQ * OWGS_ENT) {
                        uint4 rp[RQ];
#pragma unroll
                        for (int k = 0; k < RQ; ++k) {
                            const int64_t pp = p0 + (int64_t)k * OWGS_ENT;
                            rp[k] = pp < pe ? ((const uint4*)A.rel_rec)[pp] : make_uint4(~0u, ~0u, ~0u, ~0u);
                        }
#pragma unroll
                        for (int k = 0; k < 2 * RQ; ++k) {
                            const int64_t r = 2 * (p0 + (int64_t)(k >> 1) * OWGS_ENT) + (k & 1);
                            const uint32_t lo = (k & 1) ? rp[k >> 1].z : rp[k >> 1].x;
                            const uint32_t hi = (k & 1) ? rp[k >> 1].w : rp[k >> 1].y;
                            const int inv = (int)(lo & 0x7FFFu);
                            if (r < cb || r >= cm || inv == (int)OWGS_RR_NOINV || inv >= n_slots) continue;
                            if (((hi >> 17) & OWGS_AM_MAXC_MASK) > 1u) err |= OWGS_ERR_BAD_STREAM;  // (not its class)
                            else atomicAdd(&P[inv], (int)(lo >> 15));  // FS:117-120 (range check: per-batch bounds)
                        }
                    }
                }
                // concurrent: RS.release(1, true) per release through the concurrency map
                constexpr int RQ = OWGS_REL_RQ;
                const int64_t pb = cm >> 1, pe = (ce + 1) >> 1;
                if (!kConc && cm < ce) err |= OWGS_ERR_BAD_STREAM;  // (a specialisation without the map)
                for (int64_t p0 = pb + tid; kConc && p0 < pe; p0 += RQ * OWGS_ENT) {
                    uint4 rp[RQ];
#pragma unroll
                    for (int k = 0; k < RQ; ++k) {
                        const int64_t pp = p0 + (int64_t)k * OWGS_ENT;
                        rp[k] = pp < pe ? ((const uint4*)A.rel_rec)[pp] : make_uint4(0u, 0u, 0u, 0u);
                    }
                    u64 rr[2 * RQ];
#pragma unroll
                    for (int k = 0; k < RQ; ++k) {
                        const int64_t r = 2 * (p0 + (int64_t)k * OWGS_ENT);
                        rr[2 * k] = (r >= cm && r < ce) ? ((u64)rp[k].y << 32 | rp[k].x) : ~0ull;
                        rr[2 * k + 1] = (r + 1 >= cm && r + 1 < ce) ? ((u64)rp[k].w << 32 | rp[k].z) : ~0ull;
                    }
#pragma unroll
                    for (int k = 0; k < 2 * RQ; ++k) {  // (out-of-range halves read as ~0: no entry)
                        const uint32_t lo = (uint32_t)rr[k], hi = (uint32_t)(rr[k] >> 32);
                        const int inv = (int)(lo & 0x7FFFu);
                        if (inv == (int)OWGS_RR_NOINV || inv >= n_slots) continue;  // no entry / invokerSlots.lift
                        const int mem = (int)(lo >> 15);
                        const int slot = (int)(hi & 0x1FFFFu);
                        const int R = (int)((hi >> 17) & OWGS_AM_MAXC_MASK);
                        if (R <= 1) {  // (not its class)
                            err |= OWGS_ERR_BAD_STREAM;
                            continue;
                        }
                        uint32_t v;
                        const int ix = ct_find2(ct, A.ovf, rel_ovf, ct_key(inv, slot), &v);
                        const int c0 = (int)(v & OWGS_CT_C_MASK), ops0 = ct_ops(v);
                        if (ix < 0 || ops0 <= 0) {
                            // NoSuchElementException (NS:103): a flag for the caller's explicit releases
                            // (owgs_process_batch), a broken stream for the engine's own records
                            if (A.rel_src) A.rel_flags[A.rel_src[2 * (p0 + (int64_t)(k >> 1) * OWGS_ENT) + (k & 1)]] =
                                OWGS_REL_NOSUCH_BIT;
                            else err |= OWGS_ERR_BAD_STREAM;
                            continue;
                        }
                        uint32_t q;
                        if (ix < OWGS_CTC) {
                            q = atomicAdd(&rc[ix], 1u << 12) >> 12;
                            if (q == 0) atomicOr(&rc[ix], (uint32_t)R);
                        } else {  // overflow entry: its counter in HBM, first release lists it for the apply step
                            const int oj = ix - OWGS_CTC;
                            q = atomicAdd(&A.ovf.rc[oj], 1u << 12) >> 12;
                            if (q == 0) {
                                atomicOr(&A.ovf.rc[oj], (uint32_t)R);
                                A.ovf.touched[atomicAdd(A.ovf.n_touched, 1)] = oj;
                            }
                        }
                        if ((int)q >= ops0) {  // more releases than operations: which ones fail is fixed below
                            if (A.rel_src) sc[SC_IRR] = 1;
                            else err |= OWGS_ERR_BAD_STREAM;
                            continue;
                        }
                        if (mod_fast(c0 + (int)q + 1, R, __builtin_amdgcn_rcpf((float)R)) == 0)  // RS:50-52
                            atomicAdd(&P[inv], mem);
                    }
                }
            }
            if (rel_ovf && !io) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // HBM counters landed
            lds_sync();
            const bool irr = A.rel_src && sc[SC_IRR];  // (every wave reads it before the reset below)
            if (irr) {
                // explicit releases, some entry released more often than its operationCount: in stream order the
                // first ops0 releases find the entry, the rest throw NoSuchElementException (NS:103) after its
                // removal.  (The counts above already give the state; only the flags need the order.)  Invalid
                // input only -- every completion of a scheduled activation has its operation -- so one wave
                // walks the batch's concurrent records (stream order inside the class) and counts.
                const int64_t cb = A.rel_off[b], ce = A.rel_off[b + 1], cm = cb + A.relcnt[2 * b];
                if (wave == 0) {
                    for (int64_t p = cm; p < ce; ++p) {
                        const uint2 rr = A.rel_rec[p];
                        const int inv = (int)(rr.x & 0x7FFFu);
                        if (inv == (int)OWGS_RR_NOINV || inv >= n_slots) continue;
                        const uint32_t key = ct_key(inv, (int)(rr.y & 0x1FFFFu));
                        uint32_t v;
                        const int ix = ct_find2(ct, A.ovf, rel_ovf, key, &v);
                        const int ops0 = ct_ops(v);
                        if (ix < 0 || ops0 <= 0) continue;
                        const int cnt = (int)((ix < OWGS_CTC ? rc[ix]
                                                             : __hip_atomic_load(&A.ovf.rc[ix - OWGS_CTC], __ATOMIC_RELAXED,
                                                                                 __HIP_MEMORY_SCOPE_AGENT)) >> 12);
                        if (cnt <= ops0) continue;
                        int rank = 0;  // earlier releases of the same entry
                        for (int64_t q0 = cm; q0 < p; q0 += 64) {
                            const int64_t qq = q0 + lane;
                            bool same = false;
                            if (qq < p) {
                                const uint2 r2 = A.rel_rec[qq];
                                same = (int)(r2.x & 0x7FFFu) == inv && (r2.y & 0x1FFFFu) == (rr.y & 0x1FFFFu);
                            }
                            rank += __popcll(__ballot(same));
                        }
                        if (lane == 0) A.rel_flags[A.rel_src[p]] = rank >= ops0 ? OWGS_REL_NOSUCH_BIT : 0;
                    }
                }
                lds_sync();
                if (tid == 0) sc[SC_IRR] = 0;
            }
#ifdef OWGS_PROFILE
            pt_y[0] += memtime_pinned() - tb0;
#endif
            if (!io) {  // apply the release counts: c1 = (c0 + j) mod R, ops1 = ops0 - j, removed at 0 (NS:109-111)
                for (int ix = tid; ix < OWGS_CTC; ix += OWGS_ENT) {
                    const uint32_t v = rc[ix];
                    if (!v) continue;
                    rc[ix] = 0u;
                    const int R = (int)(v & 0xFFFu);
                    const uint32_t cv = ct[ix].y;
                    const int c0 = (int)(cv & OWGS_CT_C_MASK), ops0 = ct_ops(cv);
                    const int j = min((int)(v >> 12), ops0);
                    const int ops1 = ops0 - j;
                    if (ops1 == 0) {
                        ct[ix] = make_uint2(OWGS_CT_TOMB, 0u);
                    } else {
                        ct[ix].y = ct_val((c0 + j) % R, ops1);
                    }
                }
                if (rel_ovf) {  // the overflow entries this batch released
                    const int nt = __hip_atomic_load(A.ovf.n_touched, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    for (int i2 = tid; i2 < nt; i2 += OWGS_ENT) {
                        const int oj = __hip_atomic_load(&A.ovf.touched[i2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const uint32_t v = __hip_atomic_load(&A.ovf.rc[oj], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&A.ovf.rc[oj], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const int R = (int)(v & 0xFFFu);
                        const uint32_t cv = ovf_ld(A.ovf.t, oj).y;
                        const int c0 = (int)(cv & OWGS_CT_C_MASK), ops0 = ct_ops(cv);
                        const int j = min((int)(v >> 12), ops0);
                        const int ops1 = ops0 - j;
                        if (ops1 == 0) ovf_st(A.ovf.t, oj, OWGS_CT_TOMB, 0u);
                        else ovf_st_val(A.ovf.t, oj, ct_val((c0 + j) % R, ops1));
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                }
            }
            if (rel_ovf) {
                lds_sync();
                if (tid == 0) {
                    __hip_atomic_store(A.ovf.n_touched, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                }
            }
        }

        // ============================================================ concurrency-table cleanup
        // Deleted entries keep probe chains long; once live + deleted exceed half the primary (or half the overflow),
        // the live entries of both tables are parked in HBM scratch and re-inserted: the primary takes up to 3/4 of its
        // capacity, the rest goes to the overflow (batch boundary: the engine waves' stores have drained, see above).
        lds_sync();
#ifdef OWGS_PROFILE
        const u64 tb1 = memtime_pinned();
#endif
        // (a rebuild costs an HBM round trip of every live entry: at least CTC/8 new entries since the last one, so a
        // shard whose live entries stay above half the primary does not rebuild in every batch)
        if (kConc && ((sc[SC_USED] > OWGS_CTC / 2 && sc[SC_USED] >= sc[SC_CLAST] + OWGS_CTC / 8) ||
                      (A.ovf.cap > 0 && sc[SC_OVF] > A.ovf.cap / 2))) {
            const bool had_ovf = sc[SC_OVF] > 0;
            if (!io) {
                for (int ix = tid; ix < OWGS_CTC; ix += OWGS_ENT) {
                    const uint32_t k = ct[ix].x;
                    if (k != 0u && k != OWGS_CT_TOMB) {
                        const int j = atomicAdd(&sc[SC_NLIVE], 1);
                        A.ct_tmp[2 * j] = k;
                        A.ct_tmp[2 * j + 1] = ct[ix].y;
                    }
                }
                if (had_ovf)
                    for (int ix = tid; ix < A.ovf.cap; ix += OWGS_ENT) {
                        const uint2 e = ovf_ld(A.ovf.t, ix);
                        if (e.x != 0u) ovf_st(A.ovf.t, ix, 0u, 0u);
                        if (e.x != 0u && e.x != OWGS_CT_TOMB) {
                            const int j = atomicAdd(&sc[SC_NLIVE], 1);
                            A.ct_tmp[2 * j] = e.x;
                            A.ct_tmp[2 * j + 1] = e.y;
                        }
                    }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            lds_sync();
            const int nlive = sc[SC_NLIVE];
            for (int ix = tid; ix < OWGS_CTC; ix += OWGS_NT) {
                ct[ix] = make_uint2(0u, 0u);
            }
            lds_sync();
            const int nprim = min(nlive, 3 * OWGS_CTC / 4);  // the rest (a map beyond the primary) to the overflow
            if (!io) {
                for (int j = tid; j < nlive; j += OWGS_ENT) {
                    const uint32_t k = __hip_atomic_load(&A.ct_tmp[2 * j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint32_t v = __hip_atomic_load(&A.ct_tmp[2 * j + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (j < nprim) {
                        int fresh = 0;
                        const int ix = ct_insertv(ct, k, &fresh);
                        ct[ix].y = v;
                    } else if (ovf_insert(A.ovf, k, v) < 0) {
                        err |= OWGS_ERR_CTAB_FULL;
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            }
            lds_sync();
            if (tid == 0) {
                sc[SC_USED] = nprim;
                sc[SC_CLAST] = nprim;
                sc[SC_OVF] = nlive - nprim;
                sc[SC_NLIVE] = 0;
            }
            lds_sync();
        }
#ifdef OWGS_PROFILE
        pt_y[1] += memtime_pinned() - tb1;
#endif
        PT(0);
        // ============================================================ per-batch bounds
        if (!io) {
            // permits after the releases stay inside the LDS encoding's range (beyond it: error; the reference's
            // own limit, FS:48-50, is 2^31)
            for (int i = tid; i < n_slots; i += OWGS_ENT) {
                const int v = P[i];
                const bool unusable = pool_mode == 0 && i < A.n_ids && !((ub[i >> 5] >> (i & 31)) & 1u);
                if ((unusable ? v - OWGS_PENC : v) >= OWGS_PLIM) err |= OWGS_ERR_PERMITS;
            }
            int m0 = (int)0x80000000, m1 = (int)0x80000000;
            if (pool_mode == 0) {
                for (int i = tid; i < nm; i += OWGS_ENT)
                    if ((ub[i >> 5] >> (i & 31)) & 1u) m0 = max(m0, P[i]);
                for (int p = tid; p < nb; p += OWGS_ENT) {
                    const int i = A.n_ids - nb + p;
                    if ((ub[i >> 5] >> (i & 31)) & 1u) m1 = max(m1, P[i]);
                }
            } else {
                for (int i = tid; i < nm; i += OWGS_ENT)
                    if (pw[i] >= 0) m0 = max(m0, P[pw[i]]);
                for (int i = tid; i < nb; i += OWGS_ENT)
                    if (pw[nm + i] >= 0) m1 = max(m1, P[pw[nm + i]]);
            }
            m0 = wave_max(m0);
            m1 = wave_max(m1);
            if (lane == 0) {
                atomicMax(&sc[SC_U0], m0);
                atomicMax(&sc[SC_U1], m1);
            }
        }
        lds_sync();

        PT(0);
        // ============================================================ publishes (SCPB:398-436, NS:32-91)
        const uint32_t btag = (uint32_t)(A.cur_tag0 + b + 1) & 0x1FFFFu;  // HBM cursors written in this batch
        for (int64_t c0 = a_beg; c0 < a_end; c0 += A.cw, ++g) {
            const int len = (int)min((int64_t)A.cw, a_end - c0);
            ++st_chunk;
            TRACE_MARK(6);
            // ---- lane record: the pre-pass dealt the chunk's records by class (maxConcurrent == 1 first), so a wave
            // mostly runs one speculation path; li = the lane's index in the stream order of the chunk
            const bool own = !io && lane < OWGS_LPW;  // this thread may hold an activation of the chunk
            const bool held = !io && lane < wave_cap(len, wave);
            const int sl = held ? wave_off(len, wave) + lane : 0;  // record position
            const int sbuf = g % OWGS_NSTG;
            const int lx = held ? (int)stgL[sbuf * OWGS_WL + sl] : 0;
            const int li = held ? (lx & 0xFFFF) : OWGS_WL;
            const int lead = lx >> 16;  // first lane of the chunk with this lane's action (its walk-cursor word)
            uint4 rc4 = make_uint4(0, 0, 0, 0);
            int relx = -1;
            uint32_t gcw = 0;
            if (held) {
                rc4 = stgA[sbuf * OWGS_WL + sl];
                relx = A.relpos ? stgX[sbuf * OWGS_WL + li] : -1;
                gcw = stgC[(g & 1) * OWGS_WL + sl];
            }
            const bool valid = own && (rc4.y & OWGS_AM_VALID) && li < len;
            const int home = (int)(rc4.x & OWGS_AM_POS_MASK);
            const int step = (int)((rc4.x >> 15) & OWGS_AM_POS_MASK);
            const int pool = (rc4.x & OWGS_AM_POOL) ? 1 : 0;
            const bool cok = (rc4.x & OWGS_AM_COK) != 0;
            const int mem = (int)(rc4.y & OWGS_AM_MEM_MASK);
            const int maxc = conc_of(rc4.y);
            if (!kConc && held && (rc4.y & OWGS_AM_VALID) && ((rc4.y >> OWGS_AM_MAXC_SHIFT) & OWGS_AM_MAXC_MASK) != 1u)
                err |= OWGS_ERR_BAD_STREAM;  // a concurrent action in a launch of the specialisation without the map
            const bool sthrow = (rc4.y & OWGS_AM_THROW) != 0;
            const bool sempty = (rc4.y & OWGS_AM_EMPTY) != 0;
            const int a = (int)(rc4.z & OWGS_REC_NOACT);
            const int occ = (int)((rc4.z >> 17) & OWGS_RMASK);
            const int slot = (int)(rc4.w & 0x1FFFFu);
            const int nxt = (int)((rc4.w >> 17) & OWGS_REC_NONEXT);
            const int ext = (int)((rc4.z >> 27) | ((rc4.w >> 27) << 5));  // pk1 (maxConc > 1) or hot slot
            const int pk1 = (maxc > 1 && ext < HOT_CONC) ? ext : 0;
            const int n = pool ? nb : nm;
            const float rm = __builtin_amdgcn_rcpf((float)(mem > 0 ? mem : 1));
            const int64_t i = c0 + li;
            bool pending = valid;
            TRACE_MARK(7);
            // walk cursor after a forced acquire of a concurrent action at invoker x: the walk had failed everywhere,
            // and the new container at x (maxConcurrent - 1 free slots) is the only step that became feasible, so the
            // next lanes start at x's step j = (pos(x) - home) * step^-1 mod n (identity pools; else from 0)
            auto fallback_cursor = [&](int x) -> uint32_t {
                if (pool_mode != 0 || n <= 1) return 0u;
                const int xp = x - (pool ? A.n_ids - nb : 0);
                if (xp < 0 || xp >= n) return 0u;
                int t0 = 0, t1 = 1, r0 = n, r1 = step % n;  // extended Euclid: step^-1 mod n (gcd(step, n) = 1)
                while (r1 != 0) {
                    const int q = r0 / r1;
                    const int tt = t0 - q * t1;
                    t0 = t1;
                    t1 = tt;
                    const int rr = r0 - q * r1;
                    r0 = r1;
                    r1 = rr;
                }
                if (r0 != 1) return 0u;
                const int inv = t0 < 0 ? t0 + n : t0;
                const int d = xp - home;
                const int dd = d < 0 ? d + n : d;
                return (uint32_t)(int)(((long long)dd * inv) % n);
            };
            // chunk cursor word of each action, at its first lane: walk step (15 bits) | lanes committed (10 bits);
            // the step starts from the action's HBM cursor when it was written in this batch (a lower bound: steps
            // before it were full and permits only fall inside a batch)
            if (held && occ == 0) {
                // the I/O wave gathered this chunk's cursors while the previous chunk ran: a concurrent forced
                // acquire there moved its action's cursor BACK (fallback_cursor), so the gathered word may be past
                // the new container; concurrent lanes then walk from step 0 (always a valid lower bound)
                const bool stale = maxc > 1 && sc[SC_CBWD] == g;
                const uint32_t st0 =
                    (a != (int)OWGS_REC_NOACT && cok && !stale && (gcw >> 15) == btag) ? (gcw & 0x7FFFu) : 0u;
                ccw[li] = st0;
            }

            // ---- hot actions (slots assigned by the pre-pass): the first lane publishes the walk, the last lane
            // the largest occurrence index
            const int hsx = maxc > 1 ? ext - HOT_CONC : ext;  // hot slot or out of [0, NHOT)
            const int hs = (valid && hsx >= 0 && hsx < NHOT && !(A.opts & 1)) ? hsx : -1;
            if (hs >= 0) {
                if (occ == 0) {
                    hdir[hs] = make_uint4((uint32_t)li, rc4.x, rc4.y, (uint32_t)slot);  // .x = cursor word
                    hflag[hs] = 0;  // walked in the first pass (f = 0)
                    atomicMax(&sc[SC_NHOT], hs + 1);
                }
                if (nxt == (int)OWGS_REC_NONEXT) hocc[hs] = occ;
            }
            LDS_SYNC_T(1);
            const int nhot = sc[SC_NHOT];
            // ---- I/O wave: cursors of chunk g+1, records of chunk g+2
            if (io) {
                io_gather((g + 1) % OWGS_NSTG, (g + 1) & 1);
                if (io_locate(io_b, io_c0)) {
                    io_dma(io_c0, (g + 2) % OWGS_NSTG, g + 2);
                    io_c0 += A.cw;
                }
            }

            int f = 0;
            PT(1);
            // per-lane speculation, kept across the passes of the chunk: a maxConcurrent==1 lane that was known to
            // fit stays exact (its earlier walk steps only lose capacity; the next validation re-checks its target
            // against every lane before it), so only the lanes that were not known to fit speculate again
            int kind = K_NONE, t = -1, ks = 0, cons = 0, s_t = 0, r = 0;
            uint32_t cw = 0, cval = 0;
            int cidx = -1;
            bool keep = false;
            while (f < len) {
                ++st_pass;
                const bool ovf_on = kConc && OWGS_OVF && sc[SC_OVF] > 0;  // overflow keys exist: lookups fall through (uniform)
#ifdef OWGS_PROFILE
                const u64 tpass0 = memtime_pinned();
#ifdef OWGS_PROF_LATER
                pt_on = f > 0;  // phase cycles of the later passes only
#endif
#endif
                const bool act = pending && li >= f;
                // a kept concurrent lane's unit index at its target (and so its memory take) assumed every earlier
                // lane of its action lands as speculated: it speculates again when one of them did
                if (keep && maxc > 1 && cdirty[par * OWGS_WL + lead]) keep = false;
                const bool spec = act && !keep;
                // a maxConcurrent == 1 lane that speculated rank 0 at walk step s_t saw zero capacity at every step
                // before s_t; permits only fall inside a batch, so its next walk resumes there (rank 0 stays 0)
                const int resume = (spec && kind == K_TARGET && maxc == 1 && r == 0 && cok) ? s_t : 0;
                // ------------------------------------------------ speculate (packing) against the state at f
                if (spec) {
                    kind = K_NONE;
                    t = -1;
                    ks = 0;
                    cons = 0;
                    s_t = 0;
                    r = 0;
                    cw = 0;
                    cval = 0;
                    cidx = -1;
                }
                int ws = 0, wpos = 0, wcum = 0;  // long-walk resume state
#ifdef OWGS_PROFILE
                const u64 ts_beg = memtime_pinned();
                int pf_fast = 0, pf_gen = 0, pf_pre = 0;
#endif
                // ------------------------------------------------ hot actions: one wave-cooperative walk per slot
                // 64 walk steps per round: capacities, inclusive scan, then every rank q finds the step whose
                // capacity range holds it (first rank of each step marked in LDS, prefix max over ranks)
                // slot h goes to the I/O wave when h % (OWGS_EW + 1) == 0 (it holds no lanes: its speculation is
                // otherwise idle), else to engine wave h % (OWGS_EW + 1) - 1
                {
                    const int wr = (wave + OWGS_EW - OWGS_HOT_ROT % OWGS_EW) % OWGS_EW;  // (io: unused)
                    const int hw = OWGS_HOT_IO ? (io ? 0 : wr + 1) : (io ? NHOT : wr);
                    for (int h = hw; h < nhot; h += OWGS_HOT_IO ? OWGS_EW + 1 : OWGS_EW) {
                        const uint4 d = hdir[h];
                        if (d.z & (OWGS_AM_THROW | OWGS_AM_EMPTY)) continue;
                        if (hflag[h] != f) continue;  // no lane of this action speculates in this pass
                        const int hhome = (int)(d.y & OWGS_AM_POS_MASK), hstep = (int)((d.y >> 15) & OWGS_AM_POS_MASK);
                        const int hpool = (d.y & OWGS_AM_POOL) ? 1 : 0;
                        const bool hcok = (d.y & OWGS_AM_COK) != 0;
                        const int hmem = (int)(d.z & OWGS_AM_MEM_MASK);
                        const int hmc = conc_of(d.z);
                        const int hslot = (int)d.w;
                        const uint32_t hcw = ccw[d.x];
                        const int hcc = (int)((hcw >> 15) & OWGS_RMASK);
                        const int need = min(hocc[h] - hcc + 1, HOT_RANKS);
                        if (need <= 0) continue;
                        uint2* tab = htab + h * HOT_RANKS;
                        const int hn = hpool ? nb : nm;
                        if (hmc == 1 && hmem > sc[hpool ? SC_U1 : SC_U0] && ((A.shortcut_ok >> hpool) & 1)) {
                            for (int q = lane; q < need; q += 64) tab[q] = make_uint2((uint32_t)K_FALLBACK << 15, 0u);
                            continue;
                        }
                        int s0 = hcok ? (int)(hcw & 0x7FFFu) : 0;
                        const float rnn = __builtin_amdgcn_rcpf((float)hn);
                        int p0 = mod_fast(hhome + s0 * hstep, hn, rnn);
                        const int loff = mod_fast(lane * hstep, hn, rnn), boff = mod_fast(64 * hstep, hn, rnn);
                        const float rmh = __builtin_amdgcn_rcpf((float)hmem);
                        int* scr = hscr + wave * 64;
                        int cum = 0;
                        ++st_long;
                        for (;;) {
#ifdef OWGS_PROFILE
                            ++pw_c[7];
#endif
                            if (s0 >= hn) {  // every position probed: the remaining ranks fall back (SCPB:417)
                                for (int q = cum + lane; q < need; q += 64)
                                    tab[q] = make_uint2((uint32_t)K_FALLBACK << 15, 0u);
                                break;
                            }
                            const int sk = s0 + lane;
                            int pp = p0 + loff;
                            pp -= pp >= hn ? hn : 0;
                            int id = OWGS_PW_UNUSABLE, cap = 0;
                            bool bad = false;
                            if (sk < hn) {
                                int pv;
                                id = pool_probe(E, hpool, pp, &pv);
                                if (id == OWGS_PW_BADID) {
                                    bad = true;
                                } else if (id >= 0) {
                                    if (hmc == 1) {
                                        cap = cap_bf(pv, hmem, rmh);
                                    } else {
                                        uint32_t v;
                                        ct_find2(ct, A.ovf, ovf_on, ct_key(id, hslot), &v);
                                        cap = (int)(v & OWGS_CT_C_MASK) + min(cap_bf(pv, hmem, rmh) * hmc, CAPMAX);
                                    }
                                }
                            }
                            st_probe += 1;
                            const u64 bm = __ballot(bad);
                            const int qb = bm ? ffs64(bm) : 64;
                            if (lane >= qb) cap = 0;
                            const int inc = wave_incl_scan(cap), exc = inc - cap;
                            const int total = __builtin_amdgcn_readlane(inc, 63);
                            // lanes exchange marks through LDS: the fences keep the compiler from forwarding this
                            // lane's own store (the exchange is cross-lane; the wave's LDS ops execute in order)
                            scr[lane] = -1;
                            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                            if (cap > 0 && exc < 64) scr[exc] = lane;
                            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                            const int mv = scr[lane];
                            const int sj = max(wave_incl_max(mv), 0);
                            const int tid_ = __shfl(id, sj, 64);
                            const int ex_ = __shfl(exc, sj, 64);
                            const int q = cum + lane;
                            if (q < need && lane < total)
                                tab[q] = make_uint2((uint32_t)tid_ | ((uint32_t)K_TARGET << 15) |
                                                        ((uint32_t)(lane - ex_) << 18),
                                                    (uint32_t)(s0 + sj));
                            if (qb < 64) {  // the walk of every later rank reaches a throwing probe first
                                for (int q2 = cum + total + lane; q2 < need; q2 += 64)
                                    tab[q2] = make_uint2((uint32_t)K_THROW << 15, 0u);
                                break;
                            }
                            cum += total;
                            if (cum >= need) break;
                            s0 += 64;
                            p0 += boff;
                            p0 -= p0 >= hn ? hn : 0;
                        }
                    }
                }
#ifdef OWGS_PROFILE
                const u64 ts_hot = memtime_pinned();
#endif
                if (spec) {
                    if (sempty) {
                        kind = K_NONE;
                    } else if (sthrow) {
                        kind = K_THROW;
                    } else {
                        int s = 0;
                        r = occ;
                        cw = ccw[lead];  // walk step (15 bits) | committed lanes of the action in this chunk (10)
                        r = occ - (int)((cw >> 15) & OWGS_RMASK);
                        if (cok) s = (int)(cw & 0x7FFFu);
                        if (r == 0 && resume > s) s = resume;
                        const int U = sc[pool ? SC_U1 : SC_U0];
                        if (hs >= 0 && r < HOT_RANKS) {
                            kind = K_HOT;
                        } else if (maxc == 1 && mem > U && ((A.shortcut_ok >> pool) & 1)) {
                            kind = K_FALLBACK;  // every usable permit < mem: the walk fails everywhere
                        } else if (OWGS_CSCAN_ON && maxc > 1 && mem > U && pool_mode == 0 && n > OWGS_CSCAN_MIN_N && !ovf_on) {
                            kind = K_CSCAN;  // no invoker can open a container: capacity = the key's open ones
                            ws = s;          // (the ordinary walk's start, should the key have > 64 of them)
                            wpos = mod_fast(home + s * step, n, __builtin_amdgcn_rcpf((float)n));
                            wcum = 0;
                        } else {
                            int pos = mod_fast(home + s * step, n, __builtin_amdgcn_rcpf((float)n));
                            int cum = 0;
                            kind = K_LONG;
#ifdef OWGS_PROFILE
                            pf_pre = (int)(memtime_pinned() - ts_hot);
#endif
                            
                            if (maxc == 1 && pool_mode == 0) {
#ifdef OWGS_PROFILE
                                const u64 tf0 = memtime_pinned();
#endif
                                // identity pools: pool position -> id is arithmetic, so the permit and usable-bit
                                // reads of 4 walk steps are independent and issue together
                                const int base = pool ? A.n_ids - nb : 0;
                                bool done = false;
#pragma unroll 1
                                for (int g4 = 0; g4 < KPROBE / FGRP; ++g4) {
                                    if (done) break;
                                    int ps[FGRP], pv[FGRP];
                                    int pp = pos;
#pragma unroll
                                    for (int k = 0; k < FGRP; ++k) {
                                        ps[k] = pp;
                                        pv[k] = P[base + pp];  // usable flag folded in (OWGS_PENC)
                                        pp += step;
                                        pp -= pp >= n ? n : 0;
                                    }
#pragma unroll
                                    for (int k = 0; k < FGRP; ++k) asm volatile("" : "+v"(pv[k]));  // reads in flight
                                    // branch-free scan of the group's steps: first step whose cumulative capacity
                                    // exceeds the rank (hit), or the end of the walk (s + k == n: every position probed)
                                    int hit = FGRP, kc = cum, hc = cum, tsel = ps[0];
                                    bool ended = false;
#pragma unroll
                                    for (int k = 0; k < FGRP; ++k) {
                                        const int cap = pv[k] < OWGS_PLIM ? cap_bf(pv[k], mem, rm) : 0;
                                        const bool open = hit == FGRP && !ended;
                                        const bool fin = open && s + k >= n;
                                        const bool h = open && !fin && kc + cap > r;
                                        ended = ended || fin;
                                        hit = h ? k : hit;
                                        hc = h ? kc : hc;
                                        tsel = h ? ps[k] : tsel;
                                        kc += (open && !fin && !h) ? cap : 0;
                                    }
                                    st_probe += FGRP;
                                    if (hit < FGRP) {
                                        kind = K_TARGET;
                                        t = base + tsel;
                                        ks = r - hc;
                                        s_t = s + hit;
                                        done = true;
                                    } else if (ended) {
                                        kind = K_FALLBACK;  // every pool position probed: the walk fails (SCPB:417)
                                        done = true;
                                    } else {
                                        cum = kc;
                                        s += FGRP;
                                        pos = pp;
                                    }
                                }
#ifdef OWGS_PROFILE
                                pf_fast = (int)(memtime_pinned() - tf0);
#endif
                            } else {
#ifdef OWGS_PROFILE
                            const u64 tg0 = memtime_pinned();
#endif
                            ++st_glane;
                            if (maxc > 1 && pool_mode == 0) {
                                // identity pools, concurrent action: the permits and the first concurrency-table entry
                                // of 4 walk steps issue together; a key whose first entry holds another key follows
                                // its chain afterwards
                                const int base = pool ? A.n_ids - nb : 0;
                                bool done = false;
#pragma unroll 1
                                for (int g4 = 0; g4 < KPROBE_G / 4; ++g4) {
                                    if (done) break;
                                    int ps[4], pv[4];
                                    uint32_t hx[4];
                                    uint4 ea[4], eb[4];
                                    int pp = pos;
#pragma unroll
                                    for (int k = 0; k < 4; ++k) {
                                        ps[k] = pp;
                                        pv[k] = P[base + pp];
                                        hx[k] = ct_home(ct_key(base + pp, slot));
                                        ea[k] = *(const uint4*)&ct[hx[k]];
                                        eb[k] = *(const uint4*)&ct[hx[k] + 2];
                                        pp += step;
                                        pp -= pp >= n ? n : 0;
                                    }
#pragma unroll
                                    for (int k = 0; k < 4; ++k) asm volatile("" : "+v"(pv[k]), "+v"(ea[k].x), "+v"(eb[k].x));
                                    int hit = 4, kc = cum, hc = cum, hi = -1;
                                    uint32_t hv = 0;
                                    bool ended = false;
#pragma unroll
                                    for (int k = 0; k < 4; ++k) {
                                        const bool open = hit == 4 && !ended;
                                        const bool fin = open && s + k >= n;
                                        const uint32_t key = ct_key(base + ps[k], slot);
                                        uint32_t v = 0;
                                        int ci = -1;
                                        const int bst = ct_block(ea[k], eb[k], key, hx[k], &v, &ci);
                                        if ((bst == 2 || (bst == 0 && ovf_on)) && open && !fin) {
                                            ci = ct_resolve2(ct, A.ovf, ovf_on, bst, key, hx[k], &v, ci);
#ifdef OWGS_COUNT_CHAINS
                                            st_glane += 1u << 16;
#endif
                                        }
                                        const int cap = pv[k] < OWGS_PLIM
                                                            ? (int)(v & OWGS_CT_C_MASK) + min(cap_bf(pv[k], mem, rm) * maxc, CAPMAX)
                                                            : 0;
                                        const bool h = open && !fin && kc + cap > r;
                                        ended = ended || fin;
                                        if (h) {
                                            hit = k;
                                            hc = kc;
                                            hv = v;
                                            hi = ci;
                                        }
                                        kc += (open && !fin && !h) ? cap : 0;
                                    }
                                    st_probe += 4;
                                    st_gprobe += 4;
                                    if (hit < 4) {
                                        kind = K_TARGET;
                                        t = base + (hit == 0 ? ps[0] : hit == 1 ? ps[1] : hit == 2 ? ps[2] : ps[3]);
                                        ks = r - hc;
                                        s_t = s + hit;
                                        cval = hv;
                                        cidx = hi;
                                        done = true;
                                    } else if (ended) {
                                        kind = K_FALLBACK;  // every pool position probed (SCPB:417)
                                        done = true;
                                    } else {
                                        cum = kc;
                                        s += 4;
                                        pos = pp;
                                    }
                                }
                            } else {
#pragma unroll 1
                            for (int k = 0; k < KPROBE_G; ++k) {
                                if (s >= n) {  // every pool position probed: the n+2-probe walk fails (SCPB:417)
                                    kind = K_FALLBACK;
                                    break;
                                }
                                int pv;
                                const int id = pool_probe(E, pool, pos, &pv);
                                ++st_probe;
                                ++st_gprobe;
                                if (id == OWGS_PW_BADID) {
                                    kind = K_THROW;
                                    break;
                                }
                                if (id >= 0) {
                                    int cap;
                                    if (maxc == 1) {
                                        cap = cap_of(pv, mem, rm);
                                    } else {
                                        uint32_t v;
                                        const int ci = ct_find2(ct, A.ovf, ovf_on, ct_key(id, slot), &v);
                                        cap = (int)(v & OWGS_CT_C_MASK) + min(cap_of(pv, mem, rm) * maxc, CAPMAX);
                                        if (cum + cap > r) {
                                            cval = v;
                                            cidx = ci;
                                        }
                                    }
                                    if (cum + cap > r) {
                                        kind = K_TARGET;
                                        t = id;
                                        ks = r - cum;
                                        s_t = s;
                                        break;
                                    }
                                    cum += cap;
                                }
                                ++s;
                                pos += step;
                                if (pos >= n) pos -= n;
                            }
                            }
#ifdef OWGS_PROFILE
                            pf_gen = (int)(memtime_pinned() - tg0);
#endif
                            }
                            ws = s;
                            wpos = pos;
                            wcum = cum;
                        }
                    }
                }
                
#ifdef OWGS_PROFILE
                const u64 ts_lane = memtime_pinned();
#endif
                // ------------------------------------------------ concurrent lanes with mem > U (K_CSCAN)
                // Every usable permit count is below mem, so along the walk only the key's existing containers have
                // capacity (their free slots c >= 1, NS:57-82 without a new container).  The wave collects the key's
                // open entries from the concurrency table (64 per read), orders them by walk step
                // k(x) = (pos(x) - home) * step^-1 mod n, and finds the container holding rank r (cumulative free
                // slots in walk order); none -> the walk fails everywhere (SCPB:417).  More than 64 open containers:
                // the ordinary walk.  Only for pools larger than half the table: a smaller pool is walked faster.
                if (kConc && !io) {
                    u64 cm = __ballot(spec && kind == K_CSCAN);
                    int* cand = hscr + wave * 64;
                    while (cm) {
                        // one scan serves every lane of the wave with the same action (same key and walk)
                        const int j = ffs64(cm);
                        const int aj = __builtin_amdgcn_readlane(a, j);
                        const u64 same = aj == (int)OWGS_REC_NOACT ? (1ull << j)  // explicit walks: one lane each
                                                                   : (__ballot(spec && kind == K_CSCAN && a == aj) & cm);
                        cm &= ~same;
                        const int slj = __builtin_amdgcn_readlane(slot, j);
                        const int pj = __builtin_amdgcn_readlane(pool, j);
                        const int nn = __builtin_amdgcn_readlane(n, j);
                        const int hj = __builtin_amdgcn_readlane(home, j);
                        const int stp = __builtin_amdgcn_readlane(step, j);
                        const int base = pj ? A.n_ids - nb : 0;
                        int nc = 0;
                        constexpr int SCU = 8;  // table reads in flight per lane
                        for (int e0 = 0; e0 < OWGS_CTC && nc <= 64; e0 += 64 * SCU) {
                            uint2 ev[SCU];
#pragma unroll
                            for (int u = 0; u < SCU; ++u) ev[u] = ct[e0 + 64 * u + lane];
#pragma unroll
                            for (int u = 0; u < SCU; ++u) {
                                const int inv = (int)(ev[u].x & 0x7FFFu) - 1;
                                const int ps = inv - base;
                                const bool m = (int)(ev[u].x >> OWGS_CT_SLOT_SHIFT) == slj && inv >= 0 && ps >= 0 &&
                                               ps < nn && (ev[u].y & OWGS_CT_C_MASK) != 0u;
                                const u64 bm0 = __ballot(m);
                                if (bm0) {  // (rare) usable check only for the key's entries
                                    const bool mu = m && P[inv] < OWGS_PLIM;
                                    const u64 bm = __ballot(mu);
                                    const int at = nc + (int)__builtin_amdgcn_mbcnt_hi(
                                                            (uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
                                    if (mu && at < 64) cand[at] = e0 + 64 * u + lane;
                                    nc += __popcll(bm);
                                }
                            }
                        }
                        int rk0 = K_FALLBACK, ix = -1, kx = 0x7FFFFFFF, cx = 0, idv = 0, before = 0;
                        uint32_t vx = 0;
                        if (nc > 64) {
                            rk0 = K_LONG;  // too many containers: walk
                        } else if (nc > 0) {
                            rk0 = K_TARGET;
                            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                            // step^-1 mod n (gcd(step, n) = 1: pairwiseCoprimeNumbersUntil, SCPB:379-384)
                            int t0 = 0, t1 = 1, r0 = nn, r1 = stp % nn;
                            while (r1 != 0) {
                                const int q = r0 / r1;
                                const int tt = t0 - q * t1;
                                t0 = t1;
                                t1 = tt;
                                const int rr = r0 - q * r1;
                                r0 = r1;
                                r1 = rr;
                            }
                            const int sinv = t0 < 0 ? t0 + nn : t0;
                            const float rnn = __builtin_amdgcn_rcpf((float)nn);
                            if (lane < nc) {
                                ix = cand[lane];
                                const uint2 ev = ct[ix];
                                idv = (int)(ev.x & 0x7FFFu) - 1;
                                vx = ev.y;
                                cx = (int)(vx & OWGS_CT_C_MASK);
                                int d = idv - base - hj;
                                d += d < 0 ? nn : 0;
                                kx = mod_fast(d * sinv, nn, rnn);  // d, sinv < n < 2^15
                            }
                            // free slots of the containers before this one in walk order (distinct steps)
                            for (int m2 = 0; m2 < nc; ++m2) {
                                const int km = __builtin_amdgcn_readlane(kx, m2);
                                const int cmv = __builtin_amdgcn_readlane(cx, m2);
                                before += km < kx ? cmv : 0;
                            }
                            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                        }
                        // each lane of the action: the container holding its rank
                        for (u64 sm = same; sm;) {
                            const int jj = ffs64(sm);
                            sm &= sm - 1;
                            const int rj = __builtin_amdgcn_readlane(r, jj);
                            int rk = rk0, rt = -1, rks = 0, rst = 0, rci = -1;
                            uint32_t rcv = 0;
                            if (rk0 == K_TARGET) {
                                const u64 hm = __ballot(lane < nc && before <= rj && rj < before + cx);
                                if (hm) {
                                    const int L = ffs64(hm);
                                    rt = __builtin_amdgcn_readlane(idv, L);
                                    rks = rj - __builtin_amdgcn_readlane(before, L);
                                    rst = __builtin_amdgcn_readlane(kx, L);
                                    rci = __builtin_amdgcn_readlane(ix, L);
                                    rcv = (uint32_t)__builtin_amdgcn_readlane((int)vx, L);
                                } else {
                                    rk = K_FALLBACK;  // fewer free slots than ranks: the walk fails (SCPB:417)
                                }
                            }
                            if (lane == jj) {
                                kind = rk;
                                t = rt;
                                ks = rks;
                                s_t = rst;
                                cidx = rci;
                                cval = rcv;
                            }
                        }
                    }
                }
                // ------------------------------------------------ long walks: a work queue over the engine waves
                // Lanes whose walk outlasted their own probes queue it (record position, rank, walk state) and, after
                // a barrier, every engine wave takes queued walks one at a time until the queue is empty, so the
                // walks of one wave no longer serialise behind each other.  Each walk is wave-cooperative: LW_Q x 64
                // steps per round; the result goes back through the queue entry.
                // narrow chunks (fragmented slots: long walks are many and uneven) share the queue over the waves;
                // wide chunks walk their own queued entries, without the extra barrier
                const bool lqs = A.cw < OWGS_WL;
                int lq_i = -1, nown = 0;
                if (!io) {
                    const u64 lm = __ballot(spec && kind == K_LONG);
                    if (lm) {
                        int qb = wave * OWGS_LPW;
                        nown = __popcll(lm);
                        if (lqs) {
                            if (lane == 0) qb = atomicAdd(&sc[SC_LQN], nown);
                            qb = __builtin_amdgcn_readfirstlane(qb);
                        }
                        if (spec && kind == K_LONG) {
                            lq_i = qb + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(lm >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)lm, 0u));
                            lq[lq_i] = make_uint4((uint32_t)sl | ((uint32_t)r << 16), (uint32_t)ws, (uint32_t)wpos,
                                                  (uint32_t)wcum);
                        }
                    }
                }
#ifdef OWGS_PROFILE
                const u64 ts_b8a = memtime_pinned();
#endif
                if (lqs) {
                    LDS_SYNC_T(8);
                } else {
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // own entries: same wave
                }
#ifdef OWGS_PROFILE
                const u64 ts_b8b = memtime_pinned();
#endif
                if (!io || (OWGS_QUEUE_IO && lqs)) {  // (the I/O wave takes shared-queue walks too: it holds no lanes)
                    const int nq = lqs ? sc[SC_LQN] : wave * OWGS_LPW + nown;
                    int own = wave * OWGS_LPW;
                    for (;;) {
                        int item = own++;
                        if (lqs) {
                            if (lane == 0) item = atomicAdd(&sc[SC_LQH], 1);
                            item = __builtin_amdgcn_readfirstlane(item);
                        }
                        if (item >= nq) break;
                        ++st_long;
                        const uint4 qe = lq[item];
                        const uint4 qr = stgA[sbuf * OWGS_WL + (int)(qe.x & 0xFFFFu)];
                        int s0 = (int)qe.y;
                        int p0 = (int)qe.z;
                        int cum = (int)qe.w;
                        const int rj = (int)(qe.x >> 16);
                        const int stp = (int)((qr.x >> 15) & OWGS_AM_POS_MASK);
                        const int pj = (qr.x & OWGS_AM_POOL) ? 1 : 0;
                        const int nn = pj ? nb : nm;
                        const int mj = (int)(qr.y & OWGS_AM_MEM_MASK);
                        const int cj = conc_of(qr.y);
                        const int slj = (int)(qr.w & 0x1FFFFu);
                        const float rmj = __builtin_amdgcn_rcpf((float)mj);
                        const float rnn = __builtin_amdgcn_rcpf((float)nn);
                        // lane l probes steps l, 64 + l, .. of the round: each of its LW_Q reads is a stride-step
                        // gather over the wave (step sizes are odd: conflict-free over the LDS banks)
                        const int loff = mod_fast(lane * stp, nn, rnn);
                        const int boff = mod_fast(64 * stp, nn, rnn);
                        const int roff = mod_fast(64 * LW_Q * stp, nn, rnn);
                        int rk = K_FALLBACK, rt = -1, rks = 0, rst = 0, rci = -1;
                        uint32_t rcv = 0;
#ifdef OWGS_PROFILE
                        int nr_ = 0;
                        ++pw_c[1];
#endif
                        bool found = false;
                        while (s0 < nn && !found) {
#ifdef OWGS_PROFILE
                            ++nr_;
                            const u64 tr0_ = memtime_pinned();
#endif
                            int pv[LW_Q], id[LW_Q];
                            int p = p0 + loff;
                            if (p >= nn) p -= nn;
                            if (pool_mode == 0) {
                                // identity pools: the id is arithmetic, the usable flag folded into the permits: the
                                // LW_Q reads of the round issue back to back, no branch between them
                                const int base = pj ? A.n_ids - nb : 0;
#pragma unroll
                                for (int q = 0; q < LW_Q; ++q) {
                                    id[q] = base + p;
                                    pv[q] = P[base + p];
                                    p += boff;
                                    if (p >= nn) p -= nn;
                                }
#pragma unroll
                                for (int q = 0; q < LW_Q; ++q) {
                                    asm volatile("" : "+v"(pv[q]));
                                    id[q] = pv[q] < OWGS_PLIM ? id[q] : OWGS_PW_UNUSABLE;
                                }
                            } else {
#pragma unroll
                                for (int q = 0; q < LW_Q; ++q) {  // positions < nn: the reads are in bounds
                                    id[q] = pool_probe(E, pj, p, &pv[q]);
                                    p += boff;
                                    if (p >= nn) p -= nn;
                                }
                            }
                            // concurrent: the first 4-entry block of every probe's (invoker, fqn) key, read together
                            uint32_t hx[LW_Q];
                            uint4 ea[LW_Q], eb[LW_Q];
                            if (cj > 1) {
#pragma unroll
                                for (int q = 0; q < LW_Q; ++q) {
                                    hx[q] = ct_home(ct_key(id[q] >= 0 ? id[q] : 0, slj));
                                    ea[q] = *(const uint4*)&ct[hx[q]];
                                    eb[q] = *(const uint4*)&ct[hx[q] + 2];
                                }
#pragma unroll
                                for (int q = 0; q < LW_Q; ++q) asm volatile("" : "+v"(ea[q].x), "+v"(eb[q].x));
                            }
#ifdef OWGS_PROFILE
                            u64 tr1_ = 0;
#endif
#pragma unroll
                            for (int q = 0; q < LW_Q; ++q) {
                                const int sk = s0 + 64 * q + lane;
                                const bool in = sk < nn;
                                int cap = 0, ci = -1;
                                uint32_t v = 0;
                                const bool bad = in && id[q] == OWGS_PW_BADID;
                                if (rj == 0 && cj == 1) {  // (uniform) rank 0: the first step with room, no scan
                                    const u64 hm = __ballot(in && (bad || (id[q] >= 0 && pv[q] >= mj)));
                                    if (hm) {
                                        const int L = ffs64(hm);
                                        rst = s0 + 64 * q + L;
                                        if (__builtin_amdgcn_readlane((int)bad, L)) {
                                            rk = K_THROW;
                                        } else {
                                            rk = K_TARGET;
                                            rt = __builtin_amdgcn_readlane(id[q], L);
                                            rks = 0;
                                        }
                                        found = true;
                                        break;
                                    }
                                    continue;
                                }
                                if (cj == 1) {
                                    cap = (in && id[q] >= 0) ? cap_bf(pv[q], mj, rmj) : 0;
                                } else if (in && id[q] >= 0) {
                                    const uint32_t key = ct_key(id[q], slj);
                                    const int bst = ct_block(ea[q], eb[q], key, hx[q], &v, &ci);
                                    if (bst == 2 || (bst == 0 && ovf_on))
                                        ci = ct_resolve2(ct, A.ovf, ovf_on, bst, key, hx[q], &v, ci);
                                    cap = (int)(v & OWGS_CT_C_MASK) + min(cap_bf(pv[q], mj, rmj) * cj, CAPMAX);
                                }
                                const int inc = wave_incl_scan(cap);
                                const u64 hm = __ballot(in && (bad || cum + inc > rj));
                                if (hm) {
                                    const int L = ffs64(hm);
                                    rst = s0 + 64 * q + L;
                                    if (__builtin_amdgcn_readlane((int)bad, L)) {
                                        rk = K_THROW;
                                    } else {
                                        rk = K_TARGET;
                                        rt = __builtin_amdgcn_readlane(id[q], L);
                                        rks = rj - (cum + __builtin_amdgcn_readlane(inc - cap, L));
                                        rci = __builtin_amdgcn_readlane(ci, L);
                                        rcv = (uint32_t)__builtin_amdgcn_readlane((int)v, L);
                                    }
                                    found = true;
                                    break;
                                }
                                cum += __builtin_amdgcn_readlane(inc, 63);
                            }
#ifdef OWGS_PROFILE
                            pw_c[cj > 1 ? 9 : 8] += memtime_pinned() - tr0_;
                            (void)tr1_;
#endif
#ifdef OWGS_COUNT_ROUNDS
                            st_glane += lane == 0 ? 1u : 0u;
#endif
                            s0 += 64 * LW_Q;
                            p0 += roff;
                            if (p0 >= nn) p0 -= nn;
                        }
                        st_probe += (lane == 0) ? 64u * LW_Q : 0u;
#ifdef OWGS_PROFILE
                        pw_c[2] += nr_;
                        if (cj > 1) {
                            ++pw_c[3];
                            pw_c[4] += nr_;
                        }
                        if (rk == K_FALLBACK) {
                            ++pw_c[5];
                            pw_c[6] += nr_;
                        }
#endif
                        if (lane == 0)  // kind | (t + 1) << 3 | ks << 19, s_t, cval, cidx + 1 (overflow indices: 32 bits)
                            lq[item] = make_uint4((uint32_t)rk | ((uint32_t)(rt + 1) << 3) | ((uint32_t)rks << 19),
                                                  (uint32_t)rst, rcv, (uint32_t)(rci + 1));
                    }
                }
                
#ifdef OWGS_PROFILE
                const int pf_fw = wave_max(pf_pre), pf_gw = wave_max(pf_gen);
                if (!io && lane == 0) {
                    const u64 ts_end = memtime_pinned();
                    spw[4 * wave] = (int)(ts_hot - ts_beg);
                    spw[4 * wave + 1] = (int)(ts_lane - ts_hot);
                    spw[4 * wave + 2] = (int)(ts_end - ts_lane);
                    spw[4 * wave + 3] = (int)pw_c[1];
                    pfw[3 * OWGS_EW + 3 * wave] = (int)(ts_b8a - ts_lane);   // container scans + queue push
                    pfw[3 * OWGS_EW + 3 * wave + 1] = (int)(ts_b8b - ts_b8a);  // barrier 8
                    pfw[3 * OWGS_EW + 3 * wave + 2] = (int)(ts_end - ts_b8b);  // queued long walks
                    pfw[2 * wave] = pf_fw;
                    pfw[2 * wave + 1] = pf_gw;
                }
#endif
                LDS_SYNC_T(2);
                PT(2);  // hot tables written; every wave has finished reading P for its speculation
                if (tid < OWGS_WL) cdirty[par * OWGS_WL + tid] = 0;  // read above; this pass's commit fills the other half
#ifdef OWGS_PROFILE
                if (tid == 0) {
                    int worst = 0, wmax = -1;
                    for (int w = 0; w < OWGS_EW; ++w) {
                        const int tt = spw[4 * w] + spw[4 * w + 1] + spw[4 * w + 2];
                        if (tt > wmax) { wmax = tt; worst = w; }
                    }
                    pt_acc[6] += (u64)spw[4 * worst];       // worst wave: hot walks
                    pt_acc[7] += (u64)spw[4 * worst + 1];   // worst wave: per-lane speculation
                    pw_c[0] += (u64)spw[4 * worst + 2];     // worst wave: long walks (and imbalance)
                    int mx0 = 0, mx1 = 0, mx2 = 0;
                    for (int w = 0; w < OWGS_EW; ++w) {
                        mx0 = max(mx0, pfw[3 * OWGS_EW + 3 * w]);
                        mx1 = max(mx1, pfw[3 * OWGS_EW + 3 * w + 1]);
                        mx2 = max(mx2, pfw[3 * OWGS_EW + 3 * w + 2]);
                    }
                    pw_c[10] += (u64)mx0;
                    pw_c[11] += (u64)mx1;
                    sc_prof_q += (u64)mx2;
                    int lwmax = 0;  // long walks of the wave with the most of them in this pass (counters cumulative)
                    for (int w = 0; w < OWGS_EW; ++w) {
                        lwmax = max(lwmax, spw[4 * w + 3] - pfw[2 * OWGS_EW + w]);
                        pfw[2 * OWGS_EW + w] = spw[4 * w + 3];
                    }
                    pt_x[2] += (u64)lwmax;
#ifdef OWGS_PROF_SPLIT
                    if (f == 0)  // first passes, summed over the engine waves: hot walks | per-lane | long walks
                        for (int w = 0; w < OWGS_EW; ++w) {
                            pt_x[0] += (u64)spw[4 * w] | ((u64)spw[4 * w + 2] << 32);
                            pt_x[1] += (u64)spw[4 * w + 1];
                        }
#endif
                }
#endif
                if (lq_i >= 0) {  // a queued long walk: its result
                    const uint4 qe = lq[lq_i];
                    kind = (int)(qe.x & 7u);
                    t = (int)((qe.x >> 3) & 0xFFFFu) - 1;
                    ks = (int)(qe.x >> 19);
                    s_t = (int)qe.y;
                    cidx = (int)qe.w - 1;
                    cval = qe.z;
                }
                if (spec && kind == K_HOT) {
                    const uint2 e = htab[hs * HOT_RANKS + r];
                    kind = (int)((e.x >> 15) & 7u);
                    if (kind == K_TARGET) {
                        t = (int)(e.x & 0x7FFFu);
                        ks = (int)((e.x >> 18) & OWGS_RMASK);
                        s_t = (int)e.y;
                        if (maxc > 1) {
                            cidx = ct_find2(ct, A.ovf, ovf_on, ct_key(t, slot), &cval);
                        }
                    }
                }
                // ------------------------------------------------ forced fallback target (SCPB:417-424)
                // (the explicit-seq and explicit-pool variants load from HBM; they are kept on their own paths so
                // that their vmcnt waits never drain the decision stores of the common path)
                if (spec && kind == K_FALLBACK) {
                    const int hc = pool ? hb_e : hm_e;
#define OWGS_LAND(X)                                          \
    {                                                         \
        const int x_ = (X);                                   \
        if (x_ < 0 || x_ >= n_slots) {                        \
            kind = K_THROW;                                   \
        } else {                                              \
            t = x_;                                           \
            if (maxc > 1) {                                   \
                cidx = ct_find2(ct, A.ovf, ovf_on, ct_key(t, slot), &cval); \
            }                                                 \
        }                                                     \
    }
                    if (hc <= 0) {
                        kind = K_NONE;
                    } else if (seqp == nullptr && pool_mode == 0) {
                        const int k = (int)rng_index(A.rng_seed, A.seq_base + (u64)i, (uint32_t)hc);
                        OWGS_LAND(select_pool(E, pool ? A.n_ids - nb : 0, k, pool ? full_b : full_m));
                    } else {
                        const u64 seq = seqp ? seqp[i] : (A.seq_base + (u64)i);
                        const int k = (int)rng_index(A.rng_seed, seq, (uint32_t)hc);
                        OWGS_LAND(pool_mode == 0 ? select_usable(E, pool ? A.n_ids - nb : 0, k)
                                                   : A.hlist[(pool ? A.hm : 0) + k]);
                    }
#undef OWGS_LAND
                }
                const bool part = act && (kind == K_TARGET || kind == K_FALLBACK);
                if (spec && part) {
                    const int c0v = (int)(cval & OWGS_CT_C_MASK);
                    if (maxc == 1) cons = mem;
                    else if (kind == K_FALLBACK) cons = c0v >= 1 ? 0 : mem;
                    else cons = (ks < c0v) ? 0 : (mod_fast(ks - c0v, maxc, __builtin_amdgcn_rcpf((float)maxc)) == 0 ? mem : 0);
                }
                // ------------------------------------------------ bucket totals
                // every lane tentatively takes its memory from its target's permits: after the barrier P[t] is the
                // frontier permits minus the consumption of ALL lanes of the pass at t (the commit keeps it, the
                // lanes after l give it back).  "first" = lowest lane of the (hashed) bucket of t.
                const int bk = part ? (int)(((uint32_t)t * 2654435761u) >> (32 - OWGS_NBK_LOG2)) : 0;
                static_assert(OWGS_NBK == (1 << OWGS_NBK_LOG2) && OWGS_WL <= 512, "power-of-two buckets; lane fields 10 bits");
                if (part) {
                    if (cons) atomicSub(&P[t], cons);
                    atomicMax(&fst[bk], (uint32_t)(OWGS_WL - li));
                    nextl[li] = (int)atomicExch(&bhead[bk], (uint32_t)(li + 1));
                    spc[li] = cons;
                    // walk identity: the action, or the lane itself for explicit per-activation walks
                    if (maxc > 1) skey[li] = make_uint2((uint32_t)slot, a != (int)OWGS_REC_NOACT ? (uint32_t)a : 0x80000000u | li);
                }
                const int cft = SC_CFT + par * CFT_N + (int)(((uint32_t)slot * 2654435761u) >> (32 - CFT_LOG2));
                if (act && maxc > 1 && kind == K_FALLBACK) atomicMin(&sc[cft], li);
                if (own && li < OWGS_WL) spt[li] = part ? t : -1;
                LDS_SYNC_T(3);
                // (fallback+buckets accrue to PT(6));
                PT(3);
                // ------------------------------------------------ validate: known to fit?
                bool nf = false;
#ifdef OWGS_STOP_REASONS
                int why = 0;
#endif
                if (part) {
                    const bool first = fst[bk] == (uint32_t)(OWGS_WL - li);
                    // fits at t: the lowest lane of its bucket, or every lane of the pass at t fits, or (walking the
                    // bucket's lanes) the lanes before this one at t leave room for it
                    // (a concurrent lane that takes a free slot of a container needs no memory (NS:57-82): the
                    // container is an earlier commit, or an earlier lane of the pass opens it -- if that lane does
                    // not fit, it stops the pass before this one)
                    bool fit = first || P[t] >= 0 || (maxc > 1 && kind == K_TARGET && cons == 0);
                    if (!fit && kind != K_FALLBACK) {
                        int pf = 0, tot = 0;
                        for (int j = (int)bhead[bk] - 1; j >= 0; j = nextl[j] - 1)
                            if (spt[j] == t) {
                                const int cj = spc[j];
                                tot += cj;
                                pf += j < li ? cj : 0;
                            }
                        fit = P[t] + tot - pf - cons >= 0;
                    }
                    bool kf;
                    if (maxc == 1) {
                        kf = fit || kind == K_FALLBACK;
                    } else {
                        const int cfb = sc[cft];  // first forced acquire of this key in the pass
                        if (kind == K_FALLBACK) kf = first && cfb >= li;
                        else kf = fit && cfb > li;
                        // an earlier lane of this pass has the same fqn under another action (another walk): its
                        // unit at t shifts this lane's unit index (and memory take) -- uncertain when one of them
                        // shares the target (a shared earlier walk step is caught at that lane)
                        if (kf && pk1 > f) {
                            for (int j = (int)bhead[bk] - 1; j >= 0; j = nextl[j] - 1)
                                if (j >= f && j < li && spt[j] == t) {
                                    const uint2 kj = skey[j];
                                    const uint32_t wid = a != (int)OWGS_REC_NOACT ? (uint32_t)a : 0x80000000u | li;
                                    if (kj.x == (uint32_t)slot && kj.y != wid) kf = false;
                                }
                        }
                    }
                    nf = !kf;
#ifdef OWGS_STOP_REASONS
                    if (nf) {
                        const int cfb = sc[cft];
                        why = maxc == 1 ? 1 : pk1 > f ? 5 : kind == K_FALLBACK ? (!first ? 2 : 4) : (cfb <= li ? 4 : 3);
                    }
#endif
                }
#if OWGS_EXT
                if (act) {  // the summary the in-pass re-decisions read (commit phase)
                    const bool exempt = !part || kind == K_FALLBACK;
                    const bool rd = maxc == 1 && pool_mode == 0 && kind == K_TARGET && a != (int)OWGS_REC_NOACT;
                    fxa[li] = make_uint4(((uint32_t)a & OWGS_REC_NOACT) | (nf ? FX_NF : 0u) | (exempt ? FX_EXEMPT : 0u) |
                                             (rd ? FX_OK : 0u),
                                         (part ? (uint32_t)t : FX_NOT) | ((uint32_t)s_t << 16), rc4.x,
                                         (uint32_t)mem | ((part && cons) ? 0x80000000u : 0u));
#if OWGS_PRE
                    // pre-walk: a lane that does not fit walks on from its speculated step now, on the permits every
                    // earlier lane of the pass leaves where it speculated: the tentative permits (all lanes' takes)
                    // plus the takes of this lane and the later ones at each probed invoker (bucket lists).  That is
                    // this lane's exact decision unless an earlier lane is re-decided first; the I/O wave checks that
                    // (commit phase) with the signature of the invokers skipped here.  Result -> lq[li] (free after
                    // the speculation), invalid unless a target was found within PRE_G groups.
                    uint4 pre = make_uint4(0u, 0u, 0u, 0u);
                    if (nf && rd) {
                        const int base = pool ? A.n_ids - nb : 0;
                        uint32_t blo = 0u, bhi = 0u;
                        auto bmark = [&](int x) {
                            const uint32_t h = pre_bit(x);
                            if (h < 32u) blo |= 1u << h;
                            else bhi |= 1u << (h - 32u);
                        };
                        bmark(t);  // (a lane re-decided away from t leaves room there)
                        int s = s_t + 1;
                        int pos = mod_fast(home + s * step, n, __builtin_amdgcn_rcpf((float)n));
                        bool found = false;
                        int tp = 0, sp = 0;
#pragma unroll 1
                        for (int g4 = 0; g4 < PRE_G && !found && s < n; ++g4) {
                            int ps[4], pv[4];
                            uint32_t bh[4];
                            int pp = pos;
#pragma unroll
                            for (int k = 0; k < 4; ++k) {
                                ps[k] = base + pp;
                                pv[k] = P[ps[k]];
                                bh[k] = bhead[((uint32_t)ps[k] * 2654435761u) >> (32 - OWGS_NBK_LOG2)];
                                pp += step;
                                pp -= pp >= n ? n : 0;
                            }
#pragma unroll
                            for (int k = 0; k < 4; ++k) {
                                if (found || s + k >= n || pv[k] >= OWGS_PLIM) continue;  // (unusable: stays so)
                                int room = pv[k];
                                for (int m = (int)bh[k] - 1; m >= 0; m = nextl[m] - 1)
                                    if (m > li && spt[m] == ps[k]) room += spc[m];  // later lanes' takes back
                                if (room >= mem) {
                                    found = true;
                                    tp = ps[k];
                                    sp = s + k;
                                } else {
                                    bmark(ps[k]);
                                }
                            }
                            s += 4;
                            pos = pp;
                        }
                        if (found) pre = make_uint4(0x80000000u | (uint32_t)tp, (uint32_t)sp, blo, bhi);
                    }
                    lq[li] = pre;
#endif
                }
#endif
                if (!io) {
                    // (the lanes of a wave are not in stream order) the wave's smallest such lane
                    if (__ballot(nf)) {
                        const int lm = -wave_max(nf ? -li : -OWGS_WL);
                        if (lane == 0) atomicMin(&sc[SC_LMIN + par], lm);
                    }
                }
                LDS_SYNC_T(4);
                PT(4);
                // ------------------------------------------------ commit lanes [f, l)
                int l = sc[SC_LMIN + par];
                bool ovf_w = false;  // this lane wrote an overflow entry
#ifdef OWGS_PROF_COMMIT
                const u64 tc0 = memtime_pinned();
#endif
                if (l <= f) {  // the frontier lane is always exact; never loop without progress
                    l = f + 1;
                    err |= OWGS_ERR_INTERNAL;
                }
#if OWGS_EXT
                // ---- in-pass re-decisions.  Every lane before l is exact.  Lane l (maxConcurrent == 1, identity pool,
                // a walk target) is decided exactly here instead of in another pass: the state it sees is the
                // frontier minus the lanes before it = the tentative permits once the lanes from l on give their takes
                // back (below), and its walk resumes at its speculated step (every earlier step of its walk had no
                // capacity left for it: its earlier lanes of the same action took those units, others only take
                // more).  Moving l from its speculated target t to its true target t' only adds room at t and takes
                // room at t', so a later lane that was known to fit stays exact unless it targets t' or belongs to
                // l's action (its rank assumed l at t); forced acquires of the pass do not depend on either.  The
                // next lane that is not known to fit, or hits t' / l's action, is the next stop: re-decided the same
                // way, up to EXT_MAX per pass (the I/O wave does this; it holds no lanes).
                const int l0 = l;
                // (the first stop must be re-decidable, else the pass ends as before)
                const bool fixup = l < len && (fxa[l].x & FX_OK);
                if (fixup) {
                    if (io) {
#ifdef OWGS_EXT_PROF
                        const u64 tx0 = memtime_pinned();
                        u64 tq_prev = tx0;
#endif
                        // every lane from l on gives its tentative take back: the permits are then exactly what lane l
                        // sees (the frontier minus the lanes before it); the lanes that commit add theirs again below
                        for (int k0 = l; k0 < len; k0 += 64) {
                            const int k = k0 + lane;
                            if (k < len) {
                                const uint4 f2 = fxa[k];
                                if (f2.w >> 31) atomicAdd(&P[(int)(f2.y & 0xFFFFu)], (int)(f2.w & OWGS_AM_MEM_MASK));
                            }
                        }
                        int L = l, nE = 0;
                        // the re-decided lanes' targets and actions as hashed 2048-bit sets over the wave's lanes
                        uint32_t set_t = 0u, set_a = 0u;
                        auto hsh = [](uint32_t v) { return (v * 2654435761u) >> 21; };
                        auto inset = [&](uint32_t bits, uint32_t h) {  // (whole wave: ds_bpermute)
                            return ((uint32_t)__shfl((int)bits, (int)(h >> 5), 64) >> (h & 31u)) & 1u;
                        };
                        // lane i: the speculated target a re-decided lane left (room grew there), -1 = none
                        int src = -1;
                        (void)src;  // (read by the pre-walk check only)
                        // the pools' usable-permit bounds: only this wave changes them in this phase
                        int u0 = sc[SC_U0], u1 = sc[SC_U1];
                        // the stop lane's summary and pre-walk, carried from the scan that found it (uniform)
                        uint4 fx = fxa[L], px = lq[L];
                        bool a_hit = false;  // its action was re-decided in this pass (none yet)
                        while (L < len && nE < EXT_MAX) {
                            // a re-decided action's next lane waits for the next pass (its rank, and the hot table of
                            // its action, no longer hold: it re-speculates with its action's other lanes)
                            const uint32_t fxx = __builtin_amdgcn_readfirstlane(fx.x);
                            if (!(fxx & FX_OK) || a_hit) break;
                            // (uniform: scalar registers, and the pool's fields become scalar loads -- a vector load
                            // here would wait for the I/O wave's own prefetch stream, vmcnt(0))
                            const uint32_t fy = __builtin_amdgcn_readfirstlane(fx.y);
                            const uint32_t fz = __builtin_amdgcn_readfirstlane(fx.z), fw = __builtin_amdgcn_readfirstlane(fx.w);
                            const int hm_ = (int)(fz & OWGS_AM_POS_MASK), st_ = (int)((fz >> 15) & OWGS_AM_POS_MASK);
                            const int pl_ = (fz & OWGS_AM_POOL) ? 1 : 0;
                            const int mm = (int)(fw & OWGS_AM_MEM_MASK);
                            const int nn = pl_ ? nb : nm, base = pl_ ? A.n_ids - nb : 0;
                            int kn = K_FALLBACK, tn = -1, sn = nn;
#ifdef OWGS_EXT_PROF
                            const u64 tq0 = memtime_pinned();
                            xp_ph[0] += tq0 - tq_prev;
#endif
                            bool done = false;
#if OWGS_PRE
                            // the lane's own pre-walk (validate) assumed every earlier lane where it speculated.  Since
                            // then the re-decided lanes moved: room grew at their old targets (none of them may be a
                            // step the pre-walk skipped: signature test) and shrank at their new ones (the permits
                            // here are exact for this lane: the target must still hold it)
                            const uint32_t pxx = __builtin_amdgcn_readfirstlane(px.x);
                            if (pxx >> 31) {
                                const uint32_t blo = __builtin_amdgcn_readfirstlane(px.z), bhi = __builtin_amdgcn_readfirstlane(px.w);
                                const uint32_t hb = pre_bit(src);
                                const bool hit = src >= 0 && (((hb < 32u ? blo >> hb : bhi >> (hb - 32u)) & 1u) != 0u);
                                if (!__ballot(hit)) {
                                    const int tp = (int)(pxx & 0x7FFFFFFFu);
                                    const int v = P[tp];
                                    if (v < OWGS_PLIM && v >= mm) {
                                        kn = K_TARGET;
                                        tn = tp;
                                        sn = (int)__builtin_amdgcn_readfirstlane(px.y);
                                        done = true;
                                        ++st_pre;
                                    }
                                }
                            }
#endif
                            // every usable permit count below mem: the walk fails (U bounds the frontier, whose
                            // permits bound this lane's)
                            if (!done) done = mm > (pl_ ? u1 : u0) && ((A.shortcut_ok >> pl_) & 1);
                            if (!done) {
                                const float rnn = __builtin_amdgcn_rcpf((float)nn);
                                int s0 = (int)(fy >> 16);
                                for (int rd = 0; rd < EXT_ROUNDS; ++rd) {
#ifdef OWGS_EXT_PROF
                                    ++xp_rounds;
#endif
                                    if (s0 >= nn) {  // every position probed: forced acquire (SCPB:417-424)
                                        done = true;
                                        break;
                                    }
                                    // walk steps s0 + lane and s0 + 64 + lane ((s0 + 127) * step < 2^31)
                                    const int xa = base + mod_fast(hm_ + (s0 + lane) * st_, nn, rnn);
                                    const int xb = base + mod_fast(hm_ + (s0 + 64 + lane) * st_, nn, rnn);
                                    const bool ia = s0 + lane < nn, ib = s0 + 64 + lane < nn;
                                    const int va = ia ? P[xa] : OWGS_PENC, vb = ib ? P[xb] : OWGS_PENC;
                                    const bool fa = va < OWGS_PLIM && va >= mm;  // (usable: flag folded in)
                                    const bool fb = vb < OWGS_PLIM && vb >= mm;
                                    const u64 ma = __ballot(fa), mb = __ballot(fb);
                                    if (ma | mb) {
                                        const int q = ma ? ffs64(ma) : ffs64(mb);
                                        kn = K_TARGET;
                                        tn = __builtin_amdgcn_readlane(ma ? xa : xb, q);
                                        sn = s0 + q + (ma ? 0 : 64);
                                        done = true;
                                        break;
                                    }
                                    s0 += 128;
                                }
                            }
#ifdef OWGS_EXT_PROF
                            const u64 tq1 = memtime_pinned();
                            xp_ph[1] += tq1 - tq0;
#endif
                            if (!done) break;  // a long walk: the next pass takes this lane
                            if (kn == K_FALLBACK) {
                                const int hc = pl_ ? hb_e : hm_e;
                                if (hc <= 0) break;
                                // (explicit per-activation sequence numbers: the ordinary path -- a global load here
                                // would wait for the I/O wave's prefetch stream)
                                if (seqp) break;
                                const u64 sq = A.seq_base + (u64)(c0 + L);
                                tn = select_pool(E, base, (int)rng_index(A.rng_seed, sq, (uint32_t)hc), pl_ ? full_b : full_m);
                                if (tn < 0 || tn >= n_slots) break;  // (a throwing lane: the ordinary path)
                                // a failed full walk at rank 0 proves every usable permit of the pool < mem
                                if (pl_) u1 = min(u1, mm - 1);
                                else u0 = min(u0, mm - 1);
                            }
                            if (lane == 0) {
                                atomicSub(&P[tn], mm);
                                *(uint2*)&fxa[L] = make_uint2(fxx | FX_DONE | ((uint32_t)kn << 28), (uint32_t)tn | ((uint32_t)sn << 16));
                                if (kn == K_FALLBACK) atomicMin(&sc[pl_ ? SC_U1 : SC_U0], mm - 1);  // rank 0 failed
                            }
                            {
                                const uint32_t h1 = hsh((uint32_t)tn), h2 = hsh(fxx & OWGS_REC_NOACT);
                                if (lane == (int)(h1 >> 5)) set_t |= 1u << (h1 & 31u);
                                if (lane == (int)(h2 >> 5)) set_a |= 1u << (h2 & 31u);
                                if (lane == nE) src = (int)(fy & 0xFFFFu);  // the room it left
                            }
                            ++nE;
#ifdef OWGS_EXT_PROF
                            const u64 tq2 = memtime_pinned();
                            xp_ph[2] += tq2 - tq1;
#endif
                            // the next stop after L: not known to fit, or meets a re-decided target or action
                            int k0 = L + 1;
                            L = len;
                            for (; k0 < len; k0 += 64) {
#ifdef OWGS_EXT_PROF
                                ++xp_scans;
#endif
                                const int k = k0 + lane;
                                uint4 f2 = make_uint4(FX_EXEMPT, FX_NOT, 0u, 0u), p2 = make_uint4(0u, 0u, 0u, 0u);
                                if (k < len) {
                                    f2 = fxa[k];
                                    p2 = lq[k];
                                }
                                const uint32_t tk = f2.y & 0xFFFFu;
                                const uint32_t ab = inset(set_a, hsh(f2.x & OWGS_REC_NOACT));
                                const bool cl = (ab | inset(set_t, hsh(tk))) != 0u;
                                const bool stop = k < len && ((f2.x & FX_NF) || (!(f2.x & FX_EXEMPT) && cl));
                                const u64 sm = __ballot(stop);
                                const int q = sm ? ffs64(sm) : 64;
                                // the lanes before the stop commit where they speculated: their takes again
                                if (lane < q && (f2.w >> 31)) atomicSub(&P[(int)tk], (int)(f2.w & OWGS_AM_MEM_MASK));
                                if (sm) {
                                    L = k0 + q;
                                    fx = make_uint4(__builtin_amdgcn_readlane(f2.x, q), __builtin_amdgcn_readlane(f2.y, q),
                                                    __builtin_amdgcn_readlane(f2.z, q), __builtin_amdgcn_readlane(f2.w, q));
                                    px = make_uint4(__builtin_amdgcn_readlane(p2.x, q), __builtin_amdgcn_readlane(p2.y, q),
                                                    __builtin_amdgcn_readlane(p2.z, q), __builtin_amdgcn_readlane(p2.w, q));
                                    a_hit = __builtin_amdgcn_readlane(ab, q) != 0u;
                                    break;
                                }
                            }
#ifdef OWGS_EXT_PROF
                            tq_prev = memtime_pinned();
                            xp_ph[3] += tq_prev - tq2;
#endif
                        }
                        // lanes from the limit on that meet a re-decided lane's target or action must speculate again
                        // (their validation assumed the re-decided lanes where they speculated: a kept one would
                        // keep a target whose room is gone or a rank that no longer holds)
                        if (nE > 0)
                            for (int k0 = L; k0 < len; k0 += 64) {
                                const int k = k0 + lane;
                                uint4 f2 = make_uint4(FX_EXEMPT, FX_NOT, 0u, 0u);
                                if (k < len) f2 = fxa[k];
                                const bool cl = (inset(set_a, hsh(f2.x & OWGS_REC_NOACT)) | inset(set_t, hsh(f2.y & 0xFFFFu))) != 0u;
                                if (k < len && !(f2.x & (FX_EXEMPT | FX_DONE)) && cl) fxa[k].x = f2.x | FX_CLASH;
                            }
                        st_ext += (uint32_t)nE;
#ifdef OWGS_EXT_PROF
                        xp_cyc += memtime_pinned() - tx0;
#endif
                        if (lane == 0) {
                            sc[SC_LFIN] = L;
                            sc[SC_NEXT] = nE;
                        }
                    }
                    LDS_SYNC_T(9);
                    l = sc[SC_LFIN];
                }
                if (act && li >= l0 && li < l) {  // re-decided in this pass: its true decision
                    const uint2 fo = *(const uint2*)&fxa[li];
                    if (fo.x & FX_DONE) {
                        kind = (int)(fo.x >> 28);
                        t = (int)(fo.y & 0xFFFFu);
                        s_t = (int)(fo.y >> 16);
                    }
                }
#endif
#ifdef OWGS_STOP_REASONS
                if (li == l && why) atomicAdd(&A.stats[6], 1ull << (12 * (why - 1)));
#endif
                if (act && li < l) {
                    const int outv = kind == K_NONE ? OWGS_NONE_V : (kind == K_THROW ? OWGS_THROW_V : t);
#ifndef OWGS_EXP_NOSTORE
                    A.out_inv[i] = outv;
                    A.out_flags[i] = kind == K_FALLBACK ? 1 : 0;
#endif
                    if (kind == K_FALLBACK) ++st_fb;
#ifndef OWGS_EXP_NOSTORE
                    if (relx >= 0) {  // the release record its completion reads (a plain store, no atomics)
                        const uint32_t inv15 = outv >= 0 ? (uint32_t)outv : OWGS_RR_NOINV;
                        A.rel_rec[relx] = make_uint2(inv15 | ((uint32_t)mem << 15),
                                                     (uint32_t)slot | ((uint32_t)maxc << 17));
                    }
#endif
                    // walk cursor + chunk rank base, written by the last committed lane of the action
                    if (a != (int)OWGS_REC_NOACT && (nxt == (int)OWGS_REC_NONEXT || nxt >= l)) {
                        uint32_t ns = cw & 0x7FFFu;
                        if (cok) {
                            if (kind == K_TARGET) ns = (uint32_t)s_t;
                            else if (kind == K_FALLBACK) ns = maxc == 1 ? (uint32_t)n : fallback_cursor(t);
                        }
                        ccw[lead] = ((uint32_t)(occ + 1) << 15) | ns;
                        if (cok && a != (int)OWGS_REC_NOACT && ns != (cw & 0x7FFFu)) {
#ifndef OWGS_EXP_NOGCUR  // (diagnostic: no cursor stores; later chunks walk from the batch's first step)
                            A.gcur[a] = (btag << 15) | ns;  // for the later chunks of this batch
#endif
                            if (kind == K_FALLBACK && maxc > 1) {
                                // backward move: the next chunk's gathered cursors predate it (see `stale`), and
                                // the store must reach L2 before the chunk after that gathers again.  The gather is
                                // this workgroup's I/O wave reading L2 directly (sc1, same XCD), so the store's
                                // completion is enough: vmcnt(0) here, not an agent-scope fence -- that one writes
                                // back every dirty line of the XCD's L2 (buffer_wbl2), partial output lines included
                                sc[SC_CBWD] = g + 1;
                                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                            }
                        }
                    }
                    // NestedSemaphore concurrency entry: the last committed lane of the (invoker, fqn) group
                    if (maxc > 1 && (kind == K_TARGET || kind == K_FALLBACK)) {
                        const bool writer = kind == K_FALLBACK || nxt == (int)OWGS_REC_NONEXT || nxt >= l ||
                                            spt[nxt] != t;
                        if (writer) {
                            const int c0v = (int)(cval & OWGS_CT_C_MASK), ops0 = ct_ops(cval);
                            const int jn = kind == K_FALLBACK ? 1 : ks + 1;
                            const int c1 = jn <= c0v ? c0v - jn
                                                     : (maxc - 1 - mod_fast(jn - c0v - 1, maxc,
                                                                            __builtin_amdgcn_rcpf((float)maxc)));
                            const int ops1 = ops0 + jn;
                            if (ops1 > OWGS_MAX_OPS) err |= OWGS_ERR_OPS;
                            int ix = cidx;
                            const uint32_t key = ct_key(t, slot), nv = ct_val(c1, ops1);
                            if (ix < 0) {  // absent when speculated (a kept lane's group may have created it since)
                                uint32_t vv;
                                if (ovf_on) {
                                    const int oj = ovf_find(A.ovf, key, &vv);
                                    if (oj >= 0) ix = OWGS_CTC + oj;
                                }
                                if (ix < 0) {
                                    if (sc[SC_USED] < OWGS_CT_LDS_FILL || !OWGS_OVF || A.ovf.cap <= 0) {  // find or insert
                                        int fresh = 0;
                                        ix = ct_upsertv(ct, key, &fresh);
                                        if (fresh) atomicAdd(&sc[SC_USED], 1);
                                    } else {
                                        ix = ct_findv(ct, key, &vv);  // the nearly full primary may hold it
                                    }
                                }
                                if (ix < 0 && OWGS_OVF && A.ovf.cap > 0) {  // the primary is full: the key goes to the overflow
                                    const int oj = ovf_insert(A.ovf, key, nv);
                                    if (oj >= 0) {
                                        ix = OWGS_CTC + oj;
                                        atomicAdd(&sc[SC_OVF], 1);
                                    }
                                }
                            }
                            if (ix < 0) err |= OWGS_ERR_CTAB_FULL;
                            else if (ix < OWGS_CTC) ct[ix].y = nv;
                            else {
                                ovf_st_val(A.ovf.t, ix - OWGS_CTC, nv);
                                ovf_w = true;
                            }
                        }
                    }
                    // a failed full walk at rank 0 proves every usable permit of the pool < mem from now on
                    if (kind == K_FALLBACK && maxc == 1 && r == 0) atomicMin(&sc[pool ? SC_U1 : SC_U0], mem - 1);
                    pending = false;
                }
#ifdef OWGS_PROF_COMMIT
                const u64 tc1 = memtime_pinned();
#endif
                if (part) {
#if OWGS_EXT
                    if (li >= l && cons && !fixup) atomicAdd(&P[t], cons);  // not committed: give the memory back
#else
                    if (li >= l && cons) atomicAdd(&P[t], cons);  // not committed: give the memory back
#endif
                    fst[bk] = 0u;
                    bhead[bk] = 0u;
                }
                if (act && li >= l) {
                    keep = !nf;
#if OWGS_EXT
                    if (keep && fixup && sc[SC_NEXT] > 0 && (fxa[li].x & FX_CLASH)) keep = false;
#endif
                    if (!keep && hs >= 0) hflag[hs] = l;  // the action's hot table is needed in the next pass
                    if (!keep && maxc > 1) cdirty[(par ^ 1) * OWGS_WL + lead] = 1;
                }
                if (io && l >= len) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // chunk g+1 staged
#ifdef OWGS_PROF_COMMIT
                if (!io && lane == 0) {
                    const u64 tc2 = memtime_pinned();
                    atomicMax(&pfw[0], (int)(tc1 - tc0));
                    atomicMax(&pfw[1], (int)(tc2 - tc1));
                }
#endif
                if (tid < CFT_N) sc[SC_CFT + (par ^ 1) * CFT_N + tid] = OWGS_WL;  // read in this pass's other half
                if (tid == 0) {
                    sc[SC_LQN] = 0;  // the queue of this pass was drained before barrier 2
                    sc[SC_LQH] = 0;
                    sc[SC_NHOT] = 0;  // read at the chunk start, before this pass's barriers
                    sc[SC_LMIN + (par ^ 1)] = OWGS_WL;
                    if (l < len) ++st_stop;
                }
                if (!io && __ballot(ovf_w)) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // visible next pass
                LDS_SYNC_T(5);
                PT(5);
#ifdef OWGS_PROFILE
#ifdef OWGS_PROF_COMMIT
                if (tid == 0) {  // slowest wave: committing lanes, giving back and resetting
                    pt_x[0] += (u64)pfw[0];
                    pt_x[1] += (u64)pfw[1];
                    pfw[0] = 0;
                    pfw[1] = 0;
                }
#elif !defined(OWGS_PROF_SPLIT)
                if (tid == 0) pt_x[f == 0 ? 0 : 1] += memtime_pinned() - tpass0;  // first vs repeated passes
#endif
#endif
                f = l;
                par ^= 1;
            }
        }
        // U bounds are per batch (releases raise permits)
        if (tid == 0) {
            sc[SC_U0] = (int)0x80000000;
            sc[SC_U1] = (int)0x80000000;
        }
        lds_sync();
    }

    // ---------------------------------------------------------------- LDS -> state
#ifdef OWGS_PROFILE
    const u64 tk2 = memtime_pinned();
#endif
    for (int i = tid; i < n_slots; i += OWGS_NT) {
        const int v = P[i];
        A.permits[i] = v >= OWGS_PLIM ? v - OWGS_PENC : v;
    }
    if (tid == 0 && A.ovf.cap > 0) __hip_atomic_store(A.ovf.cnt, sc[SC_OVF], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0 && A.ct_clast) *A.ct_clast = sc[SC_CLAST];
    for (int i = tid; i < OWGS_CTC; i += OWGS_NT) {
        const uint2 e = ct[i];
        A.ct_keys[i] = e.x;
        A.ct_vals[i] = e.y;
    }
    if (A.out_copy_n16 > 0) {  // (uniform) this launch's outputs (HBM) into the caller's pinned block, 16 B per store
        __syncthreads();                                      // every thread's decision and flag stores done ...
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");    // ... and read past this CU's L1
        for (int k = tid; k < A.out_copy_n16; k += OWGS_NT) A.out_copy_dst[k] = A.out_copy_src[k];
    }
    if (A.err_host || A.ovf_host) {  // (uniform) the caller's pinned words: every thread's error bits first
        if (tid == 0) sc[SC_IRR] = 0;
        lds_sync();
        if (err) atomicOr(&sc[SC_IRR], (int)err);
        lds_sync();
        if (tid == 0) {
            const int e = sc[SC_IRR];
            if (e) atomicOr(A.err, e);
            if (A.err_host) *A.err_host = __hip_atomic_load(A.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) | e;
            if (A.ovf_host) *A.ovf_host = sc[SC_OVF];
        }
        err = 0;
    }
    if (err) atomicOr(A.err, (int)err);
    if (A.stats_next && tid < OWGS_NSTATS) A.stats_next[tid] = 0ull;  // the next launch's counters start at zero
#ifdef OWGS_PROFILE
    if (tid == 0 && A.stats) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const u64 tk3 = memtime_pinned();
        atomicAdd(&A.stats[40], tk1 - tk0);
        atomicAdd(&A.stats[41], tk2 - tk1);
        atomicAdd(&A.stats[42], tk3 - tk2);
    }
#endif
    if (A.stats) {
        atomicAdd(&A.stats[OWGS_ST_PROBES], (u64)st_probe);  // (the I/O wave's: its share of the hot walks)
        if (lane == 0) atomicAdd(&A.stats[OWGS_ST_LONG], (u64)st_long);
        if (!io) {
            atomicAdd(&A.stats[OWGS_ST_FALLBACKS], (u64)st_fb);
#if !defined(OWGS_PROFILE) && !defined(OWGS_STOP_REASONS)
            atomicAdd(&A.stats[6], (u64)st_gprobe);
            atomicAdd(&A.stats[7], (u64)st_glane);
#endif
        }
#ifdef OWGS_PROFILE
        if (!io && lane == 0)
            for (int k = 2; k < 10; ++k) atomicAdd(&A.stats[16 + k], pw_c[k]);
        if (tid == 0) {  // wave 0: marks sit right after barriers, so the intervals are the critical path
            atomicAdd(&A.stats[28], pw_c[10]);
            atomicAdd(&A.stats[29], pw_c[11]);
            atomicAdd(&A.stats[30], sc_prof_q);
            atomicAdd(&A.stats[26], pt_y[0]);
            atomicAdd(&A.stats[27], pt_y[1]);
            atomicAdd(&A.stats[16], pw_c[0]);
            atomicAdd(&A.stats[17], pt_x[2]);
            for (int k = 0; k < 8; ++k) atomicAdd(&A.stats[8 + k], pt_acc[k]);
            atomicAdd(&A.stats[6], pt_x[0]);
            atomicAdd(&A.stats[7], pt_x[1]);
        }
#endif
        if (io && lane == 0) atomicAdd(&A.stats[31], (u64)st_ext | ((u64)st_pre << 32));
#ifdef OWGS_EXT_PROF
        if (io && lane == 0) {
            atomicAdd(&A.stats[28], xp_cyc);
            atomicAdd(&A.stats[29], xp_rounds);
            atomicAdd(&A.stats[30], xp_scans);
            for (int k = 0; k < 4; ++k) atomicAdd(&A.stats[20 + k], xp_ph[k]);
        }
#endif
        if (tid == 0) {
            atomicAdd(&A.stats[OWGS_ST_PASSES], (u64)st_pass);
            atomicAdd(&A.stats[OWGS_ST_CHUNKS], (u64)st_chunk);
            atomicAdd(&A.stats[OWGS_ST_STOPS], (u64)st_stop);
        }
    }
}

// one shard: the argument block behind a (uniform) workgroup index, like the multi-shard kernel -- read from the
// kernarg segment where each phase needs it instead of held in registers across the whole body (a by-value block
// is hoisted: 256 VGPRs with scratch spills against 233 without)
struct OwgsEngineOne {
    OwgsEngineArgs a[1];
};
template <int FEAT>
__global__ __launch_bounds__(OWGS_NT, 1) void owgs_engine_kernel(OwgsEngineOne M) { owgs_engine_body<FEAT>(M.a[blockIdx.x]); }

// several controller shards in one launch: workgroup k replays shard k (its own LDS image, state and stream); the
// arguments stay in the kernarg segment, so every field is still a scalar load
struct OwgsEngineMulti {
    OwgsEngineArgs a[OWGS_MULTI_MAX];
};
template <int FEAT>
__global__ __launch_bounds__(OWGS_NT, 1) void owgs_engine_multi_kernel(OwgsEngineMulti M) {
    owgs_engine_body<FEAT>(M.a[blockIdx.x]);
}
// more shards than the kernarg segment holds: the argument blocks in HBM (uniform per workgroup, read-only)
template <int FEAT>
__global__ __launch_bounds__(OWGS_NT, 1) void owgs_engine_multi_dev_kernel(const OwgsEngineArgs* __restrict__ As) {
    owgs_engine_body<FEAT>(As[blockIdx.x]);
}

// ------------------------------------------------------------------------------------------------ explicit releases
// owgs_release_batch: releases in stream order, 64 at a time.  maxConcurrent == 1: FS.release (FS:117-120) with the
// overflow Error leaving the state unchanged; concurrent: RS.release(1, true) applied rank+1 times inside each group
// of 64 (NS:98-113), NoSuchElementException when the entry is absent or already removed.
// Parallel front end.  Every memory release only adds to a permit count, so releases commute unless one of them would
// overflow (FS:48-50).  owgs_rel_bound_kernel sums, per invoker, an upper bound of what the batch can return (every
// release's memory); if no invoker can overflow, the maxConcurrent == 1 releases are applied in parallel with atomics
// and the concurrent ones grouped by NestedSemaphore entry (stable sort) and applied in closed form per entry;
// otherwise every release goes through the ordered kernel (the exact sequential path).
__global__ __launch_bounds__(256) void owgs_rel_bound_kernel(OwgsReleaseArgs R) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= R.n) return;
    const int inv = R.inv[r];
    const bool in = inv >= 0 && inv < R.n_slots;
    if (in) atomicAdd(&R.bound[inv], (unsigned long long)R.mem[r]);
    if (!in && R.flags) R.flags[r] = inv < 0 ? OWGS_REL_NOENTRY_BIT : 0;  // invokerSlots.lift -> no-op (SCPB:329)
}
__global__ __launch_bounds__(256) void owgs_rel_check_kernel(OwgsReleaseArgs R) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= R.n_slots) return;
    if ((long long)R.permits[i] + (long long)R.bound[i] > 0x7FFFFFFFll) atomicOr(R.risk, 1);
    // keys in the overflow table: every release takes the ordered kernel (the grouped front end indexes the primary)
    if (i == 0 && R.ovf.cap > 0 && *R.ovf.cnt > 0) atomicOr(R.risk, 1);
}
__global__ __launch_bounds__(256) void owgs_rel_apply_kernel(OwgsReleaseArgs R) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= R.n) return;
    const int inv = R.inv[r];
    const bool in = inv >= 0 && inv < R.n_slots;
    const bool risk = *R.risk != 0;
    uint8_t sel = 0;
    uint32_t key = OWGS_CTC;  // no concurrent entry: sorts after every entry
    if (in) {
        if (risk) {
            sel = 1;
        } else if (R.maxc[r] == 1) {
            atomicAdd(&R.permits[inv], R.mem[r]);
            if (R.flags) R.flags[r] = 0;
        } else {
            const uint32_t k = ct_key(inv, R.slot[r]);
            const int ix = ct_find(R.ct_keys, k);
            const uint32_t v = ix >= 0 ? R.ct_vals[ix] : 0u;
            if ((R.w.cap > 0 && R.w.wkey[R.slot[r]] > 0 && w_find(R.w, k) >= 0) || (ix >= 0 && ct_ops(v) <= 0)) {
                sel = 1;  // a watched pair, or an entry counting at or below zero: the ordered kernel, one by one
            } else if (ix < 0) {
                if (R.flags) R.flags[r] = OWGS_REL_NOSUCH_BIT;  // NoSuchElementException (NS:103)
            } else {
                key = (uint32_t)ix;
            }
        }
    }
    R.sel_flag[r] = sel;
    R.ckey[r] = key;
    R.cval[r] = r;
}

// concurrent releases of one entry, in stream order (sorted by entry, stable): RS.release(1, true) (RS:99-108,
// NS:98-113) in closed form -- release q of the entry (0-based) finds the entry when q < opCount and returns the
// memory iff (c0 + q + 1) % maxConcurrent == 0; the entry ends at c = (c0 + j) % maxConcurrent, opCount - j
__global__ __launch_bounds__(256) void owgs_rel_cseg_kernel(OwgsReleaseArgs R) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= R.n) return;
    const uint32_t k = R.ckey_s[p];
    if (k >= OWGS_CTC) return;
    if (p == 0 || R.ckey_s[p - 1] != k) R.cbeg[k] = p;
    if (p == R.n - 1 || R.ckey_s[p + 1] != k) R.cend[k] = p + 1;
}
__global__ __launch_bounds__(256) void owgs_rel_capply_kernel(OwgsReleaseArgs R) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= R.n) return;
    const uint32_t k = R.ckey_s[p];
    if (k >= OWGS_CTC) return;
    const int r = R.cval_s[p], q = p - R.cbeg[k];
    const uint32_t v = R.ct_vals[k];
    const int c0 = (int)(v & OWGS_CT_C_MASK), o0 = ct_ops(v), maxc = R.maxc[r];
    uint8_t flag = 0;
    if (q < o0) {
        if ((c0 + q + 1) % maxc == 0) atomicAdd(&R.permits[R.inv[r]], R.mem[r]);
    } else {
        flag = OWGS_REL_NOSUCH_BIT;  // the entry was removed by an earlier release of this batch
    }
    if (R.flags) R.flags[r] = flag;
}
__global__ __launch_bounds__(256) void owgs_rel_cupdate_kernel(OwgsReleaseArgs R) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= OWGS_CTC || R.cend[k] <= R.cbeg[k]) return;
    const int r = R.cval_s[R.cbeg[k]];
    const uint32_t v = R.ct_vals[k];
    const int c0 = (int)(v & OWGS_CT_C_MASK), o0 = ct_ops(v), maxc = R.maxc[r];
    const int j = min(R.cend[k] - R.cbeg[k], o0), o1 = o0 - j;
    if (o1 == 0) {
        R.ct_keys[k] = OWGS_CT_TOMB;
        R.ct_vals[k] = 0u;
    } else {
        R.ct_vals[k] = ct_val((c0 + j) % maxc, o1);
    }
}

// the ordered part: the selected releases (all concurrent ones, or every in-range release when an overflow is
// possible) in stream order, 64 at a time.  maxConcurrent == 1: FS.release (FS:117-120) with the overflow Error
// leaving the state unchanged; concurrent: RS.release(1, true) applied rank+1 times inside each group of 64
// (NS:98-113), NoSuchElementException when the entry is absent or already removed.  Releases of watched pairs
// (owgs_watch.hip) and of entries counting at or below zero run one at a time in stream order ("serial" lanes):
// an absent watched pair with Z meets the reference's empty entry (NS:61-62), one without Z throws and lowers d.
__global__ __launch_bounds__(64) void owgs_release_seq_kernel(OwgsReleaseArgs R) {
    __shared__ uint32_t ctk[OWGS_CTC], ctv[OWGS_CTC];
    const int lane = threadIdx.x;
    int used = 0;
    for (int i = lane; i < OWGS_CTC; i += 64) {
        ctk[i] = R.ct_keys[i];
        ctv[i] = R.ct_vals[i];
        used += ctk[i] != 0u;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) used += __shfl_xor(used, d, 64);
    __syncthreads();
    const u64 lt_mask = lane == 0 ? 0ull : ((~0ull) >> (64 - lane));
    const int n_sel = *R.sel_cnt;
    bool ovf_on = R.ovf.cap > 0 && *R.ovf.cnt > 0;
    int32_t err = 0;
    for (int k0 = 0; k0 < n_sel; k0 += 64) {
        const bool valid = k0 + lane < n_sel;
        const int r = valid ? R.sel_idx[k0 + lane] : 0;
        int inv = -1, mem = 0, maxc = 1, slot = 0;
        if (valid) {
            inv = R.inv[r];
            mem = R.mem[r];
            maxc = R.maxc[r];
            slot = R.slot[r];
        }
        uint8_t flag = 0;
        bool rel = false, conc = false, ser = false;
        if (valid) {
            if (inv < 0) flag = OWGS_REL_NOENTRY_BIT;
            else if (inv >= R.n_slots) flag = 0;  // invokerSlots.lift -> no-op (SCPB:329)
            else if (maxc == 1) rel = true;
            else conc = true;
        }
        int ix = -1, c0 = 0, o0 = 0, wj = -1;
        if (conc) {
            const uint32_t key = ct_key(inv, slot);
            if (R.w.cap > 0 && R.w.wkey[slot] > 0) wj = w_find(R.w, key);
            ix = ct_find(ctk, key);
            uint32_t v = ix >= 0 ? ctv[ix] : 0u;
            if (ix < 0 && ovf_on) {  // overflow entries are indexed past the primary
                const int oj = ovf_find(R.ovf, key, &v);
                ix = oj >= 0 ? OWGS_CTC + oj : -1;
            }
            c0 = (int)(v & OWGS_CT_C_MASK);
            o0 = ct_ops(v);
            if (wj >= 0 || (ix >= 0 && o0 <= 0)) {
                ser = true;
                conc = false;
            } else if (ix < 0) {
                conc = false;
                flag = OWGS_REL_NOSUCH_BIT;
            }
        }
        // rank of each release among the group's releases of the same entry (stream order) and group size
        int rank = 0, gsz = 1;
        u64 pend = __ballot(conc);
        while (pend) {
            const int j = ffs64(pend);
            const int e = __builtin_amdgcn_readlane(ix, j);
            const u64 G = __ballot(conc && ix == e);
            if ((G >> lane) & 1) {
                rank = __popcll(G & lt_mask);
                gsz = __popcll(G);
            }
            pend &= ~G;
        }
        if (conc) {
            if (rank < o0) rel = ((c0 + rank + 1) % maxc) == 0;
            else flag = OWGS_REL_NOSUCH_BIT;  // entry already removed by an earlier release of this group
            if (rank == 0) {
                const int j = min(gsz, o0);
                const int o1 = o0 - j;
                const uint32_t nv = ct_val((c0 + j) % maxc, o1);
                if (ix >= OWGS_CTC) {
                    if (o1 == 0) ovf_st(R.ovf.t, ix - OWGS_CTC, OWGS_CT_TOMB, 0u);
                    else ovf_st_val(R.ovf.t, ix - OWGS_CTC, nv);
                } else if (o1 == 0) {
                    ctk[ix] = OWGS_CT_TOMB;
                    ctv[ix] = 0u;
                } else {
                    ctv[ix] = nv;
                }
            }
        }
        // memory releases (and the serial lanes) in stream order: lanes releasing to the same invoker are applied
        // lane by lane so the overflow Error (FS:48-50) hits exactly the releases the reference rejects
        u64 rm = __ballot(rel || ser);
        while (rm) {
            const int j = ffs64(rm);
            rm &= rm - 1;
            bool oins = false;
            if (lane == j && ser) {
                // one RS.release(1, true) (RS:99-108) against the current state of the entry (NS:98-113)
                const uint32_t key = ct_key(inv, slot);
                ix = ct_find(ctk, key);
                uint32_t v = ix >= 0 ? ctv[ix] : 0u;
                if (ix < 0 && ovf_on) {
                    const int oj = ovf_find(R.ovf, key, &v);
                    ix = oj >= 0 ? OWGS_CTC + oj : -1;
                }
                if (wj >= 0 && __hip_atomic_load(&R.w.keys[wj], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != key)
                    wj = -1;  // an earlier release of this group took the pair out of W
                const uint32_t wv = wj >= 0 ? __hip_atomic_load(&R.w.vals[wj], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
                bool apply = ix >= 0;
                if (!apply && (wv & OWGS_W_Z)) {  // the reference's empty entry from a failed try takes it
                    if (used < OWGS_CT_LDS_FILL || R.ovf.cap <= 0) {
                        int fresh = 0;
                        ix = ct_insert(ctk, key, &fresh);
                        if (ix >= 0) {
                            ctv[ix] = 0u;
                            used += fresh;
                        }
                    }
                    if (ix < 0 && R.ovf.cap > 0) {
                        const int oj = ovf_insert(R.ovf, key, 0u);
                        if (oj >= 0) {
                            ix = OWGS_CTC + oj;
                            atomicAdd(R.ovf.cnt, 1);
                            oins = true;
                        }
                    }
                    if (ix < 0) err |= OWGS_ERR_CTAB_FULL;
                    v = 0u;
                    apply = ix >= 0;
                }
                if (!apply) {
                    flag = OWGS_REL_NOSUCH_BIT;  // NoSuchElementException (NS:103)
                    if (wj >= 0) {  // one in-flight activation of the pair fewer whose release found nothing
                        const int d = (int)(wv & ~OWGS_W_Z) - 1;
                        if (d <= 0) {
                            __hip_atomic_store(&R.w.vals[wj], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            __hip_atomic_store(&R.w.keys[wj], OWGS_CT_TOMB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            atomicSub(&R.w.wkey[slot], 1);
                            atomicSub(R.w.cnt, 1);
                        } else {
                            __hip_atomic_store(&R.w.vals[wj], (uint32_t)d | (wv & OWGS_W_Z), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                        }
                    }
                } else {
                    const int cc = (int)(v & OWGS_CT_C_MASK), o1 = ct_ops(v) - 1;
                    int c1 = cc + 1;
                    const bool memrel = c1 % maxc == 0;  // RS:45-52
                    if (memrel) c1 -= maxc;
                    if (o1 < -OWGS_MAX_OPS) err |= OWGS_ERR_OPS;
                    bool removed = o1 == 0;
                    if (memrel) {
                        const int old = R.permits[inv];
                        if (old > 0x7FFFFFFF - mem) {
                            flag |= OWGS_REL_OVERFLOW_BIT;
                            removed = false;  // the Error is thrown before the map removal (NS:106-111)
                        } else {
                            R.permits[inv] = old + mem;
                        }
                    }
                    const uint32_t nk = removed ? OWGS_CT_TOMB : key, nv = removed ? 0u : ct_val(c1, o1);
                    if (ix >= OWGS_CTC) {
                        ovf_st(R.ovf.t, ix - OWGS_CTC, nk, nv);
                    } else {
                        ctk[ix] = nk;
                        ctv[ix] = nv;
                    }
                    if (removed && wj >= 0 && (wv & OWGS_W_Z))  // removal: the empty entry is gone too
                        __hip_atomic_store(&R.w.vals[wj], wv & ~OWGS_W_Z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            } else if (lane == j) {
                const int old = R.permits[inv];
                if (old > 0x7FFFFFFF - mem) flag |= OWGS_REL_OVERFLOW_BIT;
                else R.permits[inv] = old + mem;
            }
            if (__ballot(oins)) ovf_on = true;
            used = __builtin_amdgcn_readlane(used, j);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        if (valid && R.flags) R.flags[r] = flag;
        __syncthreads();
    }
    for (int i = lane; i < OWGS_CTC; i += 64) {
        R.ct_keys[i] = ctk[i];
        R.ct_vals[i] = ctv[i];
    }
    if (err) atomicOr(R.err, err);
}

// ------------------------------------------------------------------------------------------------ self-test
// DPP scan / reduction helpers against a serial computation (one wave per trial)
__global__ __launch_bounds__(64) void owgs_selftest_kernel(int* bad, int trials) {
    const int lane = threadIdx.x;
    for (int t = 0; t < trials; ++t) {
        const uint32_t h = ct_hash((uint32_t)(t * 64 + lane) * 2654435761u);
        const int v = (int)(h % 2001u) - 1000;
        const int inc = wave_incl_scan(v), mx = wave_max(v);
        int ref_inc = 0, ref_mx = (int)0x80000000;
        for (int j = 0; j < 64; ++j) {
            const int vj = __shfl(v, j, 64);
            if (j <= lane) ref_inc += vj;
            ref_mx = max(ref_mx, vj);
        }
        if (inc != ref_inc || mx != ref_mx) atomicAdd(bad, 1);
        // cap_of against integer division
        const int m = 1 + (int)(h % 4096u), pv = (int)(ct_hash(h) % 5000000u);
        const int cq = cap_of(pv, m, __builtin_amdgcn_rcpf((float)m));
        const int ref = min(pv / m, CAPMAX);
        if (cq != ref) atomicAdd(bad, 1);
    }
}

// ------------------------------------------------------------------------------------------------ launchers
#if OWGS_SHARED
extern "C" hipError_t owgs_launch_selftest(int* bad, int trials, hipStream_t s) {
    hipLaunchKernelGGL(owgs_selftest_kernel, dim3(1), dim3(64), 0, s, bad, trials);
    return hipGetLastError();
}
#endif

#if OWGS_SHARED
extern "C" hipError_t owgs_launch_hash(const OwgsHashArgs* a, hipStream_t s) {
    if (a->n <= 0) return hipSuccess;
    const int blocks = (a->n * 64 + 255) / 256;
    hipLaunchKernelGGL(owgs_hash_kernel, dim3(blocks), dim3(256), 0, s, *a);
    return hipGetLastError();
}
#endif

#if OWGS_SHARED
extern "C" hipError_t owgs_launch_lookup(const OwgsLookupArgs* a, hipStream_t s) {
    if (a->n <= 0) return hipSuccess;
    hipLaunchKernelGGL(owgs_lookup_kernel, dim3((a->n + 255) / 256), dim3(256), 0, s, *a);
    return hipGetLastError();
}
#endif

#if OWGS_SHARED
extern "C" hipError_t owgs_launch_prepare(const OwgsPrepArgs* a, hipStream_t s) {
    if (a->n <= 0) return hipSuccess;
    hipLaunchKernelGGL(owgs_prepare_kernel, dim3((a->n + 255) / 256), dim3(256), 0, s, *a);
    return hipGetLastError();
}
#endif

// chunk table + per-activation records; max_chunks >= sum of ceil(n_b / OWGS_WL)
extern "C" hipError_t OWGS_GEOM(owgs_launch_prepass)(const OwgsPrepassArgs* a, int32_t* cstart, int64_t max_chunks,
                                          hipStream_t s) {
    if (a->geom != OWGS_GEOM_TAG(OWGS_WL) || a->cw < 1 || a->cw > OWGS_WL) return hipErrorInvalidValue;
    // up to PP_INLINE batches (a shim call's runs, a span): each pre-pass workgroup finds its batch itself
    constexpr int PP_INLINE = 8;
    if (a->n_batches > PP_INLINE)
        hipLaunchKernelGGL(owgs_chunks_kernel, dim3(1), dim3(64), 0, s, a->acq_off, a->n_batches, a->cw, cstart);
    if (max_chunks <= 0) return hipGetLastError();
    OwgsPrepassArgs b = *a;
    b.cstart = a->n_batches > PP_INLINE ? cstart : nullptr;
    hipLaunchKernelGGL(owgs_prepass_kernel, dim3((unsigned)max_chunks), dim3(OWGS_WL), 0, s, b);
    return hipGetLastError();
}

// overflow table maintenance (host-driven): clear it when it holds entries; rehash its live entries into a larger one
__global__ __launch_bounds__(256) void owgs_ovf_clear_kernel(OwgsOvf O) {
    if (__hip_atomic_load(O.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < O.cap; i += (int64_t)gridDim.x * 256)
        O.t[i] = make_uint2(0u, 0u);
}
__global__ __launch_bounds__(256) void owgs_ovf_rehash_kernel(const uint2* old_t, int32_t old_cap, OwgsOvf O,
                                                              int32_t* err) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= old_cap) return;
    const uint2 e = old_t[i];
    if (e.x == 0u || e.x == OWGS_CT_TOMB) return;
    if (ovf_insert(O, e.x, e.y) < 0) atomicOr(err, OWGS_ERR_CTAB_FULL);
    else atomicAdd(O.cnt, 1);
}
#if OWGS_SHARED
extern "C" hipError_t owgs_launch_ovf_clear(const OwgsOvf* O, hipStream_t s) {
    if (O->cap <= 0) return hipSuccess;
    hipLaunchKernelGGL(owgs_ovf_clear_kernel, dim3((unsigned)std::min<int64_t>(1024, (O->cap + 255) / 256)), dim3(256),
                       0, s, *O);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemsetAsync(O->cnt, 0, sizeof(int32_t), s);
    return e;
}
#endif
#if OWGS_SHARED
extern "C" hipError_t owgs_launch_ovf_rehash(const uint2* old_t, int32_t old_cap, const OwgsOvf* O, int32_t* err,
                                            hipStream_t s) {
    if (old_cap > 0)
        hipLaunchKernelGGL(owgs_ovf_rehash_kernel, dim3((unsigned)((old_cap + 255) / 256)), dim3(256), 0, s, old_t,
                           old_cap, *O, err);
    return hipGetLastError();
}
#endif

#if OWGS_SHARED
extern "C" hipError_t owgs_launch_relpos(const OwgsRelposArgs* a, hipStream_t s) {
    if (a->n_rel > 0 && a->n_batches > 0)
        hipLaunchKernelGGL(owgs_relpos_kernel, dim3((unsigned)((a->n_rel + RP_T - 1) / RP_T)), dim3(RP_T), 0, s, *a);
    return hipGetLastError();
}
#endif

#if OWGS_SHARED
extern "C" hipError_t owgs_launch_relflags(const int64_t* rel_aid, int64_t n_rel, const int32_t* out_inv,
                                           uint8_t* rel_flags, hipStream_t s) {
    if (n_rel <= 0) return hipSuccess;
    hipLaunchKernelGGL(owgs_relflags_kernel, dim3((unsigned)((n_rel + 255) / 256)), dim3(256), 0, s, rel_aid, n_rel,
                       out_inv, rel_flags);
    return hipGetLastError();
}
#endif

#define REL_KEY_BITS 13  // entry keys 0..OWGS_CTC (4096 = no entry)

#if OWGS_SHARED
extern "C" size_t owgs_release_scratch_bytes(int32_t n) {
    size_t b = 0, c = 0;
    (void)hipcub::DeviceSelect::Flagged(nullptr, b, hipcub::CountingInputIterator<int32_t>(0), (const uint8_t*)nullptr,
                                        (int32_t*)nullptr, (int32_t*)nullptr, n);
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, c, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, n, 0, REL_KEY_BITS);
    return b > c ? b : c;
}
#endif

#if OWGS_SHARED
extern "C" hipError_t owgs_launch_release_seq(const OwgsReleaseArgs* a, hipStream_t s) {
    const OwgsReleaseArgs& R = *a;
    hipError_t e = hipMemsetAsync(R.bound, 0, (size_t)std::max(R.n_slots, 1) * 8, s);
    if (e == hipSuccess) e = hipMemsetAsync(R.risk, 0, 4, s);
    if (e == hipSuccess) e = hipMemsetAsync(R.sel_cnt, 0, 4, s);
    if (e != hipSuccess) return e;
    if (R.n > 0) {
        const unsigned gn = (unsigned)((R.n + 255) / 256), gs = (unsigned)((std::max(R.n_slots, 1) + 255) / 256);
        hipLaunchKernelGGL(owgs_rel_bound_kernel, dim3(gn), dim3(256), 0, s, R);
        hipLaunchKernelGGL(owgs_rel_check_kernel, dim3(gs), dim3(256), 0, s, R);
        hipLaunchKernelGGL(owgs_rel_apply_kernel, dim3(gn), dim3(256), 0, s, R);
        // concurrent releases by entry (nothing to do after an overflow-risk verdict: every key is OWGS_CTC)
        size_t tb = R.temp_bytes;
        e = hipcub::DeviceRadixSort::SortPairs(R.temp, tb, R.ckey, R.ckey_s, R.cval, R.cval_s, R.n, 0, REL_KEY_BITS, s);
        if (e == hipSuccess) e = hipMemsetAsync(R.cbeg, 0, OWGS_CTC * 4, s);
        if (e == hipSuccess) e = hipMemsetAsync(R.cend, 0, OWGS_CTC * 4, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(owgs_rel_cseg_kernel, dim3(gn), dim3(256), 0, s, R);
        hipLaunchKernelGGL(owgs_rel_capply_kernel, dim3(gn), dim3(256), 0, s, R);
        hipLaunchKernelGGL(owgs_rel_cupdate_kernel, dim3(OWGS_CTC / 256), dim3(256), 0, s, R);
        tb = R.temp_bytes;
        e = hipcub::DeviceSelect::Flagged(R.temp, tb, hipcub::CountingInputIterator<int32_t>(0), R.sel_flag, R.sel_idx,
                                          R.sel_cnt, R.n, s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(owgs_release_seq_kernel, dim3(1), dim3(64), 0, s, *a);
    return hipGetLastError();
}
#endif

// the engine's dynamic-LDS limit, set once per (kernel, device): the attribute is per device, and a process may drive
// contexts on several devices
static hipError_t lds_attr(const void* fn, int which) {
    static std::atomic<unsigned long long> done[9];
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const unsigned long long bit = 1ull << (dev & 63);
    if (done[which].load(std::memory_order_relaxed) & bit) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, OWGS_LDS_BYTES);
    if (e == hipSuccess) done[which].fetch_or(bit);
    return e;
}

// a launch prepared for this object's geometry (the host's tag, and a chunk width its lane fields hold)
static bool engine_args_ok(const OwgsEngineArgs& a) {
    return a.geom == OWGS_GEOM_TAG(OWGS_WL) && a.cw >= 0 && a.cw <= OWGS_WL;
}

// compiled specialisations: 0 (maxConcurrent == 1, identity pools, implicit sequence numbers), OWGS_F_CONC, and
// OWGS_F_ALL for anything else
static int feat_index(int feat) { return feat == 0 ? 0 : feat == OWGS_F_CONC ? 1 : 2; }
template <template <int> class K>
static void* pick(int fi) {
    return fi == 0 ? K<0>::fn() : fi == 1 ? K<OWGS_F_CONC>::fn() : K<OWGS_F_ALL>::fn();
}
template <int F>
struct KOne {
    static void* fn() { return (void*)owgs_engine_kernel<F>; }
};
template <int F>
struct KMulti {
    static void* fn() { return (void*)owgs_engine_multi_kernel<F>; }
};
template <int F>
struct KMultiDev {
    static void* fn() { return (void*)owgs_engine_multi_dev_kernel<F>; }
};

extern "C" hipError_t OWGS_GEOM(owgs_launch_engine_multi_dev)(const OwgsEngineArgs* a_host, const OwgsEngineArgs* a_dev, int k,
                                                   hipStream_t s) {
    if (k < 1 || k > OWGS_MULTI_DEV_MAX) return hipErrorInvalidValue;
    size_t lds = 0;
    int feat = 0;
    for (int i = 0; i < k; ++i) {
        if (!engine_args_ok(a_host[i])) return hipErrorInvalidValue;
        lds = std::max(lds, OWGS_GEOM(owgs_engine_lds_bytes)(a_host[i].n_slots, a_host[i].pool_mode, a_host[i].n_ids,
                                                  a_host[i].nm, a_host[i].nb, a_host[i].n_actions));
        feat |= a_host[i].feat;
    }
    if (lds > OWGS_LDS_BYTES) return hipErrorInvalidValue;
    const int fi = feat_index(feat);
    void* fn = pick<KMultiDev>(fi);
    const hipError_t ea = lds_attr(fn, fi);
    if (ea != hipSuccess) return ea;
    void* args[] = {(void*)&a_dev};
    return hipLaunchKernel(fn, dim3(k), dim3(OWGS_NT), args, lds, s);
}

extern "C" hipError_t OWGS_GEOM(owgs_launch_engine_multi)(const OwgsEngineArgs* a, int k, hipStream_t s) {
    if (k < 1 || k > OWGS_MULTI_MAX) return hipErrorInvalidValue;
    size_t lds = 0;
    int feat = 0;
    OwgsEngineMulti M;
    for (int i = 0; i < k; ++i) {
        if (!engine_args_ok(a[i])) return hipErrorInvalidValue;
        lds = std::max(lds, OWGS_GEOM(owgs_engine_lds_bytes)(a[i].n_slots, a[i].pool_mode, a[i].n_ids, a[i].nm, a[i].nb,
                                                  a[i].n_actions));
        feat |= a[i].feat;
        M.a[i] = a[i];
    }
    if (lds > OWGS_LDS_BYTES) return hipErrorInvalidValue;
    const int fi = feat_index(feat);
    void* fn = pick<KMulti>(fi);
    const hipError_t ea = lds_attr(fn, 3 + fi);
    if (ea != hipSuccess) return ea;
    void* args[] = {(void*)&M};
    return hipLaunchKernel(fn, dim3(k), dim3(OWGS_NT), args, lds, s);
}

extern "C" hipError_t OWGS_GEOM(owgs_launch_engine)(const OwgsEngineArgs* a, hipStream_t s) {
    if (!engine_args_ok(*a)) return hipErrorInvalidValue;
    const size_t lds = OWGS_GEOM(owgs_engine_lds_bytes)(a->n_slots, a->pool_mode, a->n_ids, a->nm, a->nb, a->n_actions);
    if (lds > OWGS_LDS_BYTES) return hipErrorInvalidValue;
    const int fi = feat_index(a->feat);
    void* fn = pick<KOne>(fi);
    const hipError_t ea = lds_attr(fn, 6 + fi);
    if (ea != hipSuccess) return ea;
    OwgsEngineOne M;
    M.a[0] = *a;
    void* args[] = {(void*)&M};
    return hipLaunchKernel(fn, dim3(1), dim3(OWGS_NT), args, lds, s);
}

#ifdef OWGS_VARIANT_NS
}  // namespace OWGS_VARIANT_NS
#endif
