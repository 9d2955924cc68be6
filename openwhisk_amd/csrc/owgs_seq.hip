// owgs_seq.hip -- the large-state engine: pools beyond the on-chip image (owgs_limits) and maxConcurrent beyond the
// 12-bit free-slot field of the on-chip concurrency map.
//
// The chunked engine (owgs_kernels.hip) and the resident engine (owgs_resident.hip) hold a controller shard's slot state
// in one CU's LDS: at most ~20k invoker ids, 15-bit ids and pool positions in the packed map key, maxConcurrent <=
// 4095.  A context whose state exceeds any of these (owgs_host.cpp: c->large) runs here instead: the ForcibleSemaphore
// permits stay in HBM (4 B per invoker id, any count), the NestedSemaphore maps are ONE open-addressing table in HBM
// keyed by the full (invoker id, fqn@version) pair with 32-bit fields {free slots, operationCount}, and walk positions
// are 32-bit.  It is the reference's sequential algorithm executed literally by one wave:
//
//   * releases in queue order (releaseInvoker SCPB:327-331 -> NestedSemaphore.releaseConcurrent NS:98-113 /
//     ForcibleSemaphore.release FS:117-120, overflow Error FS:48-50 -> flag, state as the reference leaves it);
//   * each publish: generateHash-derived home and step (SCPB:262-268, Int.MinValue -> the IndexOutOfBounds outcome),
//     then schedule (SCPB:398-436): 256 walk steps per round (4 per lane), the first usable step whose
//     tryAcquireConcurrent succeeds (NS:57-82) in walk order by ballot; every usable step the walk tried and failed
//     before it leaves an entry {0 free, 0 operations} in the map, as getOrElseUpdate does (NS:61-62) -- so empty
//     entries need no watch bookkeeping after updateCluster here; after n + 2 failed probes the counter RNG's healthy
//     invoker, forced (SCPB:417-424, forceAcquireConcurrent NS:84-91).
//
// The map grows without bound like the reference's TrieMap: the kernel stops before an operation that could take the
// table past half full, reports where, and the host grows the table and resumes there (owgs_host.cpp seq_run).
#include <hip/hip_runtime.h>

#include "owgs_internal.h"

typedef unsigned long long u64;

namespace {

__device__ __forceinline__ u64 splitmix64(u64 x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
// the bench's counter RNG replacing ThreadLocalRandom.nextInt(|H|) (SCPB:421), as every engine and the oracle
__device__ __forceinline__ uint32_t rng_index(u64 seed, u64 seq, uint32_t n) {
    const u64 u = splitmix64(seed ^ (seq * 0x9E3779B97F4A7C15ULL)) >> 32;
    return (uint32_t)((u * (u64)n) >> 32);
}
__device__ __forceinline__ int ffs64(u64 m) { return __ffsll((long long)m) - 1; }
__device__ __forceinline__ int wave_sum(int v) {  // (every lane gets the wave's sum)
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}
#ifndef SEQ_SPEC
#define SEQ_SPEC 64  // walk steps a speculated maxConcurrent == 1 decision probes (beyond them: decided alone)
#endif
#define SEQ_SPG 8    // ... in rounds of this many loads in flight
#ifndef SEQ_SPEC_C
#define SEQ_SPEC_C 16  // walk steps a speculated concurrent decision probes (4 per round)
#endif
// Java int arithmetic (wrap-around)
__device__ __forceinline__ int jadd(int a, int b) { return (int)((uint32_t)a + (uint32_t)b); }
__device__ __forceinline__ int jsub(int a, int b) { return (int)((uint32_t)a - (uint32_t)b); }

__device__ __forceinline__ uint32_t sq_hash(uint32_t inv, uint32_t slot) {
    uint32_t k = (inv * 0x9E3779B1u) ^ (slot * 0x85EBCA77u);
    k ^= k >> 16;
    k *= 0x7feb352dU;
    k ^= k >> 15;
    k *= 0x846ca68bU;
    k ^= k >> 16;
    return k;
}
// The mutable state (permits, the map) is read past the CU's L1 (agent-scope relaxed loads: `sc1`, L2): the map's
// key words are claimed by atomics, which L2 performs, so an L1 copy of such a line could be stale.  Stores are
// write-through; `mem_done` waits for them (vmcnt covers stores) before a later load of the wave may need them -- this
// replaces an agent-scope fence per decision, which also wrote back and invalidated the caches (~3.5 us each).
__device__ __forceinline__ int ld_i(const int32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ uint32_t ld_u(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint4 ld_e(const uint4* p) {
    const uint32_t* q = (const uint32_t*)p;
    return make_uint4(ld_u(q), ld_u(q + 1), ld_u(q + 2), ld_u(q + 3));
}
__device__ __forceinline__ void mem_done() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// the map: entry {invoker + 1 (0 empty, ~0 deleted), slot, free slots c, operationCount}; index of (inv, slot) or -1
__device__ __forceinline__ int sq_find(const OwgsSeqArgs& S, int inv, int slot, uint4* e) {
    const uint32_t m = (uint32_t)S.map_cap - 1u;
    uint32_t h = sq_hash((uint32_t)inv, (uint32_t)slot) & m;
    for (int p = 0; p < S.map_cap; ++p) {
        const uint4 v = ld_e(&S.map[h]);
        if (v.x == 0u) return -1;
        if (v.x == (uint32_t)inv + 1u && v.y == (uint32_t)slot) {
            *e = v;
            return (int)h;
        }
        h = (h + 1u) & m;
    }
    return -1;
}
// four lookups of one lane at once (the walk's four steps of a round): each probe round issues the loads of every
// chain still open together, so the round trips overlap instead of adding up
__device__ __forceinline__ void sq_find4(const OwgsSeqArgs& S, const int* inv, int slot, const bool* go, int* ix,
                                         uint4* e) {
    const uint32_t m = (uint32_t)S.map_cap - 1u;
    uint32_t h[4];
    bool open[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        h[u] = sq_hash((uint32_t)inv[u], (uint32_t)slot) & m;
        open[u] = go[u];
        ix[u] = -1;
        e[u] = make_uint4(0u, 0u, 0u, 0u);
    }
    for (int p = 0; p < S.map_cap && (open[0] || open[1] || open[2] || open[3]); ++p) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = open[u] ? ld_e(&S.map[h[u]]) : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (!open[u]) continue;
            if (v[u].x == 0u) {
                open[u] = false;  // absent
            } else if (v[u].x == (uint32_t)inv[u] + 1u && v[u].y == (uint32_t)slot) {
                ix[u] = (int)h[u];
                e[u] = v[u];
                open[u] = false;
            } else {
                h[u] = (h[u] + 1u) & m;
            }
        }
    }
}
// insert (inv, slot) known to be absent (distinct keys may race: the key word is claimed by CAS)
__device__ __forceinline__ int sq_insert(const OwgsSeqArgs& S, int inv, int slot, int c, int ops) {
    const uint32_t m = (uint32_t)S.map_cap - 1u;
    uint32_t h = sq_hash((uint32_t)inv, (uint32_t)slot) & m;
    for (int p = 0; p < S.map_cap;) {
        const uint32_t k = ld_u(&S.map[h].x);
        if (k == 0u || k == 0xFFFFFFFFu) {
            if (atomicCAS(&S.map[h].x, k, (uint32_t)inv + 1u) == k) {
                S.map[h].y = (uint32_t)slot;
                S.map[h].z = (uint32_t)c;
                S.map[h].w = (uint32_t)ops;
                if (k == 0u) atomicAdd(S.map_filled, 1);
                return (int)h;
            }
            continue;
        }
        h = (h + 1u) & m;
        ++p;
    }
    return -1;
}

}  // namespace

// One wave.  Runs r = S.run0 .. n_runs - 1: the releases [rel_off[r], rel_off[r+1]) in order, then the publishes
// [pub_off[r], pub_off[r+1]) in order; S.resume (if set) = {run, phase, index} to continue from, written back when the
// map needs to grow first (state[0] = 1) or the call completed (state[0] = 0).
__global__ __launch_bounds__(64) void owgs_seq_kernel(OwgsSeqArgs S) {
    __shared__ uint32_t pc[OWGS_SEQ_MAX_WORDS + 1];  // usable ids before each bitmap word
    __shared__ int32_t tgt_lo[512], tgt_hi[512];  // per group and hashed target: the speculating actions' range
    const int lane = threadIdx.x;
    const int words = (S.n_ids + 31) >> 5;
    {
        int carry = 0;
        for (int w0 = 0; w0 <= words; w0 += 64) {
            const int w = w0 + lane;
            const int c = w < words ? __popc(S.usable[w]) : 0;
            int inc = c;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int o = __shfl_up(inc, d, 64);
                inc += lane >= d ? o : 0;
            }
            if (w <= words) pc[w] = (uint32_t)(carry + inc - c);
            carry += __shfl(inc, 63, 64);
        }
    }
    __syncthreads();
    auto usable_before = [&](int x) -> int {
        if (x <= 0) return 0;
        const int w = x >> 5, b = x & 31;
        return (int)pc[w] + (b ? __popc(S.usable[w] & ((1u << b) - 1u)) : 0);
    };
    auto select_usable = [&](int lo, int k) -> int {  // k-th usable id at or after id lo
        const int target = usable_before(lo) + k;
        int a = lo >> 5, z = words - 1;
        while (a < z) {
            const int mid = (a + z + 1) >> 1;
            if ((int)pc[mid] <= target) a = mid;
            else z = mid - 1;
        }
        uint32_t m = S.usable[a];
        int need = target - (int)pc[a];
        if (need < 0 || need >= __popc(m)) return -1;
        for (; need > 0; --need) m &= m - 1u;
        return (a << 5) + __ffs(m) - 1;
    };
    const int hm = usable_before(S.nm), hb = usable_before(S.n_ids) - usable_before(S.n_ids - S.nb);
    int err = 0;
    // an upper bound of the map's non-empty entries (live + deleted) for the growth check: the count at launch plus
    // every insert of this launch (an insert that reuses a deleted entry counts too)
    long long filled = ld_i(S.map_filled);
    // walk cursors of maxConcurrent == 1 actions: valid for one generation; generations count this call's release
    // runs (only releases raise permits; nothing else changes the state inside a call)
    uint32_t gen = S.gen0;
    const float rn_m = S.nm > 0 ? 1.0f / (float)S.nm : 0.f, rn_b = S.nb > 0 ? 1.0f / (float)S.nb : 0.f;
    int r = S.resume ? S.state[1] : 0, ph = S.resume ? S.state[2] : 0;
    long long j = S.resume ? ((long long)(uint32_t)S.state[3] | ((long long)S.state[4] << 32)) : -1;
    bool stop = false;
    int n_spec = 0, n_alone = 0;  // decisions kept from the speculation / decided alone (state[6], state[7])
    // cycles (s_memtime) by phase, state[8..15] as 4 x u64: releases, a group's gather + ranks + speculation, its
    // decisions kept from the speculation, its decisions decided alone
    u64 cy0 = 0, cy1 = 0, cy2 = 0, cy3 = 0;
    u64 t_ph = clock64();
    auto tick = [&](int k) {  // (no indexed array: that would live in scratch and wait for the stores in flight)
        const u64 t = clock64(), d = t - t_ph;
        cy0 += k == 0 ? d : 0;
        cy1 += k == 1 ? d : 0;
        cy2 += k == 2 ? d : 0;
        cy3 += k == 3 ? d : 0;
        t_ph = t;
    };
    for (; r < S.n_runs && !stop; ++r, ph = 0, j = -1) {
        // ---------------------------------------------------------------- completions (lane 0, queue order)
        if (ph == 0) {
            const long long re = S.rel_off[r + 1];
            if (j < 0) j = S.rel_off[r];
            if (re > j) ++gen;
            // in groups of 64: lane q gathers release j0 + q's invoker and action fields, lane 0 applies them in order
            while (j < re) {
                const long long j0 = j;
                const int nq = (int)min(64ll, re - j0);
                int g_inv = -1, g_a = 0, g_mem = 0, g_maxc = 0, g_slot = 0;
                if (lane < nq) {
                    if (S.rel_aid) {
                        const long long aid = S.rel_aid[j0 + lane];
                        g_inv = ld_i(&S.dec_inv[aid]);  // (decided by this launch too: past L1)
                        g_a = S.dec_act[aid];
                    } else {
                        g_inv = S.rel_inv[j0 + lane];
                        if (!S.rel_mem) g_a = S.rel_act[j0 + lane];
                    }
                }
                if (lane < nq && g_inv >= 0 && g_inv < S.n_slots) {
                    if (S.rel_mem) {  // the completion path's release records (owgs_acks.hip)
                        g_mem = S.rel_mem[j0 + lane];
                        g_maxc = S.rel_maxc[j0 + lane];
                        g_slot = S.rel_slot[j0 + lane];
                    } else {
                        g_mem = S.act_mem[g_a];
                        g_maxc = S.act_maxc[g_a];
                        g_slot = S.act_slot[g_a];
                    }
                }
                // maxConcurrent == 1 releases are permit adds (FS:117-120) and commute with every other release unless
                // a permit count could leave the int range (the overflow Error, FS:48-50, depends on the order): when
                // no invoker of the group can, whatever the order (its permits plus all the memory the group returns at
                // most stay below 2^31), they are applied at once, each lane its own, and lane 0 then applies only the
                // concurrent ones in queue order
                const bool g_in = lane < nq && g_inv >= 0 && g_inv < S.n_slots;
                const int g_p = g_in ? ld_i(&S.permits[g_inv]) : 0;
                const long long g_room = (long long)wave_sum(g_in ? g_mem : 0);
                const bool par = __ballot(g_in && (long long)g_p + g_room > 0x7FFFFFFFll) == 0ull;
                const bool g_plain = par && g_in && g_maxc <= 1;
                if (g_plain) atomicAdd(&S.permits[g_inv], g_mem);
                if (__ballot(g_plain)) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                int my_f = 0;
                for (int q = 0; q < nq; ++q) {
                    const int inv = __builtin_amdgcn_readlane(g_inv, q);
                    const bool done_q = __builtin_amdgcn_readlane((int)g_plain, q) != 0;
                    int f = 0;
                    if (!done_q && inv >= 0 && inv < S.n_slots && lane == 0) {  // invokerSlots.lift (SCPB:329)
                        const int mem = __builtin_amdgcn_readlane(g_mem, q), maxc = __builtin_amdgcn_readlane(g_maxc, q);
                        if (maxc <= 1) {
                            const int p = ld_i(&S.permits[inv]), nx = jadd(p, mem);
                            if (nx < p) f = OWGS_REL_OVERFLOW_BIT;  // FS:48-50
                            else S.permits[inv] = nx;
                        } else {
                            uint4 e;
                            const int ix = sq_find(S, inv, __builtin_amdgcn_readlane(g_slot, q), &e);
                            if (ix < 0) {
                                f = OWGS_REL_NOSUCH_BIT;  // NoSuchElementException (NS:103)
                            } else {  // RS.release(1, true) (RS:99-108, 42-56)
                                const int ops = jsub((int)e.w, 1);
                                const bool arel = ops == 0;
                                const int n2 = jadd((int)e.z, 1);
                                const bool mrel = n2 % maxc == 0;
                                const int c1 = mrel ? jsub(n2, maxc) : n2;
                                bool removed = arel;
                                if (mrel) {
                                    const int p = ld_i(&S.permits[inv]), nx = jadd(p, mem);
                                    if (nx < p) {
                                        f = OWGS_REL_OVERFLOW_BIT;  // the Error after the RS update: no removal
                                        removed = false;
                                    } else {
                                        S.permits[inv] = nx;
                                    }
                                }
                                if (removed) S.map[ix].x = 0xFFFFFFFFu;  // NS:109-111
                                else {
                                    S.map[ix].z = (uint32_t)c1;
                                    S.map[ix].w = (uint32_t)ops;
                                }
                            }
                        }
                    }
                    f = __builtin_amdgcn_readlane(f, 0) | (inv < 0 ? OWGS_REL_NOENTRY_BIT : 0);  // (CLB:278-279)
                    if (lane == q) my_f = f;
                    // (lane 0 alone reads and writes the state here: its own accesses stay in program order)
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                }
                if (S.rel_flags && lane < nq) S.rel_flags[j0 + lane] = (uint8_t)my_f;
                j = j0 + nq;
            }
            mem_done();  // (the publishes' walks read these permits and entries from every lane)
            tick(0);
            ph = 1;
            j = -1;
        }
        // ---------------------------------------------------------------- publishes (one decision at a time)
        // in groups of 64: lane q gathers decision j0 + q's action fields up front (one round trip per group, not
        // two per decision) and keeps its outputs until the group ends
        const long long pe = S.pub_off[r + 1];
        if (j < 0) j = S.pub_off[r];
        while (j < pe && !stop) {
            const long long j0 = j;
            const int nq = (int)min(64ll, pe - j0);
            int g_a = 0, g_mem = 0, g_maxc = 0, g_slot = 0, g_hash = 0, g_bb = 0;
            u64 g_seq = 0;
            if (lane < nq) {
                g_a = S.pub_act[j0 + lane];
                g_seq = S.seq ? S.seq[j0 + lane] : S.seq_base + (u64)(j0 + lane);
            }
            if (lane < nq) {
                g_mem = S.act_mem[g_a];
                g_maxc = S.act_maxc[g_a];
                g_slot = S.act_slot[g_a];
                g_hash = S.act_hash[g_a];
                g_bb = S.act_bb[g_a];
            }
            // home and step size of each decision of the group, one lane each (SCPB:262-268): 0 walk, 1 empty pool,
            // 2 the Int.MinValue hash's IndexOutOfBounds
            int g_kind = 1;
            uint32_t g_home = 0u, g_step = 0u;
            if (lane < nq) {
                const int gn = g_bb ? S.nb : S.nm, gk = g_bb ? S.n_bsteps : S.n_msteps;
                if (gn > 0) {
                    if (g_hash % gn < 0 || g_hash % gk < 0) {
                        g_kind = 2;
                    } else {
                        g_kind = 0;
                        g_home = (uint32_t)(g_hash % gn);
                        g_step = (uint32_t)((g_bb ? S.bsteps : S.msteps)[g_hash % gk] % gn);
                    }
                }
            }
            // each decision's walk start: its action's cursor of this generation (maxConcurrent == 1 only; steps
            // before it had no room for the action's memory, and permits only fall inside a run)
            int g_cs = 0;
            uint32_t g_cp = g_home;  // (the cursor step's pool position)
            if (lane < nq && S.cur && g_kind == 0 && g_maxc <= 1 && g_a >= 0 && g_a < S.n_actions) {
                const uint4 cu = S.cur[g_a];
                if (cu.x == gen) {
                    g_cs = (int)cu.y;
                    g_cp = cu.z;
                }
            }
            // ---- speculation (maxConcurrent == 1 decisions, one lane each, all at once): each walks its own walk from
            // its action's cursor against the permits at the group's start, rank-packed -- the k-th decision of an
            // action in the group (k = its earlier ones) takes the step where the walk's cumulative capacity
            // floor(permits / mem) first exceeds k -- up to SEQ_SPEC steps, SEQ_SPG loads in flight per round.  Permits only
            // fall inside a run, so a step the walk passed stays full; the in-order loop below keeps the speculation
            // where the permits at the decision's turn still hold it (its target's permits at the group's start minus
            // what the group's earlier decisions took there) and decides the rest alone.
            const bool plain = lane < nq && g_kind == 0 && g_maxc <= 1 && g_mem > 0;
            int rank = 0;
            {
                u64 rem = __ballot(plain);
                while (rem) {
                    const int a0 = __builtin_amdgcn_readlane(g_a, ffs64(rem));
                    const u64 m = __ballot(plain && g_a == a0);
                    if (plain && g_a == a0)
                        rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    rem &= ~m;
                }
            }
            int sp_k = 0;  // 0 none (not a plain walk, or unfinished within the budget), 1 target, 2 the walk fails
            int sp_t = -1, sp_pv = 0, sp_s = 0, sp_ks = 0;  // (sp_ks: earlier decisions of its action at its target)
            uint32_t sp_p = 0u;
            if (plain) {
                const int n = g_bb ? S.nb : S.nm, base = g_bb ? S.n_ids - S.nb : 0;
                const uint32_t un = (uint32_t)n;
                const float rm = 1.0f / (float)g_mem;
                int sx = g_cs, cum = 0;
                uint32_t pos = g_cp;
                for (int r4 = 0; r4 < SEQ_SPEC / SEQ_SPG && sp_k == 0; ++r4) {
                    int id[SEQ_SPG], pv[SEQ_SPG];
                    uint32_t uw[SEQ_SPG], ps[SEQ_SPG];
#pragma unroll
                    for (int u = 0; u < SEQ_SPG; ++u) {
                        ps[u] = pos;
                        id[u] = base + (int)pos;
                        uw[u] = S.usable[id[u] >> 5];
                        pv[u] = id[u] < S.n_slots ? ld_i(&S.permits[id[u]]) : 0;
                        pos += g_step;
                        pos = pos >= un ? pos - un : pos;
                    }
#pragma unroll
                    for (int u = 0; u < SEQ_SPG; ++u) {
                        if (sp_k != 0) continue;
                        if (sx + u >= n) {  // every pool position: at most `rank` units anywhere (SCPB:417)
                            sp_k = 2;
                            continue;
                        }
                        const bool us = ((uw[u] >> (id[u] & 31)) & 1u) && id[u] < S.n_slots;
                        int cap = 0;
                        if (us && pv[u] >= g_mem) {  // floor(pv / mem) (float estimate, one correction), clamped
                            cap = (int)((float)pv[u] * rm);
                            const long long rr = (long long)pv[u] - (long long)cap * g_mem;
                            cap += rr >= g_mem ? 1 : 0;
                            cap -= rr < 0 ? 1 : 0;
                            cap = min(cap, 64);
                        }
                        if (cum + cap > rank) {
                            sp_k = 1;
                            sp_t = id[u];
                            sp_pv = pv[u];
                            sp_s = sx + u;
                            sp_p = ps[u];
                            sp_ks = rank - cum;
                        } else {
                            cum += cap;
                        }
                    }
                    sx += SEQ_SPG;
                }
            }
            // concurrent decisions (the key's entries change only through its own decisions): the k-th decision of an
            // fqn@version key in the group (k = crank) walks from its home at the group's start, rank-packed -- a step
            // holds c free slots plus maxConcurrent per container its permits hold (tryAcquireConcurrent, NS:57-82),
            // and the decision lands where the cumulative count first exceeds k.  The zero-capacity steps it tried whose
            // entry is absent get the empty entry getOrElseUpdate leaves (NS:61-62) when it commits (sp_mask, bit =
            // walk step; only those past the previous decision of its key's target: that one made the earlier ones).
            // A key speculates past its first decision only when one action holds all its decisions in the group (one
            // walk); otherwise the later ones are decided alone.
            const bool conc = lane < nq && g_kind == 0 && g_maxc > 1 && g_mem > 0;
            int crank = 64;      // rank among the group's decisions of its key (64: not speculated)
            bool ksolo = false;  // the key's only decision in the group
            {
                u64 rem = __ballot(conc);
                while (rem) {
                    const int j = ffs64(rem);
                    const int s0 = __builtin_amdgcn_readlane(g_slot, j), a0 = __builtin_amdgcn_readlane(g_a, j);
                    const u64 m = __ballot(conc && g_slot == s0);
                    const bool oneact = __ballot(conc && g_slot == s0 && g_a != a0) == 0;
                    if (conc && g_slot == s0) {
                        const int k = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                        crank = (k == 0 || oneact) ? k : 64;
                        ksolo = __popcll(m) == 1;
                    }
                    rem &= ~m;
                }
            }
            int sp_ix = -1;
            uint32_t sp_mask = 0u, sp_ez = 0u, sp_ew = 0u;
            if (crank < 64 && (g_bb ? S.nb : S.nm) > SEQ_SPEC_C) {
                const int n = g_bb ? S.nb : S.nm, base = g_bb ? S.n_ids - S.nb : 0;
                const uint32_t un = (uint32_t)n;
                const float rm = 1.0f / (float)g_mem;
                int cum = 0;
                uint32_t pos = g_home;
                for (int sx = 0; sx < SEQ_SPEC_C && sp_k == 0; sx += 4) {
                    int id[4], pv[4], ixs[4];
                    bool tried[4];
                    uint32_t uw[4], ps[4];
                    uint4 es[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        ps[u] = pos;
                        id[u] = base + (int)pos;
                        uw[u] = S.usable[id[u] >> 5];
                        pv[u] = id[u] < S.n_slots ? ld_i(&S.permits[id[u]]) : 0;
                        pos += g_step;
                        pos = pos >= un ? pos - un : pos;
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) tried[u] = ((uw[u] >> (id[u] & 31)) & 1u) && id[u] < S.n_slots;
                    sq_find4(S, id, g_slot, tried, ixs, es);
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        if (sp_k != 0 || !tried[u]) continue;
                        int cap = ixs[u] >= 0 ? min((int)es[u].z, 64) : 0;  // free slots, then containers
                        if (pv[u] >= g_mem) {
                            int nc = (int)((float)pv[u] * rm);
                            const long long rr = (long long)pv[u] - (long long)nc * g_mem;
                            nc += rr >= g_mem ? 1 : 0;
                            nc -= rr < 0 ? 1 : 0;
                            cap += min(nc, 64) * min(g_maxc, 64);
                        }
                        if (cum + cap > crank) {
                            sp_k = 3;
                            sp_t = id[u];
                            sp_pv = pv[u];
                            sp_s = sx + u;
                            sp_p = ps[u];
                            sp_ix = ixs[u];
                            sp_ez = ixs[u] >= 0 ? es[u].z : 0u;
                            sp_ew = ixs[u] >= 0 ? es[u].w : 0u;
                        } else {
                            if (cap == 0 && ixs[u] < 0) sp_mask |= 1u << (sx + u);
                            cum += cap;
                        }
                    }
                }
            }
            tick(1);
            // the state stores of decisions kept from the speculation are held in their lanes and written together
            // (the group's last decision per invoker / per action wins), before anything reads the state from memory:
            // a store per decision makes the next reuse of its data register wait for the store (vmcnt) on this target
            bool pw_on = false, cw_on = false;
            int pw_t = 0, pw_v = 0, cw_a = 0, cw_s = 0;
            uint32_t cw_p = 0u;
            auto flush = [&]() {
                for (u64 rem = __ballot(pw_on); rem;) {
                    const int tt = __builtin_amdgcn_readlane(pw_t, ffs64(rem));
                    const u64 m = __ballot(pw_on && pw_t == tt);
                    if (lane == 63 - __clzll((long long)m)) S.permits[tt] = pw_v;
                    rem &= ~m;
                }
                for (u64 rem = __ballot(cw_on); rem;) {
                    const int aa = __builtin_amdgcn_readlane(cw_a, ffs64(rem));
                    const u64 m = __ballot(cw_on && cw_a == aa);
                    if (lane == 63 - __clzll((long long)m)) S.cur[aa] = make_uint4(gen, (uint32_t)cw_s, cw_p, 0u);
                    rem &= ~m;
                }
                pw_on = false;
                cw_on = false;
            };
            // each key's speculated decisions in order: the previous one's target step (its empty entries end there); a
            // decision whose earlier one of the key did not speculate is decided alone too
            int sp_prev = -1;
            {
                u64 rem = __ballot(conc && crank < 64);
                while (rem) {
                    const int j = ffs64(rem);
                    const int s0 = __builtin_amdgcn_readlane(g_slot, j);
                    u64 m = __ballot(conc && crank < 64 && g_slot == s0);
                    rem &= ~m;
                    int prev = -1;
                    bool ok = true;
                    while (m) {
                        const int i = ffs64(m);
                        m &= m - 1;
                        if (!ok && lane == i) sp_k = 0;
                        if (lane == i) sp_prev = prev;
                        ok = ok && __builtin_amdgcn_readlane(sp_k, i) == 3;
                        prev = __builtin_amdgcn_readlane(sp_s, i);
                    }
                }
            }
            // speculated targets no decision of ANOTHER action speculated in the group (a hash collision counts as
            // another's): there the decisions before one of the action's own at the target are exactly its ks earlier
            // ones (rank packing), each taking its memory
            const bool spx = sp_k == 1 || sp_k == 3;
            const int th = (int)(((uint32_t)sp_t * 2654435761u) >> 23);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                tgt_lo[lane + 64 * u] = 0x7FFFFFFF;
                tgt_hi[lane + 64 * u] = (int)0x80000000;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            if (spx) {
                atomicMin(&tgt_lo[th], g_a);
                atomicMax(&tgt_hi[th], g_a);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            const bool uniq = spx && tgt_lo[th] == g_a && tgt_hi[th] == g_a;
            // this lane's speculated concurrent decision (sp_k 3), committed with `left` permits at its target: the
            // empty entries of the steps it tried and failed, then its own entry (a free slot, or a container whose
            // memory the pending permit write takes); returns the entries it inserted
            auto conc_commit = [&](int left) -> int {
                const int n_ = g_bb ? S.nb : S.nm, base_ = g_bb ? S.n_ids - S.nb : 0;
                int ins = 0;
                uint32_t pp = g_home;
                for (int sx = 0; sx < sp_s; ++sx) {
                    if (sx > sp_prev && ((sp_mask >> sx) & 1u)) {
                        ++ins;
                        if (sq_insert(S, base_ + (int)pp, g_slot, 0, 0) < 0) err = 1;
                    }
                    pp += g_step;
                    pp = pp >= (uint32_t)n_ ? pp - (uint32_t)n_ : pp;
                }
                int ix = sp_ix, c = (int)sp_ez, ops = (int)sp_ew;
                if (ix < 0) {  // getOrElseUpdate (NS:61-62)
                    ++ins;
                    ix = sq_insert(S, sp_t, g_slot, 0, 0);
                    c = 0;
                    ops = 0;
                    if (ix < 0) err = 1;
                }
                if (c - 1 >= 0) {  // RS.tryAcquire(1) (RS:62-70)
                    c = c - 1;
                    ops = jadd(ops, 1);
                } else {  // the memory: RS.release(maxConcurrent - 1, false) (written by flush)
                    pw_on = true;
                    pw_t = sp_t;
                    pw_v = left - g_mem;
                    ops = jadd(ops, 1);
                    const int n2 = jadd(c, g_maxc - 1);
                    c = n2 % g_maxc == 0 ? jsub(n2, g_maxc) : n2;
                }
                if (ix >= 0) {
                    S.map[ix].z = (uint32_t)c;
                    S.map[ix].w = (uint32_t)ops;
                }
                sp_ix = ix;  // (the entry as it leaves it: its key's later decisions at this invoker continue from it)
                sp_ez = (uint32_t)c;
                sp_ew = (uint32_t)ops;
                return ins;
            };
            int acc = 0;  // memory the group's earlier decisions took at this lane's speculated target (sp_k 1 or 3)
            bool inval = false;  // an earlier decision of its action was decided alone: its rank no longer holds
            int my_out = OWGS_NONE_V, my_fl = 0;
            int q = 0;
            for (; q < nq; ++q) {
                {  // a run of decisions kept at once: speculated targets no other decision of the group speculated,
                   // whose permits (less what the decisions decided one at a time so far took there) still hold them
                    const bool inq = lane >= q && lane < nq && uniq;
                    const bool fp = inq && sp_k == 1 && !inval && sp_pv - acc - sp_ks * g_mem >= g_mem;
                    const bool fc = inq && sp_k == 3 && ksolo && !inval && ((int)sp_ez >= 1 || sp_pv - acc >= g_mem);
                    u64 nf = ~__ballot(fp || fc) & (~0ull << q);
                    int L = min(nf ? ffs64(nf) : 64, nq);
                    // (the map must not pass half full: each concurrent decision inserts at most SEQ_SPEC_C + 1)
                    const u64 run = L >= 64 ? ~0ull << q : ((1ull << L) - 1) & (~0ull << q);
                    if (2 * (filled + (long long)(SEQ_SPEC_C + 1) * __popcll(__ballot(fc) & run)) > (long long)S.map_cap) {
                        nf = ~__ballot(fp) & (~0ull << q);
                        L = min(nf ? ffs64(nf) : 64, L);
                    }
                    const bool fast = (fp || fc) && lane < L;
                    if (L > q) {
                        int ins = 0;
                        if (fast && fc) {
                            ins = conc_commit(sp_pv - acc);
                            my_out = sp_t;
                            my_fl = 0;
                        }
                        filled += __builtin_amdgcn_readlane(wave_sum(ins), 0);
                        if (fast && fp) {  // (the cursors of decided-alone decisions after the run stay lower
                                           // bounds: they are not moved past the run's steps)
                            my_out = sp_t;
                            my_fl = 0;
                            pw_on = true;
                            pw_t = sp_t;
                            pw_v = sp_pv - acc - (sp_ks + 1) * g_mem;
                            if (S.cur && g_a >= 0 && g_a < S.n_actions) {
                                cw_on = true;
                                cw_a = g_a;
                                cw_s = sp_s;
                                cw_p = sp_p;
                            }
                        }
                        n_spec += L - q;
                        q = L;
                        tick(2);
                        if (q >= nq) break;
                    }
                }
                const int mem = __builtin_amdgcn_readlane(g_mem, q), maxc = __builtin_amdgcn_readlane(g_maxc, q);
                const int slot = __builtin_amdgcn_readlane(g_slot, q), kind = __builtin_amdgcn_readlane(g_kind, q);
                const int pool = __builtin_amdgcn_readlane(g_bb, q) ? 1 : 0;
                const u64 seq = ((u64)(uint32_t)__builtin_amdgcn_readlane((int)(g_seq >> 32), q) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)g_seq, q);
                const int n = pool ? S.nb : S.nm, base = pool ? S.n_ids - S.nb : 0;
                int out = OWGS_NONE_V, fl = 0;
                // a walk can leave up to n entries (every usable step it passes): grow the map first if that could
                // cross half of it (the host resumes here)
                if (maxc > 1 && 2 * (filled + n + 2) > (long long)S.map_cap) {
                    stop = true;
                    break;
                }
                const int qk = __builtin_amdgcn_readlane(sp_k, q);
                const bool qinv = __builtin_amdgcn_readlane((int)inval, q) != 0;
                bool spec_done = false;
                int taken_at = -1, taken = 0;  // the permits this decision took: invoker, memory
                bool kept_plain = false;  // (its action's later decisions at its target count it through their ks)
                if (kind == 0 && qk == 1 && !qinv) {  // a speculated target: held iff the permits there still hold it
                    const int t = __builtin_amdgcn_readlane(sp_t, q);
                    const bool qu = __builtin_amdgcn_readlane((int)uniq, q) != 0;
                    const int left = __builtin_amdgcn_readlane(sp_pv, q) - __builtin_amdgcn_readlane(acc, q) -
                                     (qu ? __builtin_amdgcn_readlane(sp_ks, q) * mem : 0);
                    if (left >= mem) {  // tryAcquire succeeds at its turn (FS:63-71); every step before was full
                        out = t;
                        if (lane == q) {  // (written by flush)
                            pw_on = true;
                            pw_t = t;
                            pw_v = left - mem;
                        }
                        taken_at = t;
                        taken = mem;
                        spec_done = true;
                        kept_plain = qu;
                        if (S.cur) {
                            const int aq = __builtin_amdgcn_readlane(g_a, q);
                            const int tsq = __builtin_amdgcn_readlane(sp_s, q);
                            const uint32_t tpq = (uint32_t)__builtin_amdgcn_readlane((int)sp_p, q);
                            if (lane > q && g_a == aq) {
                                g_cs = tsq;
                                g_cp = tpq;
                            }
                            if (lane == q && aq >= 0 && aq < S.n_actions) {
                                cw_on = true;
                                cw_a = aq;
                                cw_s = tsq;
                                cw_p = tpq;
                            }
                        }
                    }
                } else if (kind == 0 && qk == 3 && !qinv) {  // a speculated concurrent decision
                    const int t = __builtin_amdgcn_readlane(sp_t, q);
                    const int left = __builtin_amdgcn_readlane(sp_pv, q) - __builtin_amdgcn_readlane(acc, q);
                    const int c0 = (int)(uint32_t)__builtin_amdgcn_readlane((int)sp_ez, q);
                    if (c0 >= 1 || left >= mem) {  // a free slot of its entry as it is now, or a container's memory
                        int ins = 0;
                        if (lane == q) ins = conc_commit(left);
                        filled += __builtin_amdgcn_readlane(ins, q);
                        {  // its key's later decisions at this invoker see the entry it left
                            const int nix = __builtin_amdgcn_readlane(sp_ix, q);
                            const uint32_t nz = (uint32_t)__builtin_amdgcn_readlane((int)sp_ez, q);
                            const uint32_t nw = (uint32_t)__builtin_amdgcn_readlane((int)sp_ew, q);
                            if (lane > q && sp_k == 3 && g_slot == slot && sp_t == t) {
                                sp_ix = nix;
                                sp_ez = nz;
                                sp_ew = nw;
                            }
                        }
                        out = t;
                        taken_at = t;
                        taken = c0 >= 1 ? 0 : mem;
                        spec_done = true;
                    }
                } else if (kind == 0 && qk == 2 && !qinv) {  // the walk fails everywhere: forced (SCPB:417-424)
                    const int H = pool ? hb : hm;
                    spec_done = true;
                    if (H > 0) {
                        const int t = select_usable(base, (int)rng_index(S.rng_seed, seq, (uint32_t)H));
                        if (t < 0) err = 1;
                        else {
                            flush();
                            mem_done();  // (this group's earlier stores of its permits)
                            if (lane == 0) S.permits[t] = jsub(ld_i(&S.permits[t]), mem);  // forceAcquire (FS:107-110)
                            taken_at = t;
                            taken = mem;
                        }
                        out = t >= 0 ? t : OWGS_NONE_V;
                        fl = 1;
                    }
                    if (S.cur) {  // the cursor past the walk, as a walk that failed leaves it
                        const int aq = __builtin_amdgcn_readlane(g_a, q);
                        if (lane > q && g_a == aq) {
                            g_cs = n + 2;
                            g_cp = 0u;
                        }
                        if (lane == 0 && aq >= 0 && aq < S.n_actions) S.cur[aq] = make_uint4(gen, (uint32_t)(n + 2), 0u, 0u);
                    }
                }
                if (spec_done) {
                    ++n_spec;
                } else if (kind == 1) {
                    out = OWGS_NONE_V;  // no invokers in the pool: None (SCPB:288-290)
                } else if (kind == 2) {
                    out = OWGS_THROW_V;  // Int.MinValue hash: stepSizes / invokers index out of bounds (SCPB:266-268)
                } else {
                    flush();
                    mem_done();  // (the stores of this group's speculated decisions, before this walk reads the state)
                    ++n_alone;
                    const uint32_t step = (uint32_t)__builtin_amdgcn_readlane((int)g_step, q);
                    int t = -1;
                    // probes s = s0 + 64 u + lane, u = 0..3, in walk order (u, then lane); position (home + s step) mod
                    // n: lane l starts at home + l step (a wave scan of step mod n), then advances 64 steps at a time
                    const uint32_t un = (uint32_t)n;
                    auto madd = [&](uint32_t x, uint32_t y) -> uint32_t {
                        const uint32_t z = x + y;  // (both < n < 2^31: no wrap)
                        return z >= un ? z - un : z;
                    };
                    // (k step) mod n for k <= 64 without a division: the quotient is below 64, so a float estimate
                    // (relative error ~2^-23) is off by at most one, and one correction fixes it
                    const float rn = pool ? rn_b : rn_m;
                    auto mulmod = [&](uint32_t k) -> uint32_t {
                        const unsigned long long pr = (unsigned long long)k * step;
                        const long long qq = (long long)((float)pr * rn);
                        long long r = (long long)pr - qq * (long long)un;
                        if (r < 0) r += un;
                        else if (r >= (long long)un) r -= un;
                        return (uint32_t)r;
                    };
                    const uint32_t d64 = mulmod(64u);
                    const int sb = __builtin_amdgcn_readlane(g_cs, q);  // (0 unless a cursor of this generation)
                    const uint32_t start = (uint32_t)__builtin_amdgcn_readlane((int)g_cp, q);  // (home + sb step) mod n
                    uint32_t pos = madd(start, mulmod((uint32_t)lane));
                    auto adv = [&](uint32_t x) -> uint32_t { return madd(x, d64); };
                    long long ts = (long long)n + 2;  // the step taken (n + 2: none), its position and permits
                    uint32_t tpos = 0u;
                    int pvt = 0, tix = -1;
                    uint4 te = make_uint4(0u, 0u, 0u, 0u);
                    for (long long s0 = sb; s0 < (long long)n + 2 && t < 0; s0 += 256) {
                        bool ok[4], tried[4];
                        int id[4];
                        int pvs[4];
                        uint32_t uw[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {  // every position is inside the pool: all loads at once
                            id[u] = base + (int)pos;
                            pos = adv(pos);
                            uw[u] = S.usable[id[u] >> 5];
                            pvs[u] = id[u] < S.n_slots ? ld_i(&S.permits[id[u]]) : 0;
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const long long s = s0 + 64 * u + lane;
                            tried[u] = s < (long long)n + 2 && ((uw[u] >> (id[u] & 31)) & 1u) && id[u] < S.n_slots;
                            ok[u] = tried[u] && pvs[u] >= mem;  // tryAcquire (FS:63-71), or the memory of a container
                        }
                        int ixs[4];
                        uint4 es[4];
                        if (maxc > 1) {  // the (invoker, fqn) entry at each tried step: a free slot (NS:57-82)
                            sq_find4(S, id, slot, tried, ixs, es);
#pragma unroll
                            for (int u = 0; u < 4; ++u) ok[u] = ok[u] || (tried[u] && ixs[u] >= 0 && (int)es[u].z >= 1);
                        }
                        int uf = 4, lf = 64;
#pragma unroll
                        for (int u = 3; u >= 0; --u) {
                            const u64 m = __ballot(ok[u]);
                            if (m) {
                                uf = u;
                                lf = ffs64(m);
                            }
                        }
                        if (maxc > 1) {
                            // the tries that failed before the first success leave empty entries (getOrElseUpdate,
                            // NS:61-62); steps n and n + 1 repeat positions 0 and 1, whose entries the first pass made
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                const long long s = s0 + 64 * u + lane;
                                const bool before = u < uf || (u == uf && lane < lf);
                                bool ins = false;
                                if (tried[u] && !ok[u] && before && s < n && ixs[u] < 0) {  // (absent: looked up above)
                                    ins = true;
                                    if (sq_insert(S, id[u], slot, 0, 0) < 0) err = 1;
                                }
                                filled += __popcll(__ballot(ins));
                            }
                            mem_done();
                        }
                        if (uf < 4) {  // (uf, lf uniform: lane reads, no LDS round trip)
                            t = __builtin_amdgcn_readlane(uf == 0 ? id[0] : uf == 1 ? id[1] : uf == 2 ? id[2] : id[3], lf);
                            pvt = __builtin_amdgcn_readlane(uf == 0 ? pvs[0] : uf == 1 ? pvs[1] : uf == 2 ? pvs[2] : pvs[3], lf);
                            if (maxc > 1) {  // its entry as the walk found it (the empty entries made since are others)
                                const int sel_ix = uf == 0 ? ixs[0] : uf == 1 ? ixs[1] : uf == 2 ? ixs[2] : ixs[3];
                                const uint4 sel_e = uf == 0 ? es[0] : uf == 1 ? es[1] : uf == 2 ? es[2] : es[3];
                                tix = __builtin_amdgcn_readlane(sel_ix, lf);
                                te = make_uint4((uint32_t)__builtin_amdgcn_readlane((int)sel_e.x, lf),
                                                (uint32_t)__builtin_amdgcn_readlane((int)sel_e.y, lf),
                                                (uint32_t)__builtin_amdgcn_readlane((int)sel_e.z, lf),
                                                (uint32_t)__builtin_amdgcn_readlane((int)sel_e.w, lf));
                            }
                            ts = s0 + 64 * uf + lf;
                            tpos = (uint32_t)(t - base);
                        }
                    }
                    if (maxc <= 1 && S.cur) {  // the action's cursor: the step it took, or past the walk
                        const int aq = __builtin_amdgcn_readlane(g_a, q);
                        if (lane > q && g_a == aq) {
                            g_cs = (int)ts;
                            g_cp = tpos;
                        }
                        if (lane == 0 && aq >= 0 && aq < S.n_actions) S.cur[aq] = make_uint4(gen, (uint32_t)ts, tpos, 0u);
                    }
                    if (t < 0) {  // n + 2 failed probes: a random healthy invoker, forced (SCPB:417-424)
                        const int H = pool ? hb : hm;
                        if (H > 0) {
                            const int kk = (int)rng_index(S.rng_seed, seq, (uint32_t)H);
                            t = select_usable(base, kk);
                            if (t < 0) err = 1;
                            fl = 1;
                        }
                    }
                    if (t >= 0) {
                        out = t;
                        int took = 0;
                        if (lane == 0) {
                            if (maxc <= 1) {
                                // tryAcquire succeeded (the walk read its permits) / forceAcquire (FS:107-110)
                                S.permits[t] = jsub(fl ? ld_i(&S.permits[t]) : pvt, mem);
                                took = mem;
                            } else {
                                uint4 e = te;
                                int ix = tix;
                                if (fl) ix = sq_find(S, t, slot, &e);  // (a forced invoker: not looked up by the walk)
                                if (ix < 0) {  // getOrElseUpdate (NS:61-62)
                                    ++filled;  // (lane 0's copy; broadcast below)
                                    ix = sq_insert(S, t, slot, 0, 0);
                                    e = make_uint4(0u, 0u, 0u, 0u);
                                    if (ix < 0) err = 1;
                                }
                                int c = (int)e.z, ops = (int)e.w;
                                if (c - 1 >= 0) {  // RS.tryAcquire(1) (RS:62-70)
                                    c = c - 1;
                                    ops = jadd(ops, 1);
                                } else {  // the memory (tried above, or forced): RS.release(maxConcurrent - 1, false)
                                    S.permits[t] = jsub(fl ? ld_i(&S.permits[t]) : pvt, mem);
                                    took = mem;
                                    ops = jadd(ops, 1);
                                    const int n2 = jadd(c, maxc - 1);
                                    c = n2 % maxc == 0 ? jsub(n2, maxc) : n2;
                                }
                                if (ix >= 0) {
                                    S.map[ix].z = (uint32_t)c;
                                    S.map[ix].w = (uint32_t)ops;
                                }
                            }
                        }
                        taken_at = t;
                        taken = __builtin_amdgcn_readlane(took, 0);
                    } else {
                        out = OWGS_NONE_V;  // no healthy invoker: None (SCPB:419-420)
                    }
                    // decided alone: the group's later decisions of its action re-walk (their ranks assumed it where
                    // its speculation put it)
                    const int aq = __builtin_amdgcn_readlane(g_a, q);
                    if (maxc <= 1 && lane > q && g_a == aq) inval = true;
                    if (maxc > 1 && lane > q && g_slot == slot) inval = true;  // (its key's later speculations)
                }
                if (taken > 0) {
                    const int aq = __builtin_amdgcn_readlane(g_a, q);
                    acc += ((sp_k == 1 || sp_k == 3) && sp_t == taken_at && !(kept_plain && g_a == aq && uniq)) ? taken : 0;
                }
                if (lane == q) {
                    my_out = out;
                    my_fl = fl;
                }
                filled = ((long long)__builtin_amdgcn_readlane((int)(filled >> 32), 0) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)filled, 0);
                if (!spec_done) mem_done();  // (lane 0's permit and entry stores, before the next decision reads them)
                tick(spec_done ? 2 : 3);
            }
            flush();
            if (lane < q) {  // the decided part of the group (all of it unless the map must grow first)
                S.out_inv[j0 + lane] = my_out;
                S.out_flags[j0 + lane] = (uint8_t)my_fl;
            }
            mem_done();  // (a later run's releases read these decisions)
            j = j0 + q;
        }
        if (stop) break;
    }
    const bool any_err = __ballot(err != 0) != 0;  // (any lane's: speculated decisions commit in their own lanes)
    if (lane == 0) {
        // where to resume (the map must grow first: a publish, phase 1) or done
        S.state[0] = stop ? 1 : 0;
        S.state[1] = r;
        S.state[2] = 1;
        S.state[3] = (int)(uint32_t)(j & 0xFFFFFFFFll);
        S.state[4] = (int)(j >> 32);
        S.state[5] = (int)gen;
        S.state[6] = n_spec;
        S.state[7] = n_alone;
        const u64 cys[4] = {cy0, cy1, cy2, cy3};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            S.state[8 + 2 * k] = (int)(uint32_t)cys[k];
            S.state[9 + 2 * k] = (int)(uint32_t)(cys[k] >> 32);
        }
        if (any_err) atomicOr(S.err, OWGS_ERR_INTERNAL);
    }
}

// the map grown: live entries rehashed into the new table (one thread per old entry)
__global__ __launch_bounds__(256) void owgs_seq_rehash_kernel(const uint4* old, int32_t old_cap, OwgsSeqArgs S) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= old_cap) return;
    const uint4 e = old[i];
    if (e.x == 0u || e.x == 0xFFFFFFFFu) return;
    if (sq_insert(S, (int)e.x - 1, (int)e.y, (int)e.z, (int)e.w) < 0) atomicOr(S.err, OWGS_ERR_CTAB_FULL);
}

// A context that outgrows the on-chip engines mid-life (updateInvokers with more invokers, an action with maxConcurrent
// beyond 4095) carries its NestedSemaphore maps over: every entry of the on-chip map's HBM image (primary table, then
// its overflow) -- key (invoker + 1) | slot << 15, value c | signed operationCount << 12 -- into the large map
__global__ __launch_bounds__(256) void owgs_seq_migrate_kernel(const uint32_t* ct_keys, const uint32_t* ct_vals,
                                                               int32_t n_ct, const uint2* ovf, int32_t ovf_cap,
                                                               OwgsSeqArgs S) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n_ct + ovf_cap) return;
    const uint32_t k = i < n_ct ? ct_keys[i] : ovf[i - n_ct].x;
    const uint32_t v = i < n_ct ? ct_vals[i] : ovf[i - n_ct].y;
    if (k == 0u || k == 0xFFFFFFFFu) return;
    const int inv = (int)(k & 0x7FFFu) - 1, slot = (int)(k >> 15);
    if (sq_insert(S, inv, slot, (int)(v & 0xFFFu), (int)v >> 12) < 0) atomicOr(S.err, OWGS_ERR_CTAB_FULL);
}
// ... and the watched pairs whose empty entry the reference holds (Z): {0 free, 0 operations}
__global__ __launch_bounds__(256) void owgs_seq_migrate_w_kernel(const uint32_t* w_keys, const uint32_t* w_vals,
                                                                 int32_t w_cap, OwgsSeqArgs S) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= w_cap) return;
    const uint32_t k = w_keys[j];
    if (k == 0u || k == 0xFFFFFFFFu || !(w_vals[j] & OWGS_W_Z)) return;
    const int inv = (int)(k & 0x7FFFu) - 1, slot = (int)(k >> 15);
    uint4 e;
    if (sq_find(S, inv, slot, &e) < 0 && sq_insert(S, inv, slot, 0, 0) < 0) atomicOr(S.err, OWGS_ERR_CTAB_FULL);
}

// one (invoker, fqn@version) entry: {found, c, ops} into out (concurrentState, NS:115)
__global__ void owgs_seq_lookup_kernel(OwgsSeqArgs S, int32_t inv, int32_t slot, int32_t* out) {
    uint4 e;
    const int ix = sq_find(S, inv, slot, &e);
    out[0] = ix >= 0;
    out[1] = ix >= 0 ? (int)e.z : 0;
    out[2] = ix >= 0 ? (int)e.w : 0;
}

extern "C" hipError_t owgs_launch_seq(const OwgsSeqArgs* a, hipStream_t s) {
    if (((a->n_ids + 31) >> 5) > OWGS_SEQ_MAX_WORDS) return hipErrorInvalidValue;
    hipLaunchKernelGGL(owgs_seq_kernel, dim3(1), dim3(64), 0, s, *a);
    return hipGetLastError();
}
extern "C" hipError_t owgs_launch_seq_rehash(const uint4* old, int32_t old_cap, const OwgsSeqArgs* a, hipStream_t s) {
    if (old_cap <= 0) return hipSuccess;
    hipLaunchKernelGGL(owgs_seq_rehash_kernel, dim3((unsigned)((old_cap + 255) / 256)), dim3(256), 0, s, old, old_cap, *a);
    return hipGetLastError();
}
extern "C" hipError_t owgs_launch_seq_lookup(const OwgsSeqArgs* a, int32_t inv, int32_t slot, int32_t* out,
                                             hipStream_t s) {
    hipLaunchKernelGGL(owgs_seq_lookup_kernel, dim3(1), dim3(1), 0, s, *a, inv, slot, out);
    return hipGetLastError();
}
extern "C" hipError_t owgs_launch_seq_migrate(const uint32_t* ct_keys, const uint32_t* ct_vals, int32_t n_ct,
                                              const uint2* ovf, int32_t ovf_cap, const uint32_t* w_keys,
                                              const uint32_t* w_vals, int32_t w_cap, const OwgsSeqArgs* a, hipStream_t s) {
    const int n = n_ct + (ovf ? ovf_cap : 0);
    if (n > 0)
        hipLaunchKernelGGL(owgs_seq_migrate_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, ct_keys, ct_vals,
                           n_ct, ovf, ovf ? ovf_cap : 0, *a);
    if (w_keys && w_cap > 0)
        hipLaunchKernelGGL(owgs_seq_migrate_w_kernel, dim3((unsigned)((w_cap + 255) / 256)), dim3(256), 0, s, w_keys,
                           w_vals, w_cap, *a);
    return hipGetLastError();
}
