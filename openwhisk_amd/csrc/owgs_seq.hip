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
                int my_f = 0;
                for (int q = 0; q < nq; ++q) {
                    const int inv = __builtin_amdgcn_readlane(g_inv, q);
                    int f = 0;
                    if (inv >= 0 && inv < S.n_slots && lane == 0) {  // invokerSlots.lift (SCPB:329)
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
            int my_out = OWGS_NONE_V, my_fl = 0;
            int q = 0;
            for (; q < nq; ++q) {
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
                if (kind == 1) {
                    out = OWGS_NONE_V;  // no invokers in the pool: None (SCPB:288-290)
                } else if (kind == 2) {
                    out = OWGS_THROW_V;  // Int.MinValue hash: stepSizes / invokers index out of bounds (SCPB:266-268)
                } else {
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
                        if (lane == 0) {
                            if (maxc <= 1) {
                                // tryAcquire succeeded (the walk read its permits) / forceAcquire (FS:107-110)
                                S.permits[t] = jsub(fl ? ld_i(&S.permits[t]) : pvt, mem);
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
                    } else {
                        out = OWGS_NONE_V;  // no healthy invoker: None (SCPB:419-420)
                    }
                }
                if (lane == q) {
                    my_out = out;
                    my_fl = fl;
                }
                filled = ((long long)__builtin_amdgcn_readlane((int)(filled >> 32), 0) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)filled, 0);
                mem_done();  // (lane 0's permit and entry stores, before the next decision reads them)
            }
            if (lane < q) {  // the decided part of the group (all of it unless the map must grow first)
                S.out_inv[j0 + lane] = my_out;
                S.out_flags[j0 + lane] = (uint8_t)my_fl;
            }
            mem_done();  // (a later run's releases read these decisions)
            j = j0 + q;
        }
        if (stop) break;
    }
    if (lane == 0) {
        // where to resume (the map must grow first: a publish, phase 1) or done
        S.state[0] = stop ? 1 : 0;
        S.state[1] = r;
        S.state[2] = 1;
        S.state[3] = (int)(uint32_t)(j & 0xFFFFFFFFll);
        S.state[4] = (int)(j >> 32);
        S.state[5] = (int)gen;
        if (err) atomicOr(S.err, OWGS_ERR_INTERNAL);
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
