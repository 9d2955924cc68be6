// owgs_kernels.hip -- CDNA4 (gfx950) kernels of the batched invoker scheduler.
//
// Kernels
//   owgs_hash_kernel     generateHash(namespace, action) (SCPB:370-372): java.lang.String.hashCode of both strings,
//                        one wave per action; lane i sums c[i+64k] * 31^(L-1-i-64k) (mod 2^32), the wave reduces.
//   owgs_prepare_kernel  per action: home = hash % n, step = stepSizes(hash % k), meta bits (SCPB:262-268).
//   owgs_lookup_kernel   NestedSemaphore.concurrentState reads (introspection).
//   owgs_engine_kernel   the hot path: releases (SCPB:327-331 -> NS:98-113) and schedule() (SCPB:398-436 with
//                        NS:32-91) for a whole stream of batches, replaying the reference's SEQUENTIAL semantics.
//
// Engine design (DESIGN.md "Engine").  One wavefront owns one controller shard.  Slot permits, pool vectors and a
// per-action walk cursor live in LDS for the whole stream (HBM is read once and written once); the concurrency maps
// live in one 8-byte-entry open-addressing table (L2-resident).  Activations are taken 64 at a time (one per lane, in
// stream order) and resolved by speculation + exact validation:
//   * memory permits never increase inside a batch (releases are applied at batch boundaries), so a probe that
//     fails against the state at the chunk frontier f fails at every later time: a lane's speculated target is never
//     EARLIER in its walk than its true target, and the per-action cursor (first walk step that may still be feasible)
//     only moves forward inside a batch;
//   * lanes are grouped by target invoker (LDS stamp table + ballot); inside a group an exclusive prefix sum of the
//     memory consumed by earlier lanes gives each lane the permits left at its own time, and concurrency slots are
//     modelled per (target, action) from the rank inside the group;
//   * the first lane l* whose speculation does not hold is a TRUE rejection (every earlier lane was exact), lanes
//     [f, l*) commit, l* (and the later lanes of the same maxConcurrent==1 action at the same target) step past the
//     target, and the chunk iterates with f = l*.  The frontier lane is always exact, so every iteration commits.
//   * cases whose speculation cannot be validated cheaply (an earlier lane of the chunk that may create concurrency
//     slots for the same fqn on another walk, or a forced acquire) are treated as uncertain and resolved when they
//     reach the frontier.
#include <hip/hip_runtime.h>

#include "owgs_internal.h"

typedef unsigned long long u64;

#define K_NONE 0
#define K_THROW 1
#define K_TARGET 2
#define K_FALLBACK 3
#define K_LONG 4

#define KPROBE 4

// diagnostic build (-DOWGS_PROFILE, libowgs_prof.so): s_memtime cycle accounting per engine phase into stats[8..15]
#ifdef OWGS_PROFILE
#define PT_DECL                 \
    u64 pt_acc[8] = {0};        \
    u64 pt_t = __builtin_amdgcn_s_memtime();
#define PT(k)                                          \
    {                                                  \
        const u64 _t = __builtin_amdgcn_s_memtime();   \
        pt_acc[k] += _t - pt_t;                        \
        pt_t = _t;                                     \
    }
#else
#define PT_DECL
#define PT(k)
#endif

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

// (index + step) % numInvokers (SCPB:429) for index, step in [0, n]: one conditional subtract, no division
__device__ __forceinline__ int next_pos(int pos, int step, int n) {
    const int p = pos + step;
    return p >= n ? p - n : p;
}

// x mod R for 0 <= x < 2^24, 1 <= R < 2^24 without an integer division (float reciprocal, one correction step)
__device__ __forceinline__ int mod_small(int x, int R) {
    const int q = (int)((float)x * __builtin_amdgcn_rcpf((float)R));
    int r = x - q * R;
    if (r < 0) r += R;
    if (r >= R) r -= R;
    return r;
}

__device__ __forceinline__ int ffs64(u64 m) { return __ffsll((long long)m) - 1; }
__device__ __forceinline__ int fls64(u64 m) { return 63 - __clzll((long long)m); }

__device__ __forceinline__ void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// DPP (GFX9 row_shr / row_bcast) wave64 scans: no LDS round trip, ~6 VALU ops.
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
__device__ __forceinline__ int wave_excl_scan(int v) { return wave_incl_scan(v) - v; }

template <int CTRL, int ROWM>
__device__ __forceinline__ int dpp_keep(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWM, 0xf, false);  // invalid source lanes keep `old`
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
__device__ __forceinline__ int wave_min(int v) {
    const int I = 0x7FFFFFFF;
    v = min(v, dpp_keep<0x111, 0xf>(I, v));
    v = min(v, dpp_keep<0x112, 0xf>(I, v));
    v = min(v, dpp_keep<0x114, 0xf>(I, v));
    v = min(v, dpp_keep<0x118, 0xf>(I, v));
    v = min(v, dpp_keep<0x142, 0xa>(I, v));
    v = min(v, dpp_keep<0x143, 0xc>(I, v));
    return __builtin_amdgcn_readlane(v, 63);
}

// ---- concurrency table: entry = key32 << 32 | val32; key32 = (inv+1) | slot << 15; val32 = c | ops << 12
__device__ __forceinline__ uint32_t ct_key(int inv, int slot) {
    return (uint32_t)(inv + 1) | ((uint32_t)slot << OWGS_CT_SLOT_SHIFT);
}
__device__ __forceinline__ uint32_t ct_hash(uint32_t k) {
    k ^= k >> 16;
    k *= 0x7feb352dU;
    k ^= k >> 15;
    k *= 0x846ca68bU;
    k ^= k >> 16;
    return k;
}
__device__ __forceinline__ int ct_c(u64 e) { return (int)((uint32_t)e & OWGS_CT_C_MASK); }
__device__ __forceinline__ int ct_ops(u64 e) { return (int)((uint32_t)e >> OWGS_CT_C_BITS); }
__device__ __forceinline__ u64 ct_entry(uint32_t key, int c, int ops) {
    return ((u64)key << 32) | (u64)((uint32_t)c | ((uint32_t)ops << OWGS_CT_C_BITS));
}

// returns table index or -1; *e = entry (0 if absent)
__device__ int ct_find(const u64* tab, uint32_t mask, uint32_t key, u64* e) {
    uint32_t h = ct_hash(key) & mask;
    for (uint32_t p = 0; p <= mask; ++p) {
        const u64 v = tab[h];
        if ((uint32_t)(v >> 32) == key) {
            *e = v;
            return (int)h;
        }
        if (v == 0) break;
        h = (h + 1) & mask;
    }
    *e = 0;
    return -1;
}

__device__ int ct_insert(u64* tab, uint32_t mask, uint32_t key) {
    uint32_t h = ct_hash(key) & mask;
    for (uint32_t p = 0; p <= mask; ++p) {
        const u64 v = tab[h];
        if (v == 0 || (uint32_t)(v >> 32) == key) return (int)h;
        h = (h + 1) & mask;
    }
    return -1;
}

// c of NestedSemaphore(inv).actionConcurrentSlotsMap(slot); absent entries (operationCount 0) read as c = 0
__device__ __forceinline__ int conc_lookup(const OwgsEngineArgs& A, int inv, int slot, int* idx, int* ops) {
    u64 e;
    *idx = ct_find(A.ctab, A.ctab_mask, ct_key(inv, slot), &e);
    *ops = ct_ops(e);
    return *ops > 0 ? ct_c(e) : 0;
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
    u64 e;
    ct_find(a.ctab, a.ctab_mask, ct_key(a.inv[i], a.slot[i]), &e);
    a.out[i] = make_int2(ct_c(e), ct_ops(e));
}

// dense per-activation / per-release records (one coalesced load each in the engine instead of dependent gathers)
__global__ __launch_bounds__(256) void owgs_gather_kernel(OwgsGatherArgs g) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < g.n_act; i += stride) {
        const int a = g.act[i];
        g.info[i] = g.act_info[a];
        g.aux[i] = make_int2(g.act_slot[a], a);
    }
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < g.n_rel; r += stride) {
        int x, a;
        if (g.rel_inv) {
            x = g.rel_inv[r];
            a = g.rel_act[r];
        } else {
            const int64_t aid = g.rel_aid[r];
            x = (int)aid;
            a = g.act[aid];
        }
        const int4 ai = g.act_info[a];
        g.rinfo[r] = make_int4(x, ai.z, ai.w, g.act_slot[a]);
    }
}

// home/step selection (SCPB:266-268)
__global__ __launch_bounds__(256) void owgs_prepare_kernel(OwgsPrepArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const int pool = a.bb[i] ? 1 : 0;
    const int n = pool ? a.nb : a.nm;
    const int k = pool ? a.n_bsteps : a.n_msteps;
    const int32_t* steps = pool ? a.bsteps : a.msteps;
    uint32_t meta = (uint32_t)(a.maxc[i] & OWGS_META_MAXC_MASK) | ((uint32_t)pool << OWGS_META_POOL_SHIFT);
    if (a.cursor_ok[i]) meta |= OWGS_META_CURSOR;
    int home = 0, step = 0;
    if (n <= 0) {
        meta |= OWGS_META_EMPTY;
    } else if (k <= 0) {
        meta |= OWGS_META_THROW;
    } else {
        const int h = a.hash[i];
        home = h % n;
        const int si = h % k;
        if (si < 0 || home < 0) meta |= OWGS_META_THROW;
        else step = steps[si] % n;  // same walk; lets the engine advance with one conditional subtract
    }
    a.act_info[i] = make_int4(home, step, a.mem[i], (int)meta);
}

// ------------------------------------------------------------------------------------------------ engine
// concurrency slots an acquisition finds, given c0 at state f and q earlier same-fqn lanes at the same invoker
__device__ __forceinline__ int c_now_of(int c0, int q, int R) {
    const int x = q - c0;
    if (x < 0) return c0 - q;
    const int r = mod_small(x, R);
    return r == 0 ? 0 : R - r;
}

__device__ __forceinline__ uint32_t next_stamp(uint32_t& iter, uint32_t* st, int lane) {
    ++iter;
    if ((iter & 0x03FFFFFFu) == 0) {  // stamps are (2^26 - iter) << 6 | lane: re-arm the tables on wrap
        for (int t = lane; t < 2 * OWGS_STAMP_BUCKETS; t += 64) st[t] = 0xFFFFFFFFu;
        wave_fence();
        ++iter;
    }
    return ((0x03FFFFFFu - (iter & 0x03FFFFFFu)) << 6) | (uint32_t)lane;
}

struct CoopResult {
    int kind, tgt, pv, s, pos, c, cidx, ops;
};

// Wave-cooperative walk for lane `who` (all lanes call it): walk steps s0.. are probed 64 at a time and ballot picks
// the first feasible one.  kind = K_TARGET / K_THROW, or K_LONG when every remaining step fails (s = n).
__device__ CoopResult coop_walk(const OwgsEngineArgs& A, const int32_t* perm, const int32_t* pw, int who, int s_l,
                                int pos_l, int step_l, int n_l, int pwb_l, int mem_l, int maxc_l, int slot_l) {
    const int lane = threadIdx.x;
    int s0 = __builtin_amdgcn_readlane(s_l, who);
    int p0 = __builtin_amdgcn_readlane(pos_l, who);
    const int stp = __builtin_amdgcn_readlane(step_l, who);
    const int nn = __builtin_amdgcn_readlane(n_l, who);
    const int pb = __builtin_amdgcn_readlane(pwb_l, who);
    const int m = __builtin_amdgcn_readlane(mem_l, who);
    const int mc = __builtin_amdgcn_readlane(maxc_l, who);
    const int sl = __builtin_amdgcn_readlane(slot_l, who);
    CoopResult r{K_LONG, -1, 0, nn, p0, 0, -1, 0};
    const int loff = (int)(((uint32_t)lane * (uint32_t)stp) % (uint32_t)nn);
    const int boff = (int)((64u * (uint32_t)stp) % (uint32_t)nn);
    while (s0 < nn) {
        const int sk = s0 + lane;
        const int p = next_pos(p0, loff, nn);
        bool feas = false;
        int w = -1, c = 0, ix = -1, o = 0, pvv = 0;
        if (sk < nn) {
            w = pw[pb + p];
            if (w == OWGS_PW_BADID) {
                feas = true;
            } else if (w >= 0) {
                pvv = perm[w];
                feas = pvv >= m;
                if (mc > 1) {
                    c = conc_lookup(A, w, sl, &ix, &o);
                    feas = feas || c >= 1;
                }
            }
        }
        const u64 fm = __ballot(feas);
        if (fm) {
            const int j = ffs64(fm);
            r.tgt = __builtin_amdgcn_readlane(w, j);
            r.c = __builtin_amdgcn_readlane(c, j);
            r.cidx = __builtin_amdgcn_readlane(ix, j);
            r.ops = __builtin_amdgcn_readlane(o, j);
            r.pv = __builtin_amdgcn_readlane(pvv, j);
            r.pos = __builtin_amdgcn_readlane(p, j);
            r.s = s0 + j;
            r.kind = (r.tgt == OWGS_PW_BADID) ? K_THROW : K_TARGET;
            return r;
        }
        s0 += 64;
        p0 = next_pos(p0, boff, nn);
    }
    return r;
}

// fallback target (SCPB:417-424): H = usable pool members in pool order, r = H[rng(seq) mod |H|]
__device__ __forceinline__ void fallback_target(const OwgsEngineArgs& A, int pool, int64_t i, int n_slots, int* kind,
                                                int* tgt) {
    const int hc = pool ? A.hb : A.hm;
    if (hc <= 0) {
        *kind = K_NONE;
        return;
    }
    const u64 seq = A.seq ? A.seq[i] : (A.seq_base + (u64)i);
    const int r = A.hlist[(pool ? A.hm : 0) + (int)rng_index(A.rng_seed, seq, (uint32_t)hc)];
    if (r < 0 || r >= n_slots) {
        *kind = K_THROW;
        return;
    }
    *kind = K_FALLBACK;
    *tgt = r;
}

__global__ __launch_bounds__(64) void owgs_engine_kernel(OwgsEngineArgs A) {
    extern __shared__ __attribute__((aligned(16))) int32_t lds_raw[];
    const int lane = threadIdx.x;
    const int n_slots = A.n_slots, nm = A.nm, nb = A.nb;
    int32_t* perm = lds_raw;
    int32_t* pw = lds_raw + ((n_slots + 3) & ~3);
    uint32_t* stT = (uint32_t*)(pw + ((nm + nb + 3) & ~3));
    uint32_t* stS = stT + OWGS_STAMP_BUCKETS;
    int32_t* cur = (int32_t*)(stS + OWGS_STAMP_BUCKETS);
    const int n_cur = A.n_cursors;

    for (int i = lane; i < n_slots; i += 64) perm[i] = A.permits[i];
    for (int i = lane; i < nm + nb; i += 64) pw[i] = A.pool_words[i];
    for (int i = lane; i < 2 * OWGS_STAMP_BUCKETS; i += 64) stT[i] = 0xFFFFFFFFu;
    __syncthreads();

    uint32_t st_iter = 0, st_fb = 0, st_long = 0, st_grp = 0, st_probe = 0, st_inc = 0;
    PT_DECL
    uint32_t iter = 0;
    const u64 lt_mask = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
    const u64 self_bit = 1ull << lane;

    for (int b = 0; b < A.n_batches; ++b) {
        // ================================================================ releases (SCPB:327-331, NS:98-113)
        const int64_t r_beg = A.rel_off ? A.rel_off[b] : 0, r_end = A.rel_off ? A.rel_off[b + 1] : 0;
        for (int64_t r0 = r_beg; r0 < r_end; r0 += 64) {
            const bool valid = lane < r_end - r0;
            int inv = -1, mem = 0, maxc = 1, slot = 0;
            if (valid) {
                const int4 ri = A.rinfo[r0 + lane];
                inv = A.rel_inv ? ri.x : A.out_inv[ri.x];
                mem = ri.y;
                maxc = ri.z & OWGS_META_MAXC_MASK;
                slot = ri.w;
            }
            uint8_t flag = 0;
            bool conc = false, rel = false;
            if (valid) {
                if (inv < 0) flag = OWGS_REL_NOENTRY_BIT;  // no ActivationEntry (CLB:278-279)
                else if (inv >= n_slots) flag = 0;          // invokerSlots.lift -> no-op
                else if (maxc == 1) rel = true;
                else conc = true;
            }
            if (__ballot(conc)) {
                int idx = -1, c0 = 0, o0 = 0;
                if (conc) {
                    u64 e;
                    idx = ct_find(A.ctab, A.ctab_mask, ct_key(inv, slot), &e);
                    c0 = ct_c(e);
                    o0 = ct_ops(e);
                    if (idx < 0 || o0 <= 0) {
                        conc = false;
                        flag = OWGS_REL_NOSUCH_BIT;  // actionConcurrentSlotsMap(actionid) throws (NS:103)
                    }
                }
                // releases of one entry inside this group of 64: rank in stream order and group size
                int rank = 0, gsz = 1;
                const uint32_t stamp = next_stamp(iter, stT, lane);
                if (conc) atomicMin(&stT[idx & (OWGS_STAMP_BUCKETS - 1)], stamp);
                wave_fence();
                const bool leader = conc && stT[idx & (OWGS_STAMP_BUCKETS - 1)] == stamp;
                u64 pend = __ballot(conc && !leader);
                while (pend) {
                    const int j = ffs64(pend);
                    const int e = __builtin_amdgcn_readlane(idx, j);
                    const u64 G = __ballot(conc && idx == e);
                    if ((G >> lane) & 1) {
                        rank = __popcll(G & lt_mask);
                        gsz = __popcll(G);
                    }
                    pend &= ~G;
                }
                if (conc) {
                    // RS.release(1, opComplete = true) applied rank+1 times to (c0, o0), reductionSize = maxConc
                    if (rank < o0) rel = mod_small(c0 + rank + 1, maxc) == 0;
                    else flag = OWGS_REL_NOSUCH_BIT;  // entry already removed by an earlier release of this group
                    if (rank == 0) {
                        const int j = min(gsz, o0);
                        int c1 = mod_small(c0 + j, maxc);
                        const int o1 = o0 - j;
                        if (o1 == 0) c1 = 0;  // actionRelease: entry removed (NS:109-111)
                        A.ctab[idx] = ct_entry(ct_key(inv, slot), c1, o1);
                    }
                }
            }
            if (rel) {
                const int old = atomicAdd(&perm[inv], mem);
                if (old > 0x7FFFFFFF - mem) {  // ForcibleSemaphore overflow -> Error, state unchanged (FS:48-50)
                    atomicSub(&perm[inv], mem);
                    flag |= OWGS_REL_OVERFLOW_BIT;
                }
            }
            if (valid && A.rel_flags) A.rel_flags[r0 + lane] = flag;
            wave_fence();
            PT(0);
        }

        // ================================================================ per-batch bounds and cursors
        // U0/U1 >= max permits over usable members of the managed/blackbox pool; permits only fall inside a batch.
        int U0, U1;
        {
            int m0 = (int)0x80000000, m1 = (int)0x80000000;
            for (int i = lane; i < nm; i += 64) {
                const int w = pw[i];
                if (w >= 0) m0 = max(m0, perm[w]);
            }
            for (int i = lane; i < nb; i += 64) {
                const int w = pw[nm + i];
                if (w >= 0) m1 = max(m1, perm[w]);
            }
            U0 = wave_max(m0);
            U1 = wave_max(m1);
        }
        for (int i = lane; i < n_cur; i += 64) cur[i] = 0;
        wave_fence();
        PT(1);

        // ================================================================ acquires (SCPB:398-436, NS:32-91)
        const int64_t a_beg = A.acq_off[b], a_end = A.acq_off[b + 1];
        for (int64_t c0i = a_beg; c0i < a_end; c0i += 64) {
            bool pending = lane < a_end - c0i;
            const int64_t i = c0i + (pending ? lane : 0);
            int a = -1, home = 0, step = 0, mem = 0, meta = 0, slot = 0;
            if (pending) {
                const int4 info = A.info[i];
                const int2 ax = A.aux[i];
                home = info.x;
                step = info.y;
                mem = info.z;
                meta = info.w;
                slot = ax.x;
                a = ax.y;
            }
            const int maxc = meta & OWGS_META_MAXC_MASK;
            const int pool = (meta >> OWGS_META_POOL_SHIFT) & 1;
            const int n = pool ? nb : nm;
            const int pwb = pool ? nm : 0;
            const bool cok = (meta & OWGS_META_CURSOR) && a >= 0 && a < n_cur;
            int s = 0, pos = home;  // walk step and its pool position, kept across iterations
            if (pending && ((meta & (OWGS_META_EMPTY | OWGS_META_THROW)) || home < 0 || home >= n || step < 0)) {
                A.out_inv[i] = (meta & OWGS_META_EMPTY) ? OWGS_NONE_V : OWGS_THROW_V;  // None / schedule() throws
                A.out_flags[i] = 0;
                pending = false;
            }

            int f = 0;
            bool full = true;  // lanes >= f need (re)speculation
            // per-lane speculation, valid for lanes >= f until the next full pass
            int kind = K_NONE, tgt = -1, room = 0, c0 = 0, cidx = -1, ops0 = 0, q = 0, cons = 0;
            bool unc = false, fullwalk = false;
            PT(2);
            while (__ballot(pending)) {
                const bool act = pending && lane >= f;
                if (full) {
                    full = false;
                    ++st_iter;
                    // ---------------------------------------------------- speculate targets against state at f
                    kind = K_NONE;
                    tgt = -1;
                    c0 = 0;
                    cidx = -1;
                    ops0 = 0;
                    q = 0;
                    unc = false;
                    fullwalk = false;
                    int pv = 0;
                    if (act) {
                        if (cok) {  // cursor = walk step << 16 | pool position
                            const int cv = cur[a];
                            if ((cv >> 16) > s) {
                                s = cv >> 16;
                                pos = cv & 0xFFFF;
                            }
                        }
                        kind = K_LONG;
                        if (maxc == 1) {
                            if (mem > (pool ? U1 : U0) && ((A.shortcut_ok >> pool) & 1)) {
                                kind = K_FALLBACK;  // every usable permit < mem: the walk fails everywhere
                            } else {
#pragma unroll 1
                                for (int k = 0; k < KPROBE; ++k) {
                                    if (s >= n) {  // every pool position probed: the n+2-probe walk fails (SCPB:417)
                                        kind = K_FALLBACK;
                                        fullwalk = true;
                                        break;
                                    }
                                    const int w = pw[pwb + pos];
                                    ++st_probe;
                                    if (w >= 0) {
                                        const int p = perm[w];
                                        if (p >= mem) {
                                            kind = K_TARGET;
                                            tgt = w;
                                            pv = p;
                                            break;
                                        }
                                    } else if (w == OWGS_PW_BADID) {
                                        kind = K_THROW;
                                        break;
                                    }
                                    pos = next_pos(pos, step, n);
                                    ++s;
                                }
                            }
                        }
                    }
                    if (__ballot(act && maxc > 1)) {  // concurrent actions: c >= 1 also makes a probe feasible
                        if (act && maxc > 1) {
#pragma unroll 1
                            for (int k = 0; k < KPROBE; ++k) {
                                if (s >= n) {
                                    kind = K_FALLBACK;
                                    fullwalk = true;
                                    break;
                                }
                                const int w = pw[pwb + pos];
                                ++st_probe;
                                if (w >= 0) {
                                    const int p = perm[w];
                                    int ix, o;
                                    const int c = conc_lookup(A, w, slot, &ix, &o);
                                    if (p >= mem || c >= 1) {
                                        kind = K_TARGET;
                                        tgt = w;
                                        pv = p;
                                        c0 = c;
                                        cidx = ix;
                                        ops0 = o;
                                        break;
                                    }
                                } else if (w == OWGS_PW_BADID) {
                                    kind = K_THROW;
                                    break;
                                }
                                pos = next_pos(pos, step, n);
                                ++s;
                            }
                        }
                    }
                    PT(3);
                    // frontier lane with a long walk: wave-cooperative scan, 64 walk steps per round
                    if (__builtin_amdgcn_readlane(kind, f) == K_LONG) {
                        ++st_long;
                        const CoopResult cr = coop_walk(A, perm, pw, f, s, pos, step, n, pwb, mem, maxc, slot);
                        if (lane == f) {
                            s = cr.s;
                            pos = cr.pos;
                            if (cr.kind == K_LONG) {
                                kind = K_FALLBACK;
                                fullwalk = true;
                            } else {
                                kind = cr.kind;
                                tgt = cr.tgt;
                                pv = cr.pv;
                                c0 = cr.c;
                                cidx = cr.cidx;
                                ops0 = cr.ops;
                            }
                        }
                    }
                    // fallback target (SCPB:417-424): H = usable pool members in pool order, r = H[rng(seq) mod |H|]
                    if (__ballot(act && kind == K_FALLBACK)) {
                        if (act && kind == K_FALLBACK) {
                            fallback_target(A, pool, i, n_slots, &kind, &tgt);
                            if (kind == K_FALLBACK && maxc > 1) c0 = conc_lookup(A, tgt, slot, &cidx, &ops0);
                        }
                    }
                    PT(4);
                    // ---------------------------------------------------- group by target / by fqn (slot key)
                    const bool part = act && (kind == K_TARGET || kind == K_FALLBACK);
                    const bool cpart = part && maxc > 1;
                    const u64 anyc = __ballot(cpart);
                    const uint32_t stamp = next_stamp(iter, stT, lane);
                    if (part) atomicMin(&stT[tgt & (OWGS_STAMP_BUCKETS - 1)], stamp);
                    if (cpart) atomicMin(&stS[slot & (OWGS_STAMP_BUCKETS - 1)], stamp);
                    wave_fence();
                    const bool leadT = part && stT[tgt & (OWGS_STAMP_BUCKETS - 1)] == stamp;
                    // q = earlier lanes of the same fqn at the same invoker; cons = memory this lane takes;
                    // E = memory taken at this lane's invoker by earlier lanes of the chunk
                    int E = 0;
                    cons = part ? mem : 0;
                    if (cpart) cons = c0 >= 1 ? 0 : mem;
                    u64 pend = __ballot(part && !leadT);
                    while (pend) {
                        ++st_grp;
                        const int j = ffs64(pend);
                        const int t = __builtin_amdgcn_readlane(tgt, j);
                        const u64 G = __ballot(part && tgt == t);
                        const bool in = (G >> lane) & 1;
                        u64 Cg = G & anyc;
                        while (Cg) {
                            const int j2 = ffs64(Cg);
                            const int sl = __builtin_amdgcn_readlane(slot, j2);
                            const u64 H = Cg & __ballot(slot == sl);
                            if ((H >> lane) & 1) {
                                q = __popcll(H & lt_mask);
                                cons = c_now_of(c0, q, maxc) >= 1 ? 0 : mem;
                            }
                            Cg &= ~H;
                        }
                        const int ex = wave_excl_scan(in ? cons : 0);
                        if (in) E = ex;
                        pend &= ~G;
                    }
                    room = pv - E;  // |pv|, E < 2^30 for any sane permit count
                    // an earlier lane of the same fqn on another walk, or an earlier forced acquire of the same fqn,
                    // may create concurrency slots this lane's speculation did not see -> uncertain
                    if (anyc) {
                        const bool leadS = cpart && stS[slot & (OWGS_STAMP_BUCKETS - 1)] == stamp;
                        pend = __ballot(cpart && !leadS);
                        while (pend) {
                            const int j = ffs64(pend);
                            const int sl = __builtin_amdgcn_readlane(slot, j);
                            const u64 Gs = __ballot(cpart && slot == sl);
                            const int a0 = __builtin_amdgcn_readlane(a, ffs64(Gs));
                            const u64 D = Gs & __ballot(a != a0);
                            const u64 FB = Gs & __ballot(kind == K_FALLBACK);
                            if ((Gs >> lane) & 1) {
                                const bool lower = (Gs & lt_mask) != 0;
                                if (kind == K_FALLBACK) unc = lower;
                                else
                                    unc = lower &&
                                          (((FB & lt_mask) != 0) || ((D & (lt_mask | self_bit)) != 0) || a < 0);
                            }
                            pend &= ~Gs;
                        }
                    }
                    PT(5);
                }
                // -------------------------------------------------------- decide
                const bool part = act && (kind == K_TARGET || kind == K_FALLBACK);
                bool ok = false, rej = false;
                if (act) {
                    if (kind == K_NONE || kind == K_THROW) {
                        ok = true;
                    } else if (kind == K_FALLBACK) {
                        ok = !(maxc > 1 && unc);
                    } else if (kind == K_TARGET) {
                        if (maxc == 1) {
                            ok = room >= mem;
                            rej = !ok;
                        } else if (!unc) {
                            ok = c_now_of(c0, q, maxc) >= 1 || room >= mem;
                            rej = !ok;
                        }
                    }
                }
                const u64 stop = __ballot(act && !ok);
                const int ls = stop ? ffs64(stop) : 64;
                const bool commit = act && lane < ls;

                // -------------------------------------------------------- commit lanes [f, l*)
                if (commit && part && cons > 0) atomicSub(&perm[tgt], mem);
                if (__ballot(commit && part && maxc > 1)) {
                    // concurrency map: the last committed lane of each (invoker, fqn) group writes the entry
                    const bool cpart = part && maxc > 1;
                    u64 W = __ballot(commit && cpart);
                    bool writer = false;
                    while (W) {
                        const int j = ffs64(W);
                        const int t = __builtin_amdgcn_readlane(tgt, j);
                        const int sl = __builtin_amdgcn_readlane(slot, j);
                        const u64 K = W & __ballot(tgt == t && slot == sl);
                        if (lane == fls64(K)) writer = true;
                        W &= ~K;
                    }
                    u64 ins = __ballot(writer && cidx < 0);
                    while (ins) {
                        const int j = ffs64(ins);
                        if (lane == j) {
                            cidx = ct_insert(A.ctab, A.ctab_mask, ct_key(tgt, slot));
                            if (cidx < 0) atomicOr(A.err, 1);
                        }
                        wave_fence();
                        ins &= ins - 1;
                    }
                    if (writer && cidx >= 0) {
                        const int cn = c_now_of(c0, q, maxc);
                        int c1;
                        if (cn >= 1) {
                            c1 = cn - 1;  // RS.tryAcquire(1)
                        } else {        // memory (try or force) + RS.release(maxConcurrent - 1, false)
                            const int next2 = cn + (maxc - 1);
                            c1 = (mod_small(next2, maxc) == 0) ? next2 - maxc : next2;
                        }
                        A.ctab[cidx] = ct_entry(ct_key(tgt, slot), c1, (ops0 > 0 ? ops0 : 0) + q + 1);
                    }
                }
                if (commit) {
                    A.out_inv[i] = kind == K_NONE ? OWGS_NONE_V : (kind == K_THROW ? OWGS_THROW_V : tgt);
                    A.out_flags[i] = (kind == K_FALLBACK) ? 1 : 0;
                    // cursors: steps before the committed target / after a full walk are infeasible from now on
                    if (cok && (kind == K_TARGET || (kind == K_FALLBACK && maxc == 1)))
                        atomicMax(&cur[a], kind == K_TARGET ? ((s << 16) | pos) : (n << 16));
                    pending = false;
                }
                const u64 fbm = __ballot(commit && kind == K_FALLBACK);
                if (fbm) {
                    st_fb += __popcll(fbm);
                    wave_fence();
                    if (commit && cok && kind == K_FALLBACK && maxc > 1) cur[a] = 0;  // forced slots: anywhere
                    // a failed full walk proves every usable pool member has permits < mem from now on
                    const bool t = commit && kind == K_FALLBACK && fullwalk && maxc == 1;
                    if (__ballot(t)) {
                        U0 = min(U0, wave_min(t && pool == 0 ? mem - 1 : 0x7FFFFFFF));
                        U1 = min(U1, wave_min(t && pool == 1 ? mem - 1 : 0x7FFFFFFF));
                    }
                }
                PT(6);
                if (ls == 64) break;

                // -------------------------------------------------------- resolve l*
                const int lk = __builtin_amdgcn_readlane(kind, ls);
                const int lmc = __builtin_amdgcn_readlane(maxc, ls);
                if (lmc == 1 && (lk == K_TARGET || lk == K_LONG)) {
                    // Incremental: l* is a maxConcurrent==1 lane and every lane before it is committed, so the
                    // state is exact at l*'s time.  Walk it to its true target, commit it, and patch the
                    // remaining permits (room) of later lanes at its old and new invokers; nothing else changed.
                    ++st_inc;
                    wave_fence();
                    const int lm = __builtin_amdgcn_readlane(mem, ls);
                    if (lk == K_TARGET) {
                        const int t_old = __builtin_amdgcn_readlane(tgt, ls);
                        if (act && lane > ls && tgt == t_old && (kind == K_TARGET || kind == K_FALLBACK)) room += lm;
                        if (lane == ls) {
                            pos = next_pos(pos, step, n);
                            ++s;
                        }
                    }
                    if (lane == ls && cok) {
                        const int cv = cur[a];
                        if ((cv >> 16) > s) {
                            s = cv >> 16;
                            pos = cv & 0xFFFF;
                        }
                    }
                    const int lpool = __builtin_amdgcn_readlane(pool, ls);
                    int nk, nt = -1, nfull = 0;
                    if (lm > (lpool ? U1 : U0) && ((A.shortcut_ok >> lpool) & 1)) {
                        nk = K_LONG;  // provably no feasible step: straight to the fallback
                    } else {
                        ++st_long;
                        const CoopResult cr = coop_walk(A, perm, pw, ls, s, pos, step, n, pwb, mem, 1, slot);
                        if (lane == ls) {
                            s = cr.s;
                            pos = cr.pos;
                        }
                        nk = cr.kind;
                        nt = cr.tgt;
                        nfull = 1;
                    }
                    if (nk == K_LONG) {  // every step fails: random fallback
                        int fk = K_NONE, ft = -1;
                        if (lane == ls) fallback_target(A, pool, i, n_slots, &fk, &ft);
                        nk = __builtin_amdgcn_readlane(fk, ls);
                        nt = __builtin_amdgcn_readlane(ft, ls);
                        if (nk == K_FALLBACK) {
                            ++st_fb;
                            if (nfull) {
                                if (lpool) U1 = min(U1, lm - 1);
                                else U0 = min(U0, lm - 1);
                            }
                        }
                    }
                    if (lane == ls) {
                        A.out_inv[i] = nk == K_NONE ? OWGS_NONE_V : (nk == K_THROW ? OWGS_THROW_V : nt);
                        A.out_flags[i] = (nk == K_FALLBACK) ? 1 : 0;
                        if (nk == K_TARGET || nk == K_FALLBACK) atomicSub(&perm[nt], lm);
                        if (cok && (nk == K_TARGET || nk == K_FALLBACK))
                            atomicMax(&cur[a], nk == K_TARGET ? ((s << 16) | pos) : (n << 16));
                        pending = false;
                    }
                    if ((nk == K_TARGET || nk == K_FALLBACK) && act && lane > ls && tgt == nt &&
                        (kind == K_TARGET || kind == K_FALLBACK))
                        room -= lm;
                    wave_fence();
                    f = ls + 1;
                } else {
                    // general case: l* (and every later lane of the same maxConcurrent==1 action speculated at the
                    // same walk step, when l* is a true rejection) continue past that step; re-speculate from l*
                    if (__builtin_amdgcn_readlane((int)rej, ls)) {
                        const int as = __builtin_amdgcn_readlane(a, ls);
                        const int ss = __builtin_amdgcn_readlane(s, ls);
                        bool adv = lane == ls;
                        if (as >= 0 && lmc == 1) adv = adv || (act && lane > ls && a == as && kind == K_TARGET && s == ss);
                        if (adv) {
                            pos = next_pos(pos, step, n);
                            ++s;
                        }
                        if (lane == ls && cok) atomicMax(&cur[a], (s << 16) | pos);
                    }
                    wave_fence();
                    f = ls;
                    full = true;
                }
            }
        }
        wave_fence();
    }

    for (int i = lane; i < n_slots; i += 64) A.permits[i] = perm[i];
    if (A.stats) {
        atomicAdd(&A.stats[1], (u64)st_probe);
        if (lane == 0) {
            atomicAdd(&A.stats[0], (u64)st_iter);
            atomicAdd(&A.stats[2], (u64)st_fb);
            atomicAdd(&A.stats[3], (u64)st_long);
            atomicAdd(&A.stats[4], (u64)st_grp);
            atomicAdd(&A.stats[5], (u64)st_inc);
#ifdef OWGS_PROFILE
            for (int k = 0; k < 8; ++k) atomicAdd(&A.stats[8 + k], pt_acc[k]);
#endif
        }
    }
}

// ------------------------------------------------------------------------------------------------ self-test
// DPP scan / reduction helpers against a serial computation (one wave per trial)
__global__ __launch_bounds__(64) void owgs_selftest_kernel(int* bad, int trials) {
    const int lane = threadIdx.x;
    for (int t = 0; t < trials; ++t) {
        const uint32_t h = ct_hash((uint32_t)(t * 64 + lane) * 2654435761u);
        const int v = (int)(h % 2001u) - 1000;
        const int inc = wave_incl_scan(v), exc = wave_excl_scan(v), mx = wave_max(v), mn = wave_min(v);
        int ref_inc = 0, ref_mx = (int)0x80000000, ref_mn = 0x7FFFFFFF;
        for (int j = 0; j < 64; ++j) {
            const int vj = __shfl(v, j, 64);
            if (j <= lane) ref_inc += vj;
            ref_mx = max(ref_mx, vj);
            ref_mn = min(ref_mn, vj);
        }
        if (inc != ref_inc || exc != ref_inc - v || mx != ref_mx || mn != ref_mn) atomicAdd(bad, 1);
    }
}

// ------------------------------------------------------------------------------------------------ launchers
extern "C" hipError_t owgs_launch_selftest(int* bad, int trials, hipStream_t s) {
    hipLaunchKernelGGL(owgs_selftest_kernel, dim3(1), dim3(64), 0, s, bad, trials);
    return hipGetLastError();
}

extern "C" hipError_t owgs_launch_hash(const OwgsHashArgs* a, hipStream_t s) {
    if (a->n <= 0) return hipSuccess;
    const int blocks = (a->n * 64 + 255) / 256;
    hipLaunchKernelGGL(owgs_hash_kernel, dim3(blocks), dim3(256), 0, s, *a);
    return hipGetLastError();
}

extern "C" hipError_t owgs_launch_gather(const OwgsGatherArgs* g, hipStream_t s) {
    const int64_t n = g->n_act > g->n_rel ? g->n_act : g->n_rel;
    if (n <= 0) return hipSuccess;
    const int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(owgs_gather_kernel, dim3((unsigned)(blocks < 2048 ? blocks : 2048)), dim3(256), 0, s, *g);
    return hipGetLastError();
}

extern "C" hipError_t owgs_launch_lookup(const OwgsLookupArgs* a, hipStream_t s) {
    if (a->n <= 0) return hipSuccess;
    hipLaunchKernelGGL(owgs_lookup_kernel, dim3((a->n + 255) / 256), dim3(256), 0, s, *a);
    return hipGetLastError();
}

extern "C" hipError_t owgs_launch_prepare(const OwgsPrepArgs* a, hipStream_t s) {
    if (a->n <= 0) return hipSuccess;
    hipLaunchKernelGGL(owgs_prepare_kernel, dim3((a->n + 255) / 256), dim3(256), 0, s, *a);
    return hipGetLastError();
}

extern "C" size_t owgs_engine_lds_bytes(int n_slots, int nm, int nb, int n_cursors) {
    return (size_t)(((n_slots + 3) & ~3) + ((nm + nb + 3) & ~3) + 2 * OWGS_STAMP_BUCKETS) * 4 +
           (size_t)((n_cursors + 3) & ~3) * 4;
}

extern "C" hipError_t owgs_launch_engine(const OwgsEngineArgs* a, hipStream_t s) {
    const size_t lds = owgs_engine_lds_bytes(a->n_slots, a->nm, a->nb, a->n_cursors);
    if (lds > OWGS_LDS_BYTES) return hipErrorInvalidValue;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)owgs_engine_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, OWGS_LDS_BYTES);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    hipLaunchKernelGGL(owgs_engine_kernel, dim3(1), dim3(64), lds, s, *a);
    return hipGetLastError();
}
