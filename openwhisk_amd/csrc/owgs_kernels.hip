// owgs_kernels.hip -- CDNA4 (gfx950) kernels of the batched invoker scheduler.
//
// Kernels
//   owgs_hash_kernel     java.lang.String.hashCode of many strings, one wave per string: lane i sums
//                        c[i + 64k] * 31^(L-1-i-64k) (mod 2^32) and the wave reduces (SCPB:370-372 call site).
//   owgs_prepare_kernel  per action: generateHash combine, home = hash % n, step = stepSizes(hash % k),
//                        meta bits (SCPB:262-268).
//   owgs_engine_kernel   the hot path: releases (SCPB:327-331 -> NS:98-113) and schedule() (SCPB:398-436 with
//                        NS:32-91) for a whole stream of batches, replaying the reference's SEQUENTIAL semantics.
//
// Engine design (DESIGN.md "Engine"): one wavefront owns one controller shard.  The slot permits and the pool
// vectors live in LDS for the whole stream (HBM is read once and written once).  Activations are taken 64 at a
// time (one per lane, in stream order).  Every lane speculates its walk target against the current state, which is
// the exact state at the chunk frontier f.  Because memory permits never increase inside a batch (releases happen
// only at batch boundaries), a probe that fails against an earlier state fails at every later time, so the
// speculated target is never EARLIER than the true one.  It is exactly the true one iff the permits consumed at that
// invoker by earlier lanes of the chunk still leave room: lanes are grouped by target (LDS stamp table + ballot),
// an exclusive prefix sum of the consumed memory inside each group gives every lane its remaining permits, and the
// first lane l* that does not fit is a TRUE rejection (every earlier lane fitted, so the prefix it saw is exact).
// Lanes [f, l*) are committed, l* advances its walk, and the chunk iterates with f = l*.  Concurrency slots (maxConc
// > 1) can increase when an earlier lane of the same action starts a container, so a lane with an earlier
// same-action lane in [f, lane) is treated as uncertain and resolved once it is the frontier.
#include <hip/hip_runtime.h>

#include "owgs_internal.h"

typedef unsigned long long u64;

#define K_NONE 0
#define K_THROW 1
#define K_TARGET 2
#define K_FALLBACK 3
#define K_LONG 4

#define KPROBE 4

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

__device__ __forceinline__ int jmod_step(int pos, int step, int n) {
    return (int)((int)((unsigned)pos + (unsigned)step) % n);  // Java (index + step) % numInvokers
}

__device__ __forceinline__ int ffs64(u64 m) { return __ffsll((long long)m) - 1; }

__device__ __forceinline__ int wave_excl_scan(int v) {
    const int lane = __lane_id();
    int x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        int y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x - v;
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, __shfl_xor(v, d, 64));
    return v;
}

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = min(v, __shfl_xor(v, d, 64));
    return v;
}

__device__ __forceinline__ uint32_t ctab_hash(u64 k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return (uint32_t)k;
}

__device__ __forceinline__ u64 ctab_keyof(int inv, int slot) { return ((u64)(uint32_t)(inv + 1) << 32) | (uint32_t)slot; }

__device__ int ctab_find(const u64* keys, uint32_t mask, u64 key) {
    uint32_t h = ctab_hash(key) & mask;
    for (uint32_t p = 0; p <= mask; ++p) {
        u64 k = keys[h];
        if (k == key) return (int)h;
        if (k == 0) return -1;
        h = (h + 1) & mask;
    }
    return -1;
}

__device__ int ctab_insert(u64* keys, uint32_t mask, u64 key) {
    uint32_t h = ctab_hash(key) & mask;
    for (uint32_t p = 0; p <= mask; ++p) {
        u64 k = keys[h];
        if (k == key) return (int)h;
        if (k == 0) {
            keys[h] = key;
            return (int)h;
        }
        h = (h + 1) & mask;
    }
    return -1;
}

// c of NestedSemaphore(inv).actionConcurrentSlotsMap(slot); absent entries (operationCount 0) read as c = 0
__device__ __forceinline__ int conc_c(const OwgsEngineArgs& A, int inv, int slot, int* eidx) {
    int e = ctab_find(A.ctab_key, A.ctab_mask, ctab_keyof(inv, slot));
    *eidx = e;
    if (e < 0) return 0;
    int2 v = A.ctab_val[e];
    return v.y > 0 ? v.x : 0;
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
    const int e = ctab_find(a.ctab_key, a.ctab_mask, ctab_keyof(a.inv[i], a.slot[i]));
    a.out[i] = e < 0 ? make_int2(0, 0) : a.ctab_val[e];
}

// generateHash combine + home/step selection (SCPB:266-268)
__global__ __launch_bounds__(256) void owgs_prepare_kernel(OwgsPrepArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const int pool = a.bb[i] ? 1 : 0;
    const int n = pool ? a.nb : a.nm;
    const int k = pool ? a.n_bsteps : a.n_msteps;
    const int32_t* steps = pool ? a.bsteps : a.msteps;
    uint32_t meta = (uint32_t)(a.maxc[i] & OWGS_META_MAXC_MASK) | ((uint32_t)pool << OWGS_META_POOL_SHIFT);
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
        else step = steps[si];
    }
    a.act_info[i] = make_int4(home, step, a.mem[i], (int)meta);
}

// ------------------------------------------------------------------------------------------------ engine
struct Lds {
    int32_t* perm;
    int32_t* pw;
    uint32_t* stT;
    uint32_t* stS;
};

// fallback target (SCPB:417-424): H = usable pool members in pool order, r = H[rng(seq) mod |H|]
__device__ __forceinline__ void fallback_target(const OwgsEngineArgs& A, int pool, u64 seq, int* kind, int* tgt) {
    const int hc = pool ? A.hb : A.hm;
    if (hc <= 0) {
        *kind = K_NONE;
        return;
    }
    const int r = A.hlist[(pool ? A.hm : 0) + (int)rng_index(A.rng_seed, seq, (uint32_t)hc)];
    if (r < 0 || r >= A.n_slots) {
        *kind = K_THROW;
        return;
    }
    *kind = K_FALLBACK;
    *tgt = r;
}

__global__ __launch_bounds__(64) void owgs_engine_kernel(OwgsEngineArgs A) {
    extern __shared__ __attribute__((aligned(16))) int32_t lds_raw[];
    const int lane = threadIdx.x;
    const int nsl_al = (A.n_slots + 3) & ~3;
    const int npw_al = (A.nm + A.nb + 3) & ~3;
    Lds L;
    L.perm = lds_raw;
    L.pw = lds_raw + nsl_al;
    L.stT = (uint32_t*)(L.pw + npw_al);
    L.stS = L.stT + OWGS_STAMP_BUCKETS;

    for (int i = lane; i < A.n_slots; i += 64) L.perm[i] = A.permits[i];
    for (int i = lane; i < A.nm + A.nb; i += 64) L.pw[i] = A.pool_words[i];
    for (int i = lane; i < 2 * OWGS_STAMP_BUCKETS; i += 64) L.stT[i] = 0xFFFFFFFFu;
    __syncthreads();

    u64 st_iter = 0, st_probe = 0, st_fb = 0, st_long = 0, st_grp = 0;
    uint32_t iter = 0;
    const u64 lt_mask = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));

    for (int b = 0; b < A.n_batches; ++b) {
        // ================================================================ releases (SCPB:327-331)
        const int64_t r_beg = A.rel_off ? A.rel_off[b] : 0, r_end = A.rel_off ? A.rel_off[b + 1] : 0;
        for (int64_t r0 = r_beg; r0 < r_end; r0 += 64) {
            const int64_t r = r0 + lane;
            const bool valid = r < r_end;
            int inv = -1, a = 0;
            if (valid) {
                if (A.rel_inv) {
                    inv = A.rel_inv[r];
                    a = A.rel_act[r];
                } else {
                    const int64_t aid = A.rel_aid[r];
                    inv = A.out_inv[aid];
                    a = A.act[aid];
                }
            }
            int mem = 0, maxc = 1, slot = 0;
            if (valid) {
                const int4 info = A.act_info[a];
                mem = info.z;
                maxc = info.w & OWGS_META_MAXC_MASK;
                slot = A.act_slot[a];
            }
            uint8_t flag = 0;
            bool simple = false, conc = false;
            if (valid) {
                if (inv < 0) flag = OWGS_REL_NOENTRY_BIT;
                else if (inv >= A.n_slots) flag = 0;  // invokerSlots.lift -> no-op
                else if (maxc == 1) simple = true;
                else conc = true;
            }
            int eidx = -1;
            if (conc) {
                eidx = ctab_find(A.ctab_key, A.ctab_mask, ctab_keyof(inv, slot));
                int2 v = eidx >= 0 ? A.ctab_val[eidx] : make_int2(0, 0);
                if (eidx < 0 || v.y <= 0) {
                    conc = false;
                    flag = OWGS_REL_NOSUCH_BIT;  // actionConcurrentSlotsMap(actionid) throws NS:103
                }
            }
            // group concurrent releases of the same entry: rank in stream order, group size
            int rank = 0, gsz = 1;
            {
                ++iter;
                const uint32_t stamp = ((0x03FFFFFFu - (iter & 0x03FFFFFFu)) << 6) | (uint32_t)lane;
                if (conc) atomicMin(&L.stT[eidx & (OWGS_STAMP_BUCKETS - 1)], stamp);
                __syncthreads();
                const bool leader = conc && L.stT[eidx & (OWGS_STAMP_BUCKETS - 1)] == stamp;
                u64 pend = __ballot(conc && !leader);
                while (pend) {
                    const int j = ffs64(pend);
                    const int e = __builtin_amdgcn_readlane(eidx, j);
                    const u64 G = __ballot(conc && eidx == e);
                    if ((G >> lane) & 1) {
                        rank = __popcll(G & lt_mask);
                        gsz = __popcll(G);
                    }
                    pend &= ~G;
                }
            }
            bool mem_rel = false;
            int2 v0 = make_int2(0, 0);
            if (conc) v0 = A.ctab_val[eidx];
            if (conc) {
                // NS:98-113 / RS:99-108 applied rank+1 times to (c0, ops0), R = maxConcurrent
                const int c0 = v0.x, o = v0.y;
                if (rank < o) {
                    mem_rel = ((c0 + rank + 1) % maxc) == 0;
                } else {
                    flag = OWGS_REL_NOSUCH_BIT;  // entry already removed by an earlier release of this batch
                }
            }
            __syncthreads();
            if (conc && rank == 0) {
                const int c0 = v0.x, o = v0.y;
                const int j = min(gsz, o);
                int c1 = (c0 + j) % maxc;
                const int o1 = o - j;
                if (o1 == 0) c1 = 0;  // actionRelease: entry removed (NS:109-111)
                A.ctab_val[eidx] = make_int2(c1, o1);
            }
            if (simple || mem_rel) {
                const int old = atomicAdd(&L.perm[inv], mem);
                if (old > 0x7FFFFFFF - mem) {  // ForcibleSemaphore overflow -> Error, state unchanged (FS:48-50)
                    atomicSub(&L.perm[inv], mem);
                    flag |= OWGS_REL_OVERFLOW_BIT;
                }
            }
            if (valid && A.rel_flags) A.rel_flags[r] = flag;
            __threadfence_block();
            __syncthreads();
        }

        // ================================================================ per-batch pool bounds
        // U[p] >= max permits over usable members of pool p; permits only fall until the next batch.
        int U[2];
        for (int p = 0; p < 2; ++p) {
            const int base = p ? A.nm : 0, n = p ? A.nb : A.nm;
            int m = (int)0x80000000;
            for (int i = lane; i < n; i += 64) {
                const int w = L.pw[base + i];
                if (w >= 0) m = max(m, L.perm[w]);
            }
            U[p] = wave_max(m);
        }

        // ================================================================ acquires (SCPB:398-436)
        const int64_t a_beg = A.acq_off[b], a_end = A.acq_off[b + 1];
        for (int64_t c0 = a_beg; c0 < a_end; c0 += 64) {
            const int64_t i = c0 + lane;
            bool pending = i < a_end;
            int home = 0, step = 0, mem = 0, meta = 0, slot = 0;
            if (pending) {
                int4 info;
                if (A.xw_info) {
                    info = A.xw_info[i];
                    slot = A.xw_slot[i];
                } else {
                    const int a = A.act[i];
                    info = A.act_info[a];
                    slot = A.act_slot[a];
                }
                home = info.x;
                step = info.y;
                mem = info.z;
                meta = info.w;
            }
            const u64 seq = A.seq ? A.seq[i < a_end ? i : a_beg] : (A.seq_base + (u64)i);
            const int maxc = meta & OWGS_META_MAXC_MASK;
            const int pool = (meta >> OWGS_META_POOL_SHIFT) & 1;
            const int n = pool ? A.nb : A.nm;
            const int pwb = pool ? A.nm : 0;
            int pos = home, s = 0;
            int out_kind = K_NONE, out_tgt = -1;
            bool fullwalk = false;

            if (pending) {
                if (meta & OWGS_META_EMPTY) {
                    out_kind = K_NONE;
                    pending = false;
                } else if ((meta & OWGS_META_THROW) || home < 0 || home >= n || step < 0) {
                    out_kind = K_THROW;
                    pending = false;
                }
                if (!pending) {
                    A.out_inv[i] = out_kind == K_NONE ? OWGS_NONE_V : OWGS_THROW_V;
                    A.out_flags[i] = 0;
                }
            }

            int f = 0;
            while (__ballot(pending)) {
                ++st_iter;
                // -------------------------------------------------------- speculate targets
                int kind = K_NONE, tgt = -1, cval = 0, eidx = -1;
                const bool act = pending && lane >= f;
                if (act) {
                    if (maxc == 1 && mem > U[pool] && ((A.shortcut_ok >> pool) & 1)) {
                        fallback_target(A, pool, seq, &kind, &tgt);
                        fullwalk = false;
                    } else {
                        kind = K_LONG;
                        for (int k = 0; k < KPROBE; ++k) {
                            if (s >= n) {  // every pool position probed: the n+2-probe walk fails (SCPB:417)
                                fallback_target(A, pool, seq, &kind, &tgt);
                                fullwalk = true;
                                break;
                            }
                            if (pos < 0 || pos >= n) {
                                kind = K_THROW;
                                break;
                            }
                            const int w = L.pw[pwb + pos];
                            ++st_probe;
                            if (w == OWGS_PW_BADID) {
                                kind = K_THROW;
                                break;
                            }
                            if (w >= 0) {
                                bool feas = L.perm[w] >= mem;
                                if (maxc > 1) {
                                    int e;
                                    const int c = conc_c(A, w, slot, &e);
                                    if (c >= 1) feas = true;
                                    if (feas) {
                                        cval = c;
                                        eidx = e;
                                    }
                                }
                                if (feas) {
                                    kind = K_TARGET;
                                    tgt = w;
                                    break;
                                }
                            }
                            pos = jmod_step(pos, step, n);
                            ++s;
                        }
                    }
                }
                // -------------------------------------------------------- frontier lane with a long walk:
                // wave-cooperative scan of 64 walk positions per step (ballot picks the first feasible one)
                const int kf = __builtin_amdgcn_readlane(kind, f);
                if (kf == K_LONG) {
                    ++st_long;
                    int p0 = __builtin_amdgcn_readlane(pos, f);
                    int s0 = __builtin_amdgcn_readlane(s, f);
                    const int stp = __builtin_amdgcn_readlane(step, f);
                    const int nn = __builtin_amdgcn_readlane(n, f);
                    const int pb = __builtin_amdgcn_readlane(pwb, f);
                    const int m = __builtin_amdgcn_readlane(mem, f);
                    const int mc = __builtin_amdgcn_readlane(maxc, f);
                    const int sl = __builtin_amdgcn_readlane(slot, f);
                    int fk = K_LONG, ft = -1, fpos = p0, fs = s0, fc = 0, fe = -1;
                    while (s0 < nn) {
                        const int sk = s0 + lane;
                        const int p = (int)(((long long)p0 + (long long)lane * (long long)stp) % (long long)nn);
                        bool feas = false;
                        int w = -1, c = 0, e = -1;
                        if (sk < nn) {
                            w = L.pw[pb + p];
                            if (w == OWGS_PW_BADID) {
                                feas = true;
                            } else if (w >= 0) {
                                feas = L.perm[w] >= m;
                                if (mc > 1) {
                                    c = conc_c(A, w, sl, &e);
                                    if (c >= 1) feas = true;
                                }
                            }
                        }
                        st_probe += (sk < nn);
                        const u64 fm = __ballot(feas);
                        if (fm) {
                            const int j = ffs64(fm);
                            ft = __builtin_amdgcn_readlane(w, j);
                            fpos = __builtin_amdgcn_readlane(p, j);
                            fc = __builtin_amdgcn_readlane(c, j);
                            fe = __builtin_amdgcn_readlane(e, j);
                            fs = s0 + j;
                            fk = (ft == OWGS_PW_BADID) ? K_THROW : K_TARGET;
                            break;
                        }
                        s0 += 64;
                        p0 = (int)(((long long)p0 + 64ll * (long long)stp) % (long long)nn);
                    }
                    if (lane == f) {
                        if (fk == K_LONG) {
                            s = nn;
                            fallback_target(A, pool, seq, &kind, &tgt);
                            fullwalk = true;
                        } else {
                            kind = fk;
                            tgt = ft;
                            pos = fpos;
                            s = fs;
                            cval = fc;
                            eidx = fe;
                        }
                    }
                }
                if (act && kind == K_FALLBACK && maxc > 1) {
                    int e;
                    cval = conc_c(A, tgt, slot, &e);
                    eidx = e;
                }
                // -------------------------------------------------------- conflict groups
                const bool part = act && (kind == K_TARGET || kind == K_FALLBACK);
                const int cons = part ? ((kind == K_TARGET && maxc > 1 && cval >= 1) ? 0 : mem) : 0;
                const bool cpart = part && maxc > 1;
                ++iter;
                if ((iter & 0x03FFFFFFu) == 0) {
                    for (int t = lane; t < 2 * OWGS_STAMP_BUCKETS; t += 64) L.stT[t] = 0xFFFFFFFFu;
                    __syncthreads();
                    ++iter;
                }
                const uint32_t stamp = ((0x03FFFFFFu - (iter & 0x03FFFFFFu)) << 6) | (uint32_t)lane;
                if (part) atomicMin(&L.stT[tgt & (OWGS_STAMP_BUCKETS - 1)], stamp);
                if (cpart) atomicMin(&L.stS[slot & (OWGS_STAMP_BUCKETS - 1)], stamp);
                __syncthreads();
                const bool leadT = part && L.stT[tgt & (OWGS_STAMP_BUCKETS - 1)] == stamp;
                const bool leadS = cpart && L.stS[slot & (OWGS_STAMP_BUCKETS - 1)] == stamp;
                int E = 0;
                u64 pend = __ballot(part && !leadT);
                while (pend) {
                    ++st_grp;
                    const int j = ffs64(pend);
                    const int t = __builtin_amdgcn_readlane(tgt, j);
                    const u64 G = __ballot(part && tgt == t);
                    const bool in = (G >> lane) & 1;
                    const int ex = wave_excl_scan(in ? cons : 0);
                    if (in) E = ex;
                    pend &= ~G;
                }
                bool ssl = false;  // an earlier lane of this chunk may change this action's concurrency slots
                pend = __ballot(cpart && !leadS);
                while (pend) {
                    const int j = ffs64(pend);
                    const int sl = __builtin_amdgcn_readlane(slot, j);
                    const u64 G = __ballot(cpart && slot == sl);
                    if (((G >> lane) & 1) && (G & lt_mask)) ssl = true;
                    pend &= ~G;
                }
                // -------------------------------------------------------- decide
                bool ok = false, rej = false;
                if (act) {
                    if (kind == K_NONE || kind == K_THROW) {
                        ok = true;
                    } else if (kind == K_FALLBACK) {
                        ok = !(maxc > 1 && ssl);
                    } else if (kind == K_TARGET) {
                        const long long room = (long long)L.perm[tgt] - (long long)E;
                        if (maxc == 1) {
                            ok = room >= mem;
                            rej = !ok;
                        } else if (!ssl) {
                            ok = (cval >= 1) || room >= mem;
                            rej = !ok;
                        }
                    }
                }
                const u64 stop = __ballot(act && !ok);
                const int ls = stop ? ffs64(stop) : 64;
                const bool commit = act && lane < ls;
                // -------------------------------------------------------- commit lanes [f, l*)
                if (commit && part && maxc == 1) atomicSub(&L.perm[tgt], mem);
                if (commit && part && maxc > 1) {
                    // NS:63-81: concurrency slot if available, else memory (try or force) + release(maxConc-1)
                    if (cons > 0) atomicSub(&L.perm[tgt], mem);
                }
                {
                    u64 ins = __ballot(commit && part && maxc > 1 && eidx < 0);
                    while (ins) {
                        const int j = ffs64(ins);
                        if (lane == j) {
                            eidx = ctab_insert(A.ctab_key, A.ctab_mask, ctab_keyof(tgt, slot));
                            if (eidx < 0) atomicOr(A.err, 1);
                            else A.ctab_val[eidx] = make_int2(0, 0);
                        }
                        __threadfence_block();
                        ins &= ins - 1;
                    }
                }
                if (commit && part && maxc > 1 && eidx >= 0) {
                    int2 v = A.ctab_val[eidx];
                    int c = v.y > 0 ? v.x : 0, o = v.y > 0 ? v.y : 0;
                    if (c >= 1) {
                        c -= 1;
                    } else {
                        const int next2 = c + (maxc - 1);
                        c = (next2 % maxc == 0) ? next2 - maxc : next2;
                    }
                    o += 1;
                    A.ctab_val[eidx] = make_int2(c, o);
                }
                if (commit) {
                    int oi;
                    if (kind == K_NONE) oi = OWGS_NONE_V;
                    else if (kind == K_THROW) oi = OWGS_THROW_V;
                    else oi = tgt;
                    A.out_inv[i] = oi;
                    A.out_flags[i] = (kind == K_FALLBACK) ? 1 : 0;
                    if (kind == K_FALLBACK) ++st_fb;
                }
                // a failed full walk proves every usable pool member has permits < mem from now on
                for (int p = 0; p < 2; ++p) {
                    const bool t = commit && kind == K_FALLBACK && fullwalk && maxc == 1 && pool == p;
                    const int mm = wave_min(t ? mem - 1 : 0x7FFFFFFF);
                    U[p] = min(U[p], mm);
                }
                if (commit) pending = false;
                if (lane == ls && rej) {  // true rejection at tgt: continue the walk past it
                    pos = jmod_step(pos, step, n);
                    ++s;
                }
                __threadfence_block();
                __syncthreads();
                f = ls;
            }
        }
        __threadfence_block();
        __syncthreads();
    }

    for (int i = lane; i < A.n_slots; i += 64) A.permits[i] = L.perm[i];
    if (A.stats) {
        // each lane counted its own probes; lane-uniform counters are identical in every lane
        atomicAdd(&A.stats[1], st_probe);
        if (lane == 0) {
            atomicAdd(&A.stats[0], st_iter);
            atomicAdd(&A.stats[2], st_fb);
            atomicAdd(&A.stats[3], st_long);
            atomicAdd(&A.stats[4], st_grp);
        }
    }
}

// ------------------------------------------------------------------------------------------------ launchers
extern "C" hipError_t owgs_launch_hash(const OwgsHashArgs* a, hipStream_t s) {
    if (a->n <= 0) return hipSuccess;
    const int blocks = (a->n * 64 + 255) / 256;
    hipLaunchKernelGGL(owgs_hash_kernel, dim3(blocks), dim3(256), 0, s, *a);
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

extern "C" size_t owgs_engine_lds_bytes(int n_slots, int nm, int nb) {
    return (size_t)(((n_slots + 3) & ~3) + ((nm + nb + 3) & ~3) + 2 * OWGS_STAMP_BUCKETS) * 4;
}

extern "C" hipError_t owgs_launch_engine(const OwgsEngineArgs* a, hipStream_t s) {
    const size_t lds = owgs_engine_lds_bytes(a->n_slots, a->nm, a->nb);
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
