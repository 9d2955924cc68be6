// owgs_resident.hip -- the JVM shim's path (owgs_process_batch) served by a resident engine.
//
// A drained batch of the shim's queue is small (tens to hundreds of jobs), so a launch chain per call pays more for
// itself -- launches, copies, loading and storing the slot image -- than for the decisions (BENCH shim_path, DESIGN.md
// section 5.6).  The resident engine is ONE workgroup that loads a controller shard's slot state (ForcibleSemaphore
// permits with the usable bit folded in, the usable bitmap and its prefix counts, the NestedSemaphore map's primary
// table) into LDS once and then serves calls through a control block in pinned, coherent host memory: the host writes
// the call (runs of completions then publishes, in queue order) and rings a doorbell; the engine stages the inputs into
// LDS, replays the runs, writes decisions, overload flags and release flags straight into pinned host memory and
// answers.  No launch, no copy and no stream synchronisation per call.  It writes the state back and exits on a stop
// word, or by itself after idle_ticks without a call (the host relaunches it on the next call), so every launch ends.
//
// Decisions are exact and sequential, one activation at a time in stream order: wave 0 walks 64 probes per round
// (home, home + step, ... mod n, SCPB:398-436) with one LDS read of the permits each (and, for concurrent actions, the
// key's entry of the map: NestedSemaphore.tryAcquireConcurrent, NS:57-82), takes the first probe whose invoker can
// take the activation, or -- after every pool position failed -- forces the counter-RNG's healthy invoker (SCPB:417-
// 424, forceAcquireConcurrent NS:84-91).  Releases: maxConcurrent == 1 ones are permit adds (ForcibleSemaphore.release,
// FS:117-120; order-free, the call is refused before anything is applied when one could leave the LDS range),
// concurrent ones RS.release(1, true) on their entry in queue order (NS:98-113).  Identity pools, no watched pairs:
// the host routes every other call to the chained path (owgs_host.cpp, res_eligible).
#include <hip/hip_runtime.h>

#include "owgs_internal.h"
#include "owgs_table.h"

typedef unsigned long long u64;

namespace {

__device__ __forceinline__ int ld_sys(const int32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(int32_t* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ u64 splitmix64(u64 x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
// counter RNG replacing ThreadLocalRandom.nextInt(|H|) (SCPB:421): the engine's and the oracle's
__device__ __forceinline__ uint32_t rng_index(u64 seed, u64 seq, uint32_t n) {
    const u64 u = splitmix64(seed ^ (seq * 0x9E3779B97F4A7C15ULL)) >> 32;
    return (uint32_t)((u * (u64)n) >> 32);
}
__device__ __forceinline__ int ffs64(u64 m) { return __ffsll((long long)m) - 1; }
// x mod n for 0 <= x < 2^31, 1 <= n < 2^15 (float reciprocal, exact correction)
__device__ __forceinline__ int mod_fast(int x, int n, float rn) {
    const int q = (int)((float)x * rn);
    int r = x - q * n;
    r += r < 0 ? n : 0;
    r += r < 0 ? n : 0;
    r -= r >= n ? n : 0;
    r -= r >= n ? n : 0;
    return r;
}
// position of the need-th set bit of m (need < popc(m))
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

struct ResLayout {
    uint32_t P, ub, pc, ct, sc, stage, end;
};
__host__ __device__ inline ResLayout res_layout(int n_slots, int n_ids) {
    const uint32_t words = (uint32_t)(n_ids + 31) / 32;
    ResLayout y;
    y.P = 0;
    y.ub = y.P + (((uint32_t)n_slots + 3u) & ~3u) * 4u;
    y.pc = y.ub + ((words + 4u) & ~3u) * 4u;
    y.ct = y.pc + ((words + 2u + 3u) & ~3u) * 4u;
    y.sc = y.ct + OWGS_CTC * 8u;
    y.stage = y.sc + 64u * 4u;
    y.end = y.stage;
    return y;
}

// LDS scalars
#define RS_USED 0    // primary entries (live + deleted)
#define RS_OVF 1     // overflow entries (live + deleted)
#define RS_K 2       // the call being served (-1: exit)
#define RS_MAXP 3    // upper bound of every slot's plain permits (release range check)
#define RS_ERR 4
#define RS_LIVE 5    // cleanup: live primary entries
#define RS_BAIL 6
#define RS_RSUM 8    // (u64, 8-aligned) memory the call's releases return at most

// primary table (LDS, interleaved {key, value}): index of key or -1, *val (0 if absent); chains end at an empty entry
__device__ __forceinline__ int ct_lookup(const uint2* ct, uint32_t key, uint32_t* val) {
    uint32_t h = ct_home(key);
    *val = 0u;
    for (int p = 0; p < OWGS_CTC / CT_BLK; ++p) {
        const uint4 e01 = *(const uint4*)&ct[h];
        const uint4 e23 = *(const uint4*)&ct[h + 2];
        const bool h0 = e01.x == key, h1 = e01.z == key, h2 = e23.x == key, h3 = e23.z == key;
        if (h0 || h1 || h2 || h3) {
            *val = h0 ? e01.y : h1 ? e01.w : h2 ? e23.y : e23.w;
            return (int)h + (h0 ? 0 : h1 ? 1 : h2 ? 2 : 3);
        }
        if (e01.x == 0u || e01.z == 0u || e23.x == 0u || e23.z == 0u) return -1;
        h = (h + CT_BLK) & (OWGS_CTC - 1);
    }
    return -1;
}
// both tables: index < OWGS_CTC primary, OWGS_CTC + j overflow entry j
__device__ __forceinline__ int ct_lookup2(const uint2* ct, const OwgsOvf& O, bool ovf_on, uint32_t key, uint32_t* val) {
    int i = ct_lookup(ct, key, val);
    if (i < 0 && ovf_on) {
        const int j = ovf_find(O, key, val);
        i = j >= 0 ? OWGS_CTC + j : -1;
    }
    return i;
}

}  // namespace

// One workgroup of 256 threads; wave 0 decides, every wave loads, stages and writes back.
__global__ __launch_bounds__(256, 1) void owgs_resident_kernel(OwgsResArgs A) {
    extern __shared__ uint4 lds_raw[];
    char* Lb = (char*)lds_raw;
    const ResLayout Y = res_layout(A.n_slots, A.n_ids);
    int32_t* P = (int32_t*)(Lb + Y.P);
    uint32_t* ub = (uint32_t*)(Lb + Y.ub);
    uint32_t* pc = (uint32_t*)(Lb + Y.pc);
    uint2* ct = (uint2*)(Lb + Y.ct);
    int32_t* sc = (int32_t*)(Lb + Y.sc);
    char* stg = Lb + Y.stage;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int n_slots = A.n_slots, nm = A.nm, nb = A.nb;
    const int words = (A.n_ids + 31) >> 5;

    // ------------------------------------------------------------------ state -> LDS (once per launch)
    if (tid < 16) sc[tid] = 0;
    __syncthreads();
    {
        int used = 0, mx = (int)0x80000000, e = 0;
        for (int i = tid; i < n_slots; i += 256) {
            const int v = A.permits[i];
            const bool unusable = !(i < A.n_ids && ((A.usable[i >> 5] >> (i & 31)) & 1u));
            if (v < -OWGS_PLIM || v >= OWGS_PLIM) e |= OWGS_ERR_PERMITS;
            P[i] = unusable ? v + OWGS_PENC : v;
            mx = max(mx, v);
        }
        for (int i = tid; i <= words; i += 256) ub[i] = i < words ? A.usable[i] : 0u;
        for (int i = tid; i < OWGS_CTC; i += 256) {
            const uint32_t k = A.ct_keys[i];
            ct[i] = make_uint2(k, A.ct_vals[i]);
            used += k != 0u;
        }
        if (used) atomicAdd(&sc[RS_USED], used);
        atomicMax(&sc[RS_MAXP], mx);
        if (e) atomicOr(&sc[RS_ERR], e);
        if (tid == 0 && A.ovf.cap > 0)
            sc[RS_OVF] = __hip_atomic_load(A.ovf.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (wave == 0) {  // prefix counts of the usable bitmap
        int carry = 0;
        for (int w0 = 0; w0 <= words; w0 += 64) {
            const int w = w0 + lane;
            const int c = w < words ? __popc(ub[w]) : 0;
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
    // healthy invokers per pool (|H| of the fallback, SCPB:417-424) and whether every id of a pool is usable
    auto usable_before = [&](int x) -> int {
        if (x <= 0) return 0;
        const int w = x >> 5, b = x & 31;
        return (int)pc[w] + (b ? __popc(ub[w] & ((1u << b) - 1u)) : 0);
    };
    const int hm_e = usable_before(nm), hb_e = usable_before(A.n_ids) - usable_before(A.n_ids - nb);
    const bool full_m = hm_e == nm, full_b = hb_e == nb;
    auto select_usable = [&](int lo, int k) {  // k-th usable id at or after id lo
        const int target = usable_before(lo) + k;
        int a = lo >> 5, z = (A.n_ids - 1) >> 5;
        while (a < z) {
            const int mid = (a + z + 1) >> 1;
            if ((int)pc[mid] <= target) a = mid;
            else z = mid - 1;
        }
        const uint32_t m = ub[a];
        const int need = target - (int)pc[a];
        if (need < 0 || need >= __popc(m)) return -1;
        return (a << 5) + select_in_word(m, need);
    };
    if (tid == 0) st_sys(&A.ctl[OWGS_RES_STATE], 1);

    // ------------------------------------------------------------------ calls
    int last = A.last_call;
    u64 t_idle = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (tid == 0) {
            int k = last;
            bool stop = false;
            for (long long spin = 0;; ++spin) {
                k = ld_sys(&A.ctl[OWGS_RES_BELL]);
                if (k != last) break;
                const u64 now = __builtin_amdgcn_s_memrealtime();
                if ((long long)(now - t_idle) > A.idle_ticks || spin > (1ll << 32)) {
                    stop = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(4);
            }
            sc[RS_K] = stop ? -1 : k;
        }
        __syncthreads();
        const int k = sc[RS_K];
        if (k < 0) break;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the host's inputs, written before the bell
        const int32_t* H = A.ctl + OWGS_RES_HDR;
        const int n_runs = ld_sys(H + 0), NR = ld_sys(H + 1), NP = ld_sys(H + 2), has_seq = ld_sys(H + 3);
        const u64 seq_base = (u64)(uint32_t)ld_sys(H + 4) | ((u64)(uint32_t)ld_sys(H + 5) << 32);
        const int i_roff = ld_sys(H + 6), i_poff = ld_sys(H + 7), i_rinv = ld_sys(H + 8), i_ract = ld_sys(H + 9),
                  i_pact = ld_sys(H + 10), i_seq = ld_sys(H + 11);
        const int o_inv = ld_sys(H + 12), o_fl = ld_sys(H + 13), o_rfl = ld_sys(H + 14);
        // staging: run offsets, releases {inv, meta.y, slot, -}, publishes {meta.x, meta.y, slot, -}, sequence numbers
        const uint32_t s_roff = 0, s_poff = s_roff + (((uint32_t)n_runs + 4u) & ~3u) * 4u;
        const uint32_t s_rel = s_poff + (((uint32_t)n_runs + 4u) & ~3u) * 4u;
        const uint32_t s_pub = s_rel + (uint32_t)NR * 16u, s_seq = s_pub + (uint32_t)NP * 16u;
        const uint32_t s_end = s_seq + (has_seq ? (uint32_t)NP * 8u : 0u);
        if (tid == 0) {
            sc[RS_BAIL] = s_end > (uint32_t)A.stage_bytes ? OWGS_RES_BAIL_STAGE : 0;
            *(u64*)&sc[RS_RSUM] = 0ull;
        }
        __syncthreads();
        int32_t* roff = (int32_t*)(stg + s_roff);
        int32_t* poff = (int32_t*)(stg + s_poff);
        uint4* rel = (uint4*)(stg + s_rel);
        uint4* pub = (uint4*)(stg + s_pub);
        u64* sq = (u64*)(stg + s_seq);
        if (sc[RS_BAIL] == 0) {
            for (int r = tid; r <= n_runs; r += 256) {
                roff[r] = ld_sys(A.in + i_roff + r);
                poff[r] = ld_sys(A.in + i_poff + r);
            }
            u64 rsum = 0;
            int e = 0;
            // one pass over both lists: every host-memory read of an iteration is in flight together (PCIe latency),
            // then the action meta gathers (HBM, L2-resident)
            for (int x = tid; x < max(NR, NP); x += 256) {
                const bool hr = x < NR, hp = x < NP;
                const int inv = hr ? ld_sys(A.in + i_rinv + x) : -1, ar = hr ? ld_sys(A.in + i_ract + x) : 0;
                const int ap = hp ? ld_sys(A.in + i_pact + x) : 0;
                uint32_t s_lo = 0u, s_hi = 0u;
                if (hp && has_seq) {
                    s_lo = (uint32_t)ld_sys(A.in + i_seq + 2 * x);
                    s_hi = (uint32_t)ld_sys(A.in + i_seq + 2 * x + 1);
                }
                const bool okr = ar >= 0 && ar < A.n_actions, okp = ap >= 0 && ap < A.n_actions;
                if ((hr && !okr) || (hp && !okp)) e |= OWGS_ERR_BAD_STREAM;
                const uint32_t my = (hr && okr) ? A.act_meta[ar].y : 0u;
                const uint32_t rs = (hr && okr) ? (uint32_t)A.act_slot[ar] : 0u;
                const uint2 m = (hp && okp) ? A.act_meta[ap] : make_uint2(0u, OWGS_AM_EMPTY);
                const uint32_t ps = (hp && okp) ? (uint32_t)A.act_slot[ap] : 0u;
                if (hr) {
                    rel[x] = make_uint4((uint32_t)inv, my, rs, 0u);
                    if (inv >= 0 && inv < n_slots) rsum += my & OWGS_AM_MEM_MASK;
                }
                if (hp) {
                    pub[x] = make_uint4(m.x, m.y, ps, 0u);
                    if (has_seq) sq[x] = (u64)s_lo | ((u64)s_hi << 32);
                }
            }
            if (rsum) atomicAdd((u64*)&sc[RS_RSUM], rsum);
            if (e) atomicOr(&sc[RS_ERR], e);
        }
        __syncthreads();
        // releases that could leave the LDS permit range: exact maximum first, then refuse the call untouched
        if (sc[RS_BAIL] == 0 && (long long)sc[RS_MAXP] + (long long)*(u64*)&sc[RS_RSUM] >= (long long)OWGS_PLIM) {
            if (tid == 0) sc[RS_MAXP] = (int)0x80000000;
            __syncthreads();
            int mx = (int)0x80000000;
            for (int i = tid; i < n_slots; i += 256) mx = max(mx, P[i] >= OWGS_PLIM ? P[i] - OWGS_PENC : P[i]);
            atomicMax(&sc[RS_MAXP], mx);
            __syncthreads();
            if (tid == 0 && (long long)sc[RS_MAXP] + (long long)*(u64*)&sc[RS_RSUM] >= (long long)OWGS_PLIM)
                sc[RS_BAIL] = OWGS_RES_BAIL_RELRISK;
            __syncthreads();
        }
        const int bail = sc[RS_BAIL];
        if (bail == 0 && wave == 0) {
            int err = 0;
            bool ovf_on = sc[RS_OVF] > 0;
            int used = sc[RS_USED];
            int32_t* out_inv = (int32_t*)(A.out + o_inv);
            uint8_t* out_fl = (uint8_t*)(A.out + o_fl);
            uint8_t* rel_fl = (uint8_t*)(A.out + o_rfl);
            // a new (invoker, fqn) entry (lane 0): the primary while it has room, else the overflow (the engine's rule)
            auto insert = [&](uint32_t key, uint32_t nv) -> int {
                int ix = -1;
                if (used < OWGS_CT_LDS_FILL || A.ovf.cap <= 0) {
                    uint32_t h = ct_home(key);
                    for (int p = 0; p < OWGS_CTC; ++p) {
                        const uint32_t kk = ct[h].x;
                        if (kk == 0u || kk == OWGS_CT_TOMB) {
                            ct[h] = make_uint2(key, nv);
                            used += kk == 0u;
                            ix = (int)h;
                            break;
                        }
                        h = (h + 1) & (OWGS_CTC - 1);
                    }
                }
                if (ix < 0 && A.ovf.cap > 0) {
                    const int oj = ovf_insert(A.ovf, key, nv);
                    if (oj >= 0) {
                        ix = OWGS_CTC + oj;
                        ovf_on = true;
                        sc[RS_OVF] += 1;
                    }
                }
                if (ix < 0) err |= OWGS_ERR_CTAB_FULL;
                return ix;
            };
            for (int r = 0; r < n_runs; ++r) {
                // ---- completions of run r (releaseInvoker SCPB:327-331 via processCompletion CLB:260-346)
                const int rb = roff[r], re = roff[r + 1];
                for (int j0 = rb; j0 < re; j0 += 64) {
                    const int j = j0 + lane;
                    const bool valid = j < re;
                    const uint4 rr = valid ? rel[j] : make_uint4(0xFFFFFFFFu, 0u, 0u, 0u);
                    const int inv = (int)rr.x;
                    const int mem = (int)(rr.y & OWGS_AM_MEM_MASK);
                    const int maxc = (int)((rr.y >> OWGS_AM_MAXC_SHIFT) & OWGS_AM_MAXC_MASK);
                    uint8_t flag = 0;
                    const bool in = valid && inv >= 0 && inv < n_slots;
                    if (valid && inv < 0) flag = OWGS_REL_NOENTRY_BIT;  // no ActivationEntry (CLB:278-279)
                    // maxConcurrent == 1: ForcibleSemaphore.release (FS:117-120), order-free (range checked above)
                    if (in && maxc <= 1) atomicAdd(&P[inv], mem);
                    // concurrent: RS.release(1, true) on the entry, in queue order (NS:98-113)
                    u64 cm = __ballot(in && maxc > 1);
                    while (cm) {
                        const int q = ffs64(cm);
                        cm &= cm - 1;
                        if (lane == q) {
                            const uint32_t key = ct_key(inv, (int)(rr.z & 0x1FFFFu));
                            uint32_t v;
                            const int ix = ct_lookup2(ct, A.ovf, ovf_on, key, &v);
                            const int c0 = (int)(v & OWGS_CT_C_MASK), o0 = ct_ops(v);
                            if (ix < 0 || o0 <= 0) {
                                flag = OWGS_REL_NOSUCH_BIT;  // NoSuchElementException (NS:103)
                            } else {
                                int c1 = c0 + 1;
                                const int o1 = o0 - 1;
                                if (c1 % maxc == 0) {  // RS:45-52: a whole container free -> its memory
                                    c1 -= maxc;
                                    P[inv] += mem;
                                }
                                const bool removed = o1 == 0;  // NS:109-111
                                const uint32_t nk = removed ? OWGS_CT_TOMB : key, nv = removed ? 0u : ct_val(c1, o1);
                                if (ix < OWGS_CTC) ct[ix] = make_uint2(nk, nv);
                                else ovf_st(A.ovf.t, ix - OWGS_CTC, nk, nv);
                            }
                        }
                        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    }
                    if (valid) rel_fl[j] = flag;
                }
                // ---- publishes of run r (SCPB:257-290 -> schedule SCPB:398-436)
                const int pb = poff[r], pe = poff[r + 1];
                for (int i0 = pb; i0 < pe; i0 += 64) {
                    const int nq = min(64, pe - i0);
                    const uint4 me = lane < nq ? pub[i0 + lane] : make_uint4(0u, OWGS_AM_EMPTY, 0u, 0u);
                    const u64 myseq = has_seq ? (lane < nq ? sq[i0 + lane] : 0ull) : seq_base + (u64)(i0 + lane);
                    int o_v = OWGS_NONE_V, o_f = 0;
                    for (int q = 0; q < nq; ++q) {
                        const uint32_t mx = (uint32_t)__builtin_amdgcn_readlane((int)me.x, q);
                        const uint32_t my = (uint32_t)__builtin_amdgcn_readlane((int)me.y, q);
                        const int slot = __builtin_amdgcn_readlane((int)me.z, q);
                        int x = OWGS_NONE_V, fl = 0;
                        if (my & OWGS_AM_EMPTY) {
                            x = OWGS_NONE_V;  // no invokers in the pool: None (SCPB:288-290)
                        } else if (my & OWGS_AM_THROW) {
                            x = OWGS_THROW_V;  // Int.MinValue hash: IndexOutOfBoundsException (SCPB:266-268)
                        } else {
                            const int home = (int)(mx & OWGS_AM_POS_MASK), step = (int)((mx >> 15) & OWGS_AM_POS_MASK);
                            const int pool = (mx & OWGS_AM_POOL) ? 1 : 0;
                            const int mem = (int)(my & OWGS_AM_MEM_MASK);
                            const int maxc = (int)((my >> OWGS_AM_MAXC_SHIFT) & OWGS_AM_MAXC_MASK);
                            const int n = pool ? nb : nm, base = pool ? A.n_ids - nb : 0;
                            const float rn = __builtin_amdgcn_rcpf((float)n);
                            int p = mod_fast(home + lane * step, n, rn);
                            const int adv = mod_fast(64 * step, n, rn);
                            int t = -1, tix = -1;
                            uint32_t tv = 0u;
                            // every pool position once: probes n and n + 1 repeat the first two with the same state
                            for (int s0 = 0; s0 < n; s0 += 64) {
                                const bool valid = s0 + lane < n;
                                const int id = base + p;
                                const int pv = valid ? P[id] : OWGS_PENC;
                                bool ok;
                                int ix = -1;
                                uint32_t v = 0u;
                                if (maxc <= 1) {
                                    ok = pv >= mem && pv < OWGS_PLIM;  // usable (folded) and tryAcquire (FS:63-71)
                                } else {
                                    ok = false;
                                    if (pv < OWGS_PLIM) {  // usable: a free slot of the key's container, or memory
                                        ix = ct_lookup2(ct, A.ovf, ovf_on, ct_key(id, slot), &v);
                                        ok = (v & OWGS_CT_C_MASK) != 0u || pv >= mem;
                                    }
                                }
                                const u64 m = __ballot(ok);
                                if (m) {
                                    const int L = ffs64(m);
                                    t = __builtin_amdgcn_readlane(id, L);
                                    tix = __builtin_amdgcn_readlane(ix, L);
                                    tv = (uint32_t)__builtin_amdgcn_readlane((int)v, L);
                                    break;
                                }
                                p += adv;
                                p -= p >= n ? n : 0;
                            }
                            if (t < 0) {  // overload: a random healthy invoker, forced (SCPB:417-424)
                                const int Hn = pool ? hb_e : hm_e;
                                if (Hn > 0) {
                                    const u64 sqv = (u64)__builtin_amdgcn_readlane((int)(uint32_t)myseq, q) |
                                                    ((u64)(uint32_t)__builtin_amdgcn_readlane((int)(myseq >> 32), q) << 32);
                                    const int kk = (int)rng_index(A.rng_seed, sqv, (uint32_t)Hn);
                                    t = (pool ? full_b : full_m) ? base + kk : select_usable(base, kk);
                                    if (t < 0) err |= OWGS_ERR_INTERNAL;
                                    else if (maxc > 1) tix = ct_lookup2(ct, A.ovf, ovf_on, ct_key(t, slot), &tv);
                                    fl = 1;
                                }
                            }
                            x = t;
                            if (t >= 0 && lane == 0) {
                                // tryAcquireConcurrent / forceAcquireConcurrent at t (NS:32-91, FS:63-110)
                                if (maxc <= 1) {
                                    P[t] -= mem;
                                } else {
                                    const int c0 = tix >= 0 ? (int)(tv & OWGS_CT_C_MASK) : 0;
                                    const int o0 = tix >= 0 ? ct_ops(tv) : 0;
                                    const bool slot_free = c0 >= 1;  // RS.tryAcquire(1) (NS:63)
                                    if (!slot_free) P[t] -= mem;     // a new container: its memory (NS:70-79)
                                    const int c1 = slot_free ? c0 - 1 : maxc - 1;
                                    const int o1 = o0 + 1;
                                    if (o1 > OWGS_MAX_OPS) err |= OWGS_ERR_OPS;
                                    const uint32_t nv = ct_val(c1, o1);
                                    if (tix < 0) insert(ct_key(t, slot), nv);
                                    else if (tix < OWGS_CTC) ct[tix].y = nv;
                                    else ovf_st_val(A.ovf.t, tix - OWGS_CTC, nv);
                                }
                                const int pt = P[t] >= OWGS_PLIM ? P[t] - OWGS_PENC : P[t];
                                if (pt < -OWGS_PLIM) err |= OWGS_ERR_PERMITS;
                            }
                            // lane 0's table updates (used, overflow in use) for every lane's next lookups
                            used = __builtin_amdgcn_readfirstlane(used);
                            ovf_on = __builtin_amdgcn_readfirstlane((int)ovf_on) != 0;
                            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                        }
                        if (lane == q) {
                            o_v = x;
                            o_f = fl;
                        }
                    }
                    if (lane < nq) {
                        out_inv[i0 + lane] = o_v;
                        out_fl[i0 + lane] = (uint8_t)o_f;
                    }
                }
            }
            // the call's releases may have raised permits: the range bound grows by what they returned at most
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) err |= __shfl_xor(err, d, 64);
            if (lane == 0) {
                sc[RS_USED] = used;
                const long long mp = (long long)sc[RS_MAXP] + (long long)*(u64*)&sc[RS_RSUM];
                sc[RS_MAXP] = (int)min(mp, (long long)0x7FFFFFFF);
                if (err) atomicOr(&sc[RS_ERR], err);
            }
        }
        __syncthreads();
        // ---- primary-table cleanup between calls: deleted entries keep chains long and fill the primary
        if (sc[RS_USED] > OWGS_CTC / 2) {
            int live = 0;
            for (int i = tid; i < OWGS_CTC; i += 256) live += ct[i].x != 0u && ct[i].x != OWGS_CT_TOMB;
            if (tid == 0) sc[RS_LIVE] = 0;
            __syncthreads();
            if (live) atomicAdd(&sc[RS_LIVE], live);
            __syncthreads();
            const int nlive = sc[RS_LIVE];
            if (sc[RS_USED] - nlive >= OWGS_CTC / 8) {  // (uniform) enough deleted entries to pay for a rebuild
                if (tid == 0) sc[RS_LIVE] = 0;
                __syncthreads();
                for (int i = tid; i < OWGS_CTC; i += 256) {
                    const uint2 e = ct[i];
                    if (e.x != 0u && e.x != OWGS_CT_TOMB) {
                        const int j = atomicAdd(&sc[RS_LIVE], 1);
                        A.ct_tmp[2 * j] = e.x;
                        A.ct_tmp[2 * j + 1] = e.y;
                    }
                }
                __threadfence_block();
                __syncthreads();
                for (int i = tid; i < OWGS_CTC; i += 256) ct[i] = make_uint2(0u, 0u);
                __syncthreads();
                for (int j = tid; j < nlive; j += 256) {  // distinct keys into an empty table: claim by CAS
                    const uint32_t kk = A.ct_tmp[2 * j], vv = A.ct_tmp[2 * j + 1];
                    uint32_t h = ct_home(kk);
                    for (int p = 0; p < OWGS_CTC; ++p) {
                        if (atomicCAS((uint32_t*)&ct[h], 0u, kk) == 0u) {
                            ct[h].y = vv;
                            break;
                        }
                        h = (h + 1) & (OWGS_CTC - 1);
                    }
                }
                if (tid == 0) sc[RS_USED] = nlive;
                __syncthreads();
            }
        }
        // ---- answer: outputs are in host memory before the result and the done word
        if (tid == 0) {
            const int e = sc[RS_ERR];  // (reported in the result word, not the context's error word)
            sc[RS_ERR] = 0;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            st_sys(&A.ctl[OWGS_RES_RESULT], bail | (e << 8));
            st_sys(&A.ctl[OWGS_RES_USED], sc[RS_USED]);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            st_sys(&A.ctl[OWGS_RES_DONE], k);
        }
        __syncthreads();
        last = k;
        t_idle = __builtin_amdgcn_s_memrealtime();
    }

    // ------------------------------------------------------------------ LDS -> state, exit
    for (int i = tid; i < n_slots; i += 256) {
        const int v = P[i];
        A.permits[i] = v >= OWGS_PLIM ? v - OWGS_PENC : v;
    }
    for (int i = tid; i < OWGS_CTC; i += 256) {
        const uint2 e = ct[i];
        A.ct_keys[i] = e.x;
        A.ct_vals[i] = e.y;
    }
    if (tid == 0 && A.ovf.cap > 0) __hip_atomic_store(A.ovf.cnt, sc[RS_OVF], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __threadfence();
    __syncthreads();
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        st_sys(&A.ctl[OWGS_RES_STATE], 2);
    }
}

extern "C" size_t owgs_resident_image_bytes(int32_t n_slots, int32_t n_ids) {
    return (size_t)res_layout(n_slots, n_ids).end;
}

extern "C" hipError_t owgs_launch_resident(const OwgsResArgs* a, size_t lds_bytes, hipStream_t s) {
    static bool attr = false;  // (per process: one device geometry)
    if (!attr) {
        const hipError_t e = hipFuncSetAttribute((const void*)owgs_resident_kernel,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, OWGS_LDS_BYTES);
        if (e != hipSuccess) return e;
        attr = true;
    }
    if (lds_bytes > OWGS_LDS_BYTES || a->n_slots > OWGS_MAX_SLOTS_CT) return hipErrorInvalidValue;
    hipLaunchKernelGGL(owgs_resident_kernel, dim3(1), dim3(256), lds_bytes, s, *a);
    return hipGetLastError();
}
