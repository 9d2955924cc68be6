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
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, __shfl_xor(v, d, 64));
    return v;
}
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = min(v, __shfl_xor(v, d, 64));
    return v;
}
// walk-cursor cache (LDS): per action (hashed) the first walk step that may still fit, valid for one cursor generation;
// an entry is one 64-bit word {action + 1 | generation mod 2^15 << 17, step}, written by atomic exchange so that lanes
// storing into the same entry leave one whole entry (the cache is cleared when the generation wraps mod 2^15)
__device__ __forceinline__ uint32_t cc_tag(uint32_t a, uint32_t gen) { return (a + 1u) | ((gen & 0x7FFFu) << 17); }
__device__ __forceinline__ uint32_t cc_slot(uint32_t a) { return (a * 2654435761u) >> (32 - 11); }
__device__ __forceinline__ int cc_get(const uint2* cc, uint32_t a, uint32_t gen) {
    const uint2 e = cc[cc_slot(a)];
    return e.x == cc_tag(a, gen) ? (int)e.y : 0;
}
__device__ __forceinline__ void cc_put(uint2* cc, uint32_t a, uint32_t gen, int step) {
    (void)__hip_atomic_exchange((u64*)&cc[cc_slot(a)], ((u64)(uint32_t)step << 32) | cc_tag(a, gen), __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_WORKGROUP);
}
// publish record .w: action handle | rank << 17 (earlier publishes of the same action in the decision's chunk of 64,
// at most 63) | RES_SHARED (an earlier concurrent publish of the chunk has the same fqn@version key under another
// action); written by the host (pinned calls) or by the staging waves (stream mode)
#define RES_ACT_MASK 0x1FFFFu
#define RES_RANK_SHIFT 17
#define RES_SHARED (1u << 23)
// speculative walk outcomes (resident engine, per decision of a chunk)
#define SP_NONE 0    // no decision in this lane
#define SP_TRIV 1    // decided without touching the state (None, the throw, a fallback without a healthy invoker)
#define SP_FOUND 2   // a target with room at the chunk's start: holds unless the decisions before took that room
#define SP_FORCED 3  // every pool position was full: the fallback's invoker, forced
#define SP_STOP 4    // decided alone: concurrent, or the walk was not finished within the budget
#define SP_FAIL 5    // (transient) the walk found no room anywhere

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

#define RES_CC 2048  // walk-cursor cache entries (LDS, 16 KB)
#define RES_BF 2048  // Bloom filter words over the primary table's keys (LDS, 8 KB)
#define RES_WF 256   // watched-key filter words (LDS, 1 KB): one bit per hashed fqn@version key with watched pairs
#define RES_WL 128   // watched-walk list (LDS, 1 KB): {action, deepest walk} of a run's decisions with watched keys
#ifndef RES_FIRST_READ_KB
#define RES_FIRST_READ_KB 4  // a call's input block: KB read together with the header (the rest in a second round)
#endif
// the primary table is rebuilt between calls once it holds more than RES_CLEAN_USED entries of which at least
// RES_CLEAN_TOMBS are deleted ones (deleted entries lengthen every probe chain through them)
#ifndef RES_CLEAN_USED
#define RES_CLEAN_USED (OWGS_CTC / 2)
#endif
#ifndef RES_CLEAN_TOMBS
#define RES_CLEAN_TOMBS (OWGS_CTC / 8)
#endif
struct ResLayout {
    uint32_t P, ub, pc, ct, sc, cc, mv, bf, wf, wl, hx, stage, end;
};
__host__ __device__ inline ResLayout res_layout(int n_slots, int n_ids) {
    const uint32_t words = (uint32_t)(n_ids + 31) / 32;
    ResLayout y;
    y.P = 0;
    y.ub = y.P + (((uint32_t)n_slots + 3u) & ~3u) * 4u;
    y.pc = y.ub + ((words + 4u) & ~3u) * 4u;
    y.ct = y.pc + ((words + 2u + 3u) & ~3u) * 4u;
    y.sc = y.ct + OWGS_CTC * 8u;
    y.cc = y.sc + 64u * 4u;
    y.mv = y.cc + RES_CC * 8u;
    y.bf = y.mv + 64u * 4u;
    y.wf = y.bf + RES_BF * 4u;
    y.wl = y.wf + RES_WF * 4u;
    y.hx = y.wl + RES_WL * 8u;       // the helper wave's speculation of one chunk: 64 x 2 x 16 B
    y.stage = y.hx + 64u * 32u;
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
#define RS_GEN 7     // walk-cursor generation: counts release runs (permits rise only there)
#define RS_RSUM 8    // (u64, 8-aligned) memory the call's releases return at most
#define RS_U0 10     // upper bound of every usable permit count of the managed / blackbox pool
#define RS_U1 11
#define RS_TOMB 12   // deleted primary entries (the cleanup between calls runs when they pile up)
#define RS_WLN 13    // entries of the watched-walk list (wl)
#define RS_HGO 14    // helper wave: request number (wave 0 -> wave 1; -1 = the call's decisions are done)
#define RS_HDONE 15  // helper wave: the request it answered
#define RS_HI0 16    // helper wave: the chunk's first publish and its size
#define RS_HNQ 17
#define RS_HPRE 18   // helper wave: 1 = the request is the next chunk's (its walk budget: cspec_pre)

// blocked Bloom filter over the primary table's keys (LDS, RES_BF words): one word and two bits per key, set on
// every insert into the primary and rebuilt with it; a key whose bits are not all set is not in the primary, so a
// lookup that misses -- the common case on a concurrent walk -- reads one word instead of a probe chain.  The word and
// the bits come from the same hash as the key's home block (ct_hash: bits 0-9 the home block of OWGS_CTC / 4, 10-20
// the word, 21-25 and 26-30 the bits), so a walk step hashes its key once
static_assert(OWGS_CTC / CT_BLK == 1024 && RES_BF == 2048, "the filter's bits sit above the home block's in one hash");
__device__ __forceinline__ uint2 bf_pos_h(uint32_t h) {
    return make_uint2((h >> 10) & (RES_BF - 1), (1u << ((h >> 21) & 31)) | (1u << ((h >> 26) & 31)));
}
__device__ __forceinline__ uint2 bf_pos(uint32_t key) { return bf_pos_h(ct_hash(key)); }
__device__ __forceinline__ void bf_add(uint32_t* bf, uint32_t key) {
    const uint2 b = bf_pos(key);
    atomicOr(&bf[b.x], b.y);
}
// primary table (LDS, interleaved {key, value}): index of key or -1, *val (0 if absent); chains end at an empty entry
__device__ __forceinline__ int ct_lookup(const uint2* ct, const uint32_t* bf, uint32_t key, uint32_t* val) {
    const uint32_t kh = ct_hash(key);
    uint32_t h = (kh & (OWGS_CTC / CT_BLK - 1)) * CT_BLK;  // (ct_home)
    *val = 0u;
    if (bf) {  // (null: the caller tested the filter)
        const uint2 b = bf_pos_h(kh);
        if ((bf[b.x] & b.y) != b.y) return -1;
    }
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
// the rest of a lookup whose first block (e01, e23 at h = ct_home(key)) the caller read: hit, chain end, or the next
// blocks
__device__ __forceinline__ int ct_lookup_after(const uint2* ct, uint32_t key, uint32_t h, uint4 e01, uint4 e23,
                                               uint32_t* val) {
    *val = 0u;
    for (int p = 0;;) {
        const bool h0 = e01.x == key, h1 = e01.z == key, h2 = e23.x == key, h3 = e23.z == key;
        if (h0 || h1 || h2 || h3) {
            *val = h0 ? e01.y : h1 ? e01.w : h2 ? e23.y : e23.w;
            return (int)h + (h0 ? 0 : h1 ? 1 : h2 ? 2 : 3);
        }
        if (e01.x == 0u || e01.z == 0u || e23.x == 0u || e23.z == 0u || ++p == OWGS_CTC / CT_BLK) return -1;
        h = (h + CT_BLK) & (OWGS_CTC - 1);
        e01 = *(const uint4*)&ct[h];
        e23 = *(const uint4*)&ct[h + 2];
    }
}
// watched pairs: the filter bit of an fqn@version key, the key's entry of the host-built
// index (A.w_sidx: {slot + 1, first, count, primary action}), and x^-1 mod n for a walk step coprime to n
__device__ __forceinline__ uint32_t wf_bit(uint32_t slot) { return (slot * 2654435761u) >> 19; }
__device__ __forceinline__ bool wf_test(const uint32_t* wf, uint32_t slot) {
    const uint32_t b = wf_bit(slot);
    return (wf[b >> 5] >> (b & 31)) & 1u;
}
__device__ __forceinline__ bool res_w_sfind(const OwgsResArgs& A, uint32_t slot, uint4* e) {
    const uint32_t m = (uint32_t)A.w_scap - 1u;
    uint32_t h = ct_hash(slot + 1u) & m;
    for (int p = 0; p < A.w_scap; ++p) {
        const uint4 v = A.w_sidx[h];
        if (v.x == slot + 1u) {
            *e = v;
            return true;
        }
        if (v.x == 0u) return false;
        h = (h + 1u) & m;
    }
    return false;
}
__device__ __forceinline__ int res_inv_mod(int x, int n) {
    int t = 0, nt = 1, r = n, nr = x % n;
    while (nr) {
        const int q = r / nr;
        int tmp = t - q * nt;
        t = nt;
        nt = tmp;
        tmp = r - q * nr;
        r = nr;
        nr = tmp;
    }
    return t < 0 ? t + n : t;
}

// both tables: index < OWGS_CTC primary, OWGS_CTC + j overflow entry j
__device__ __forceinline__ int ct_lookup2(const uint2* ct, const uint32_t* bf, const OwgsOvf& O, bool ovf_on,
                                          uint32_t key, uint32_t* val) {
    int i = ct_lookup(ct, bf, key, val);
    if (i < 0 && ovf_on) {
        const int j = ovf_find(O, key, val);
        i = j >= 0 ? OWGS_CTC + j : -1;
    }
    return i;
}

}  // namespace

// One workgroup of 256 threads; wave 0 decides, every wave loads, stages and writes back.  SMODE: stream mode
// (owgs_replay_device, OWGS_SPEC_REPLAY=1) -- a separate instantiation, so the shim's engine carries none of its code.
template <bool SMODE>
__global__ __launch_bounds__(256, 1) void owgs_resident_kernel(OwgsResArgs A) {
    extern __shared__ uint4 lds_raw[];
    char* Lb = (char*)lds_raw;
    const ResLayout Y = res_layout(A.n_slots, A.n_ids);
    int32_t* P = (int32_t*)(Lb + Y.P);
    uint32_t* ub = (uint32_t*)(Lb + Y.ub);
    uint32_t* pc = (uint32_t*)(Lb + Y.pc);
    uint2* ct = (uint2*)(Lb + Y.ct);
    int32_t* sc = (int32_t*)(Lb + Y.sc);
    uint2* cc = (uint2*)(Lb + Y.cc);
    int32_t* mv = (int32_t*)(Lb + Y.mv);
    uint32_t* bf = (uint32_t*)(Lb + Y.bf);
    uint32_t* wf = (uint32_t*)(Lb + Y.wf);
    uint2* wl = (uint2*)(Lb + Y.wl);
    uint4* hx = (uint4*)(Lb + Y.hx);
    char* stg = Lb + Y.stage;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int n_slots = A.n_slots, nm = A.nm, nb = A.nb;
    const int words = (A.n_ids + 31) >> 5;

    // ------------------------------------------------------------------ state -> LDS (once per launch)
    if (tid < 16) sc[tid] = (tid == RS_U0 || tid == RS_U1) ? (int)0x80000000 : (tid == RS_GEN ? (int)A.gen_base : 0);
    for (int i = tid; i < RES_CC; i += 256) cc[i] = make_uint2(0u, 0u);
    for (int i = tid; i < RES_BF; i += 256) bf[i] = 0u;
    for (int i = tid; i < RES_WF; i += 256) wf[i] = 0u;
    __syncthreads();
    for (int i = tid; A.w.cap > 0 && i < A.w_scap; i += 256) {  // the keys with watched pairs
        const uint32_t k = A.w_sidx[i].x;
        if (k != 0u) {
            const uint32_t b = wf_bit(k - 1u);
            atomicOr(&wf[b >> 5], 1u << (b & 31));
        }
    }
    {
        int used = 0, tombs = 0, mx = (int)0x80000000, u0 = (int)0x80000000, u1 = (int)0x80000000, e = 0;
        auto slot_in = [&](int i, int v, uint32_t u) {
            const bool unusable = !(i < A.n_ids && ((u >> (i & 31)) & 1u));
            if (v < -OWGS_PLIM || v >= OWGS_PLIM) e |= OWGS_ERR_PERMITS;
            mx = max(mx, v);
            if (!unusable && i < nm) u0 = max(u0, v);
            if (!unusable && i >= A.n_ids - nb && i < A.n_ids) u1 = max(u1, v);
            return unusable ? v + OWGS_PENC : v;
        };
        // four slots per 16-byte load, ten loads in flight per thread: one round trip per 10,240 slots
        constexpr int LB4 = 10;
        const int n4 = n_slots >> 2;
        for (int j0 = 0; j0 < n4; j0 += 256 * LB4) {
            int4 v[LB4];
            uint32_t u[LB4];
#pragma unroll
            for (int k = 0; k < LB4; ++k) {
                const int j = j0 + k * 256 + tid;
                v[k] = j < n4 ? ((const int4*)A.permits)[j] : make_int4(0, 0, 0, 0);
                u[k] = (j < n4 && 4 * j < A.n_ids) ? A.usable[j >> 3] : 0u;
            }
#pragma unroll
            for (int k = 0; k < LB4; ++k) {
                const int j = j0 + k * 256 + tid;
                if (j < n4)
                    ((int4*)P)[j] = make_int4(slot_in(4 * j, v[k].x, u[k]), slot_in(4 * j + 1, v[k].y, u[k]),
                                              slot_in(4 * j + 2, v[k].z, u[k]), slot_in(4 * j + 3, v[k].w, u[k]));
            }
        }
        for (int i = 4 * n4 + tid; i < n_slots; i += 256)  // (the last n_slots % 4 slots)
            P[i] = slot_in(i, A.permits[i], i < A.n_ids ? A.usable[i >> 5] : 0u);
        atomicMax(&sc[RS_U0], u0);
        atomicMax(&sc[RS_U1], u1);
        for (int i = tid; i <= words; i += 256) ub[i] = i < words ? A.usable[i] : 0u;
        // the primary table: four entries per 16-byte load of keys and of values, all in flight together
        {
            uint4 kq[OWGS_CTC / 1024], vq[OWGS_CTC / 1024];
#pragma unroll
            for (int k = 0; k < OWGS_CTC / 1024; ++k) {
                kq[k] = ((const uint4*)A.ct_keys)[k * 256 + tid];
                vq[k] = ((const uint4*)A.ct_vals)[k * 256 + tid];
            }
#pragma unroll
            for (int k = 0; k < OWGS_CTC / 1024; ++k) {
                const int i = 4 * (k * 256 + tid);
                const uint32_t kk[4] = {kq[k].x, kq[k].y, kq[k].z, kq[k].w}, vv[4] = {vq[k].x, vq[k].y, vq[k].z, vq[k].w};
                ((uint4*)ct)[i / 2] = make_uint4(kk[0], vv[0], kk[1], vv[1]);
                ((uint4*)ct)[i / 2 + 1] = make_uint4(kk[2], vv[2], kk[3], vv[3]);
#pragma unroll
                for (int e4 = 0; e4 < 4; ++e4) {
                    if (kk[e4] != 0u && kk[e4] != OWGS_CT_TOMB) bf_add(bf, kk[e4]);
                    used += kk[e4] != 0u;
                    tombs += kk[e4] == OWGS_CT_TOMB;
                }
            }
        }
        static_assert(OWGS_CTC % 1024 == 0, "the primary table loads 4 entries per thread per round");
        if (used) atomicAdd(&sc[RS_USED], used);
        if (tombs) atomicAdd(&sc[RS_TOMB], tombs);
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
    // stream mode (owgs_replay_device): no doorbell; the calls are the stream's batches, each as pieces of its
    // releases and then of its publishes that fit the staging area, read from HBM
    constexpr bool smode = SMODE;
    if (tid == 0 && !smode) st_sys(&A.ctl[OWGS_RES_STATE], 1);
    int s_b = 0, s_ph = 0;                  // (thread 0, stream mode) batch, phase (0 releases, 1 publishes),
    long long s_o = 0, s_r0 = 0, s_r1 = 0, s_p0 = 0, s_p1 = 0;  // offset in the phase, the batch's ranges
    bool s_loaded = false;
    const int s_rcap = min(4096, (A.stage_bytes - 96) / 17), s_pcap = min(2048, (A.stage_bytes - 128) / 29);

    // ------------------------------------------------------------------ calls
    int last = A.last_call;
    u64 t_idle = __builtin_amdgcn_s_memrealtime();
    const u64 t_launch = t_idle;
    int why = 0;  // (thread 0) why the engine exits: 0 the stop word, 1 idle, 2 its lifetime (OWGS_RES_WHY)
    for (;;) {
        if (smode) {
            if (tid == 0) {
                int kk = -1, nr = 0, np = 0;
                long long base = 0;
                while (s_b < A.s_nb) {
                    if (!s_loaded) {  // the batch's ranges (four independent loads: one round trip)
                        s_r0 = A.s_rel_off ? A.s_rel_off[s_b] : 0;
                        s_r1 = A.s_rel_off ? A.s_rel_off[s_b + 1] : 0;
                        s_p0 = A.s_acq_off[s_b];
                        s_p1 = A.s_acq_off[s_b + 1];
                        s_loaded = true;
                    }
                    if (s_ph == 0) {
                        if (s_r0 + s_o < s_r1) {
                            base = s_r0 + s_o;
                            nr = (int)min((long long)s_rcap, s_r1 - base);
                            s_o += nr;
                            kk = 1;
                            break;
                        }
                        s_ph = 1;
                        s_o = 0;
                    } else {
                        if (s_p0 + s_o < s_p1) {
                            base = s_p0 + s_o;
                            np = (int)min((long long)s_pcap, s_p1 - base);
                            s_o += np;
                            kk = 1;
                            break;
                        }
                        s_ph = 0;
                        s_o = 0;
                        s_loaded = false;
                        ++s_b;
                    }
                }
                int32_t* h = sc + 32;
                const u64 sb = A.s_seq_base + (u64)(np ? base : 0);
                h[0] = 1;
                h[1] = nr;
                h[2] = np;
                h[3] = 0;
                h[4] = (int32_t)(uint32_t)sb;
                h[5] = (int32_t)(uint32_t)(sb >> 32);
                h[6] = 16;
                h[7] = 32;
                h[8] = 32 + 16 * nr;
                h[9] = 32 + 16 * nr + 16 * np;
                h[10] = h[9];
                h[11] = h[12] = 0;
                h[13] = (int32_t)base;  // first release / publish of the piece in the stream
                h[14] = (int32_t)s_p0;  // the batch's first activation (its releases name earlier ones)
                sc[RS_K] = kk;
                *(u64*)&sc[RS_RSUM] = 0ull;
            }
        } else if (tid == 0) {
            int k = last;
            bool stop = false;
            for (long long spin = 0;; ++spin) {
                k = ld_sys(&A.ctl[OWGS_RES_BELL]);
                if (k != last) break;
                const u64 now = __builtin_amdgcn_s_memrealtime();
                // idle, or (between calls) past the launch's lifetime: the hardware queue this kernel holds may be
                // shared with another context's stream, whose launches wait behind it until it exits
                const bool life = A.life_ticks > 0 && (long long)(now - t_launch) > A.life_ticks;
                if ((long long)(now - t_idle) > A.idle_ticks || life || spin > (1ll << 32)) {
                    stop = true;
                    why = life ? 2 : 1;
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
        const u64 t_call = clock64();
        // ---- the call: its header (control block) and its input block (pinned host memory) into LDS.  The block holds
        // handles only (a word per publish: action, rank, shared flag; an invoker and an action per release): the
        // engine gathers each record's action meta and slot key from HBM.  The header and the first 4 KB of the block
        // are read together (one PCIe round trip for a call of up to ~1000 jobs)
        int32_t* hdr = sc + 32;  // RS_HDR words
        if (!smode) {  // (the block holds >= 4 KB: its capacity is larger; reading 16 KB at once measured slower)
            if (tid < OWGS_RES_NHDR) hdr[tid] = ld_sys(A.ctl + OWGS_RES_HDR + tid);
#if RES_FIRST_READ_KB == 8
            const uint4 v0 = ((const uint4*)A.in)[tid], v1 = ((const uint4*)A.in)[tid + 256];
            ((uint4*)stg)[tid] = v0;
            if (16 * (tid + 256) < A.stage_bytes) ((uint4*)stg)[tid + 256] = v1;
#else
            const uint4 v = ((const uint4*)A.in)[tid];
            ((uint4*)stg)[tid] = v;
#endif
        }
        __syncthreads();
        const int n_runs = hdr[0], NR = hdr[1], NP = hdr[2], has_seq = hdr[3];
        const u64 seq_base = (u64)(uint32_t)hdr[4] | ((u64)(uint32_t)hdr[5] << 32);
        const uint32_t s_poff = (uint32_t)hdr[6], s_seq = (uint32_t)hdr[9], s_in = (uint32_t)hdr[10];
        const long long s_first = hdr[13];  // (stream mode) the piece's first release / publish in the stream
        u64 rsum = (u64)(uint32_t)hdr[11] | ((u64)(uint32_t)hdr[12] << 32);  // memory the releases return at most
        // LDS after the input block: the records {invoker, meta.y, slot key, 0} per release and {meta.x, meta.y, slot
        // key, word} per publish (stream mode: inside the block, at the header's offsets), each publish's walk
        // cursor {generation, step}, then the outputs (mirrored by the host's output block): out_inv i32[NP],
        // out_flags u8[NP], rel_flags u8[NR]
        const uint32_t s_rel = smode ? (uint32_t)hdr[7] : ((s_in + 15u) & ~15u);
        const uint32_t s_pub = smode ? (uint32_t)hdr[8] : s_rel + 16u * (uint32_t)NR;
        const uint32_t s_cur = smode ? ((s_in + 15u) & ~15u) : s_pub + 16u * (uint32_t)NP;
        const uint32_t s_out = (s_cur + 8u * (uint32_t)NP + 15u) & ~15u;
        const uint32_t s_ofl = s_out + 4u * (uint32_t)NP, s_orf = s_ofl + (uint32_t)NP;
        const uint32_t s_end = (s_orf + (uint32_t)NR + 15u) & ~15u;
        if (tid == 0) sc[RS_BAIL] = s_end > (uint32_t)A.stage_bytes ? OWGS_RES_BAIL_STAGE : 0;
        __syncthreads();
        int32_t* roff = (int32_t*)(stg);
        int32_t* poff = (int32_t*)(stg + s_poff);
        uint4* rel = (uint4*)(stg + s_rel);
        uint4* pub = (uint4*)(stg + s_pub);
        u64* sq = (u64*)(stg + s_seq);
        uint2* pcur = (uint2*)(stg + s_cur);
        if (sc[RS_BAIL] == 0 && smode) {
            // the piece's records from the stream in HBM: a release names an activation decided earlier in this
            // launch (its invoker read through L2: written by wave 0's stores of an earlier piece), a publish an action
            if (tid == 0) {
                roff[0] = poff[0] = 0;
                roff[1] = NR;
                poff[1] = NP;
            }
            // (8 records per thread per round, each level of the gathers issued for all 8 before the next: three
            // dependent HBM round trips per round instead of per record)
            u64 rs = 0;
            for (int j0 = 0; j0 < NR; j0 += 8 * 256) {
                long long aid[8];
                int inv[8], a[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int j = j0 + u * 256 + tid;
                    aid[u] = j < NR ? A.s_rel_aid[s_first + j] : -1;
                    // (device streams are not checked on the host): a release names an activation of an earlier batch
                    if (j < NR && (aid[u] < 0 || aid[u] >= A.s_nact || aid[u] >= (long long)hdr[14])) {
                        atomicOr(&sc[RS_ERR], OWGS_ERR_BAD_STREAM);
                        aid[u] = -1;
                    }
                }
                if (A.s_claim) {  // ... and at most once (CommonLoadBalancer removes its entry, CLB:278-279)
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        if (aid[u] >= 0) {
                            const uint32_t bit = 1u << (aid[u] & 31);
                            if (atomicOr(&A.s_claim[aid[u] >> 5], bit) & bit) {
                                atomicOr(&sc[RS_ERR], OWGS_ERR_BAD_STREAM);
                                aid[u] = -1;
                            }
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    inv[u] = aid[u] >= 0 ? __hip_atomic_load(A.s_out_inv + aid[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : -1;
                    a[u] = aid[u] >= 0 ? A.s_act[aid[u]] : 0;
                    if ((uint32_t)a[u] >= (uint32_t)A.n_actions) {
                        atomicOr(&sc[RS_ERR], OWGS_ERR_BAD_STREAM);
                        a[u] = 0;
                        inv[u] = -1;
                    }
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int j = j0 + u * 256 + tid;
                    if (j < NR) {
                        const uint32_t my = A.act_meta[a[u]].y;
                        rel[j] = make_uint4((uint32_t)inv[u], my, (uint32_t)A.act_slot[a[u]], 0u);
                        if (inv[u] >= 0 && inv[u] < n_slots) rs += (u64)(my & OWGS_AM_MEM_MASK);
                    }
                }
            }
            for (int i0 = 0; i0 < NP; i0 += 8 * 256) {
                int a[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int i = i0 + u * 256 + tid;
                    a[u] = i < NP ? A.s_act[s_first + i] : -1;
                    if (i < NP && (uint32_t)a[u] >= (uint32_t)A.n_actions) {
                        atomicOr(&sc[RS_ERR], OWGS_ERR_BAD_STREAM);
                        a[u] = 0;
                    }
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int i = i0 + u * 256 + tid;
                    if (i < NP) {
                        const uint2 m = A.act_meta[a[u]];
                        pub[i] = make_uint4(m.x, m.y, (uint32_t)A.act_slot[a[u]], (uint32_t)a[u]);
                    }
                }
            }
            if (rs) atomicAdd((u64*)&sc[RS_RSUM], rs);
            __syncthreads();
            // each chunk's ranks (the host writes them for pinned calls): the waves take a chunk each in turn
            for (int c = wave; c * 64 < NP; c += 4) {
                const int i = c * 64 + lane;
                const bool v = i < NP;
                const uint4 r = v ? pub[i] : make_uint4(0u, 0u, 0u, 0u);
                const bool conc = v && !(r.y & (OWGS_AM_EMPTY | OWGS_AM_THROW)) &&
                                  ((r.y >> OWGS_AM_MAXC_SHIFT) & OWGS_AM_MAXC_MASK) > 1u;
                const int abits = 32 - __clz(max(A.n_actions - 1, 1));
                u64 same_a = __ballot(v);
                for (int b = 0; b < abits; ++b) {
                    const bool bit = (r.w >> b) & 1u;
                    const u64 m = __ballot(v && bit);
                    same_a &= bit ? m : ~m;
                }
                const u64 lt = (1ull << lane) - 1ull;
                bool shared = false;
                if (__ballot(conc)) {
                    u64 same_s = __ballot(conc);
                    for (int b = 0; b < 17; ++b) {
                        const bool bit = (r.z >> b) & 1u;
                        const u64 m = __ballot(conc && bit);
                        same_s &= bit ? m : ~m;
                    }
                    shared = conc && (same_s & ~same_a & lt) != 0ull;
                }
                if (v) pub[i].w = r.w | ((uint32_t)__popcll(same_a & lt) << RES_RANK_SHIFT) | (shared ? RES_SHARED : 0u);
            }
            __syncthreads();
            rsum = *(const u64*)&sc[RS_RSUM];
            for (int i0 = 0; i0 < NP; i0 += 8 * 256) {
                uint2 cu[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int i = i0 + u * 256 + tid;
                    const uint32_t a = i < NP ? (pub[i].w & RES_ACT_MASK) : 0xFFFFFFFFu;
                    cu[u] = (A.cur && a < (uint32_t)A.n_actions) ? A.cur[a] : make_uint2(0u, 0u);
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int i = i0 + u * 256 + tid;
                    if (i < NP) pcur[i] = cu[u];
                }
            }
        } else if (sc[RS_BAIL] == 0) {
            // the rest of a block beyond 4 KB, four 16-byte reads in flight per thread
            for (uint32_t o = 1024u * RES_FIRST_READ_KB + 16u * tid; o < s_in; o += 4u * 16u * 256u) {
                uint4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t ou = o + (uint32_t)u * 16u * 256u;
                    v[u] = ou < s_in ? ((const uint4*)A.in)[ou / 16u] : make_uint4(0u, 0u, 0u, 0u);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t ou = o + (uint32_t)u * 16u * 256u;
                    if (ou < s_in) ((uint4*)stg)[ou / 16u] = v[u];
                }
            }
            if (s_in > 1024u * RES_FIRST_READ_KB) __syncthreads();
            // every record's action meta and slot key, and every publish's walk cursor, gathered from HBM (four
            // records of each kind per thread in flight: one HBM round trip for a call of up to 1024 of each; the
            // decision loop then waits on nothing in HBM)
            const int32_t* rinv = (const int32_t*)(stg + (uint32_t)hdr[7]);
            const int32_t* ract = (const int32_t*)(stg + (uint32_t)hdr[8]);
            const uint32_t* pw = (const uint32_t*)(stg + (uint32_t)hdr[13]);
            for (int b0 = 0; b0 < max(NR, NP); b0 += 4 * 256) {
                uint2 pm[4], cu[4];
                uint32_t ps[4], rm[4], rs[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int i = b0 + 256 * u + tid;
                    const uint32_t a = i < NP ? (pw[i] & RES_ACT_MASK) : 0xFFFFFFFFu;
                    const bool ok = a < (uint32_t)A.n_actions;
                    pm[u] = ok ? A.act_meta[a] : make_uint2(0u, 0u);
                    ps[u] = ok ? (uint32_t)A.act_slot[a] : 0u;
                    cu[u] = (ok && A.cur) ? A.cur[a] : make_uint2(0u, 0u);
                    const uint32_t r = i < NR ? (uint32_t)ract[i] : 0xFFFFFFFFu;
                    const bool rok = r < (uint32_t)A.n_actions;
                    rm[u] = rok ? A.act_meta[r].y : 0u;
                    rs[u] = rok ? (uint32_t)A.act_slot[r] : 0u;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int i = b0 + 256 * u + tid;
                    if (i < NP) {
                        pub[i] = make_uint4(pm[u].x, pm[u].y, ps[u], pw[i]);
                        pcur[i] = cu[u];
                    }
                    if (i < NR) rel[i] = make_uint4((uint32_t)rinv[i], rm[u], rs[u], 0u);
                }
            }
        }
        if (tid == 0) {
            sc[RS_HGO] = 0;
            sc[RS_HDONE] = 0;
        }
        __syncthreads();
        // releases that could leave the LDS permit range: exact maximum first, then refuse the call untouched
        if (sc[RS_BAIL] == 0 && (long long)sc[RS_MAXP] + (long long)rsum >= (long long)OWGS_PLIM) {
            if (tid == 0) sc[RS_MAXP] = (int)0x80000000;
            __syncthreads();
            int mx = (int)0x80000000;
            for (int i = tid; i < n_slots; i += 256) mx = max(mx, P[i] >= OWGS_PLIM ? P[i] - OWGS_PENC : P[i]);
            atomicMax(&sc[RS_MAXP], mx);
            __syncthreads();
            if (tid == 0 && (long long)sc[RS_MAXP] + (long long)rsum >= (long long)OWGS_PLIM)
                sc[RS_BAIL] = OWGS_RES_BAIL_RELRISK;
            __syncthreads();
        }
        // speculation of a chunk's concurrent decisions (maxConcurrent > 1) against the state at the chunk's start, one
        // lane per decision: run by wave 0 itself, or by wave 1 while wave 0 walks the chunk's other decisions (the
        // speculation only reads the state; round 5)
        const bool hsplit = !smode && A.hsplit != 0;
        const int nhelp = hsplit ? min(max(A.hsplit, 1), 3) : 0;  // helper waves (1..3): lane i goes to wave 1 + i % nhelp
        auto cspec = [&](const uint4 me, const int nq_, const bool ovf_on_, const int cbudget, int& sp, int& sp_t, int& c_ix,
                         uint32_t& c_nv, bool& c_take, int& e_, uint32_t& n_ovf) {
            const int l_mem = (int)(me.y & OWGS_AM_MEM_MASK);
            const int l_pool = (me.x & OWGS_AM_POOL) ? 1 : 0;
            const int l_n = l_pool ? nb : nm, l_base = l_pool ? A.n_ids - nb : 0;
            const int l_home = (int)(me.x & OWGS_AM_POS_MASK), l_step = (int)((me.x >> 15) & OWGS_AM_POS_MASK);
            const int l_maxc = (int)((me.y >> OWGS_AM_MAXC_SHIFT) & OWGS_AM_MAXC_MASK);
            const bool l_cc = lane < nq_ && !(me.y & (OWGS_AM_EMPTY | OWGS_AM_THROW)) && l_maxc > 1;
            const int l_rank = (int)((me.w >> RES_RANK_SHIFT) & 63u);
            const float rmem = __builtin_amdgcn_rcpf((float)max(l_mem, 1));
                            // another action of the same key earlier in the chunk walks differently and shares the
                            // key's entries: its effect on mine is not predicted, so such a decision is decided alone
                            const int c_rank = l_rank;
                            int cneed = c_rank;
                            const float rmx = __builtin_amdgcn_rcpf((float)max(l_maxc, 1));
                            bool cw = l_cc && !(me.w & RES_SHARED);
                            int cpos = cw ? mod_fast(l_home, l_n, __builtin_amdgcn_rcpf((float)l_n)) : 0, cst = 0;
                            // 4 walk steps per round: their permits and Bloom-filter words read together, the map
                            // probed only where the filter says the key may be
                            while (__ballot(cw)) {
                                if (cw) {
                                    int idk[4], pvk[4];
                                    bool bk[4];
                                    int pp = cpos;
#pragma unroll
                                    for (int k = 0; k < 4; ++k) {
                                        idk[k] = l_base + pp;
                                        pvk[k] = P[idk[k]];
                                        pp += l_step;
                                        pp -= pp >= l_n ? l_n : 0;
                                    }
                                    uint32_t hk[4];  // each step's key hashed once: its filter word and home block
#pragma unroll
                                    for (int k = 0; k < 4; ++k) {
                                        const uint32_t kh = ct_hash(ct_key(idk[k], (int)me.z));
                                        hk[k] = (kh & (OWGS_CTC / CT_BLK - 1)) * CT_BLK;
                                        const uint2 b = bf_pos_h(kh);
                                        bk[k] = (bf[b.x] & b.y) == b.y;
                                    }
                                    // the first map block of every step the filter passes, read together (the
                                    // lookups below only continue a chain past it)
                                    uint4 fa[4], fb[4];
#pragma unroll
                                    for (int k = 0; k < 4; ++k) {
                                        fa[k] = fb[k] = make_uint4(0u, 0u, 0u, 0u);
                                        if (bk[k]) {
                                            fa[k] = *(const uint4*)&ct[hk[k]];
                                            fb[k] = *(const uint4*)&ct[hk[k] + 2];
                                        }
                                    }
                                    // each step's entry: a hit in its first block, or absent when that block has an
                                    // empty entry (the chain ends there); a chain past the block (rare) is followed
                                    // below.  Then each step's capacity for the key in units, c + floor(permits /
                                    // mem) * maxConcurrent (free slots, then containers the memory holds; the
                                    // container count capped at 64: a rank is below 64), and the walk's step is the
                                    // first whose units exceed what the rank still needs
                                    uint32_t vk[4];
                                    int ixk[4], uk[4];
                                    bool chain = false;
#pragma unroll
                                    for (int k = 0; k < 4; ++k) {
                                        const uint32_t key = ct_key(idk[k], (int)me.z);
                                        const bool h0 = fa[k].x == key, h1 = fa[k].z == key, h2 = fb[k].x == key,
                                                   h3 = fb[k].z == key;
                                        const bool hit = bk[k] && (h0 || h1 || h2 || h3);
                                        vk[k] = hit ? (h0 ? fa[k].y : h1 ? fa[k].w : h2 ? fb[k].y : fb[k].w) : 0u;
                                        ixk[k] = hit ? (int)hk[k] + (h0 ? 0 : h1 ? 1 : h2 ? 2 : 3) : -1;
                                        const bool open = fa[k].x == 0u || fa[k].z == 0u || fb[k].x == 0u || fb[k].z == 0u;
                                        chain = chain || (bk[k] && !hit && !open);
                                    }
                                    if (__ballot(chain)) {
#pragma unroll
                                        for (int k = 0; k < 4; ++k) {
                                            const uint32_t key = ct_key(idk[k], (int)me.z);
                                            const bool open = fa[k].x == 0u || fa[k].z == 0u || fb[k].x == 0u || fb[k].z == 0u;
                                            if (bk[k] && ixk[k] < 0 && !open)
                                                ixk[k] = ct_lookup_after(ct, key, hk[k], fa[k], fb[k], &vk[k]);
                                        }
                                    }
                                    if (ovf_on_) {  // (wave 0 only) keys beyond the primary
#pragma unroll
                                        for (int k = 0; k < 4; ++k) {
                                            if (ixk[k] < 0 && cst + k < l_n && pvk[k] < OWGS_PLIM) {
                                                ++n_ovf;
                                                const int oj = ovf_find(A.ovf, ct_key(idk[k], (int)me.z), &vk[k]);
                                                ixk[k] = oj >= 0 ? OWGS_CTC + oj : -1;
                                            }
                                        }
                                    }
#pragma unroll
                                    for (int k = 0; k < 4; ++k) {
                                        const int pv = pvk[k];
                                        int m = 0;
                                        if (pv >= 64 * l_mem) {
                                            m = 64;
                                        } else if (pv >= l_mem) {  // (pv < 64 mem: exact after correction)
                                            m = (int)((float)pv * rmem);
                                            m -= m * l_mem > pv ? 1 : 0;
                                            m += (m + 1) * l_mem <= pv ? 1 : 0;
                                        }
                                        const bool stepv = cst + k < l_n && pv < OWGS_PLIM;
                                        uk[k] = stepv ? (int)(vk[k] & OWGS_CT_C_MASK) + m * l_maxc : 0;
                                    }
                                    int kf = 4, need_f = cneed;
                                    {
                                        int need = cneed;
#pragma unroll
                                        for (int k = 0; k < 4; ++k) {
                                            const bool here = kf == 4 && need < uk[k];
                                            kf = here ? k : kf;
                                            need_f = here ? need : need_f;
                                            need -= kf == 4 ? uk[k] : 0;
                                        }
                                        if (kf == 4) cneed = need;
                                    }
                                    if (kf < 4) {
                                        const uint32_t v = kf == 0 ? vk[0] : kf == 1 ? vk[1] : kf == 2 ? vk[2] : vk[3];
                                        const int ix = kf == 0 ? ixk[0] : kf == 1 ? ixk[1] : kf == 2 ? ixk[2] : ixk[3];
                                        const int c0 = (int)(v & OWGS_CT_C_MASK), o0 = ix >= 0 ? ct_ops(v) : 0;
                                        int c1;
                                        bool tk = false;
                                        if (need_f < c0) {  // a free slot of the key's container
                                            c1 = c0 - need_f - 1;
                                        } else {  // a container the memory holds, maxConcurrent slots each
                                            const int kp = need_f - c0;
                                            int qc = (int)((float)kp * rmx);
                                            qc -= qc * l_maxc > kp ? 1 : 0;
                                            qc += (qc + 1) * l_maxc <= kp ? 1 : 0;
                                            const int j = kp - qc * l_maxc;  // (kp < 64: exact)
                                            tk = j == 0;
                                            c1 = l_maxc - j - 1;
                                        }
                                        if (o0 + need_f + 1 > OWGS_MAX_OPS) e_ |= OWGS_ERR_OPS;
                                        cneed = need_f;
                                        c_ix = ix;
                                        c_take = tk;
                                        c_nv = ct_val(c1, o0 + need_f + 1);
                                    }
                                    if (kf < 4) {
                                        sp = SP_FOUND;
                                        sp_t = kf == 0 ? idk[0] : kf == 1 ? idk[1] : kf == 2 ? idk[2] : idk[3];
                                        cw = false;
                                    } else {
                                        cst += 4;
                                        cpos = pp;
                                        if (cst >= l_n) {
                                            if (c_rank == 0) sp = SP_FAIL;  // every pool position: forced below (a
                                            cw = false;                     // repeat: decided alone)
                                        } else if (cst >= cbudget) {
                                            cw = false;  // SP_STOP: decided alone
                                        }
                                    }
                                }
                            }
                                };
        // speculation of a chunk's maxConcurrent == 1 decisions, one lane per decision (wave 0): each walks on its own
        // against the state at the chunk's start, A.spec steps at most (4 permit reads in flight per round), from sbeg
        // (its cursor).  Permits only fall inside a run (releases come first, SCPB:327-331 via CLB:260-346), so a step
        // full then is full at the decision's turn: the walk's target stays the decision's unless the decisions before
        // it took the room there, and a walk that found no room anywhere is a fallback whatever came before
        // (SCPB:417-424).  Repeats of one action in the chunk share its walk: the k-th (rank k among the chunk's plain
        // decisions of that action, from the record) passes over the room the k before it take, so it walks to the
        // step where the capacity for its memory met so far, sum of floor(permits / mem), exceeds k.
        auto pspec = [&](const uint4 me, const int nq_, const int sbeg, const int U0_, const int U1_, int& sp, int& sp_t,
                         int& sp_ts, uint32_t& rounds) {
            const int l_mem = (int)(me.y & OWGS_AM_MEM_MASK);
            const int l_pool = (me.x & OWGS_AM_POOL) ? 1 : 0;
            const int l_n = l_pool ? nb : nm, l_base = l_pool ? A.n_ids - nb : 0;
            const int l_home = (int)(me.x & OWGS_AM_POS_MASK), l_step = (int)((me.x >> 15) & OWGS_AM_POS_MASK);
            const bool l_c1 = lane < nq_ && !(me.y & (OWGS_AM_EMPTY | OWGS_AM_THROW)) &&
                              ((me.y >> OWGS_AM_MAXC_SHIFT) & OWGS_AM_MAXC_MASK) <= 1u;
            const bool l_plain = l_c1 && l_mem <= (l_pool ? U1_ : U0_);
            int need = l_plain ? (int)((me.w >> RES_RANK_SHIFT) & 63u) : 0;
            const float rmem = __builtin_amdgcn_rcpf((float)max(l_mem, 1));
            bool walking = false;
            int wp = 0, ws = sbeg;
            if (l_c1) {
                if (!l_plain || sbeg >= l_n) {
                    sp = SP_FAIL;  // mem above the pool's bound U, or a cursor past every step
                } else {
                    walking = true;
                    wp = mod_fast(l_home + ws * l_step, l_n, __builtin_amdgcn_rcpf((float)l_n));
                }
            }
            for (int it = 0; __ballot(walking); it += 4) {
                if (walking) {
                    int pk[4], vk[4];
                    int pp = wp;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        pk[k] = pp;
                        vk[k] = P[l_base + pp];
                        pp += l_step;
                        pp -= pp >= l_n ? l_n : 0;
                    }
                    int kf = 4;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int v = vk[k];
                        if (kf == 4 && ws + k < l_n && v >= l_mem && v < OWGS_PLIM) {
                            if (v >= (need + 1) * l_mem) {
                                kf = k;
                            } else {  // room for 1..need activations here (v < 64 mem: exact after correction)
                                int c = (int)((float)v * rmem);
                                c -= c * l_mem > v ? 1 : 0;
                                c += (c + 1) * l_mem <= v ? 1 : 0;
                                need -= c;
                            }
                        }
                    }
                    if (kf < 4) {
                        sp = SP_FOUND;
                        sp_t = l_base + (kf == 0 ? pk[0] : kf == 1 ? pk[1] : kf == 2 ? pk[2] : pk[3]);
                        sp_ts = ws + kf;
                        walking = false;
                    } else {
                        ws += 4;
                        wp = pp;
                        if (ws >= l_n) {
                            sp = SP_FAIL;  // every pool position probed
                            walking = false;
                        } else if (it + 4 >= A.spec) {
                            sp = SP_STOP;  // the rest of the walk: one at a time, from ws
                            sp_ts = ws;
                            walking = false;
                        }
                    }
                }
            }
            rounds += (uint32_t)__popcll(__ballot(l_c1 && l_plain));
        };
        // the concurrent decisions of a run's next chunk speculated by the helper wave while wave 0 makes the current
        // chunk's last decisions (round 6): one helper wave, no watched pairs (their walks leave marks), and wave 0
        // takes such a speculation only while no overflow entry exists.  Read before some of the current chunk's takes,
        // the permits are at least what the next chunk finds (capacities too high, never too low: a walk's target is
        // at or before the decision's, and no step before it has room for the decision at its turn)
        const bool pre_on = hsplit && A.hsplit == 1 && A.prespec != 0 && A.w.cap <= 0;
        // walk steps of a concurrent speculation: on the chunk's critical path 4 (8 measured slower, round 5); the next
        // chunk's, which the helper starts while wave 0 finishes the current chunk, may walk further
        const int cb_now = A.cspec > 0 ? A.cspec : max(4, A.spec >> 2);
        const int cb_pre = A.cspec_pre > 0 ? A.cspec_pre : cb_now;
        const int bail = sc[RS_BAIL];
        if (bail == 0 && wave == 0) {
            int err = 0, hreq_n = 0;  // (hreq_n: requests posted to the helper wave in this call)
            bool ovf_on = sc[RS_OVF] > 0;
            int used = sc[RS_USED], tombs = 0;  // (tombs: per lane, deleted entries made - reused this call)
            // maxConcurrent == 1 walks: U = an upper bound of every usable permit count of the pool (a walk with
            // mem > U fails everywhere: straight to the fallback), and per action the first walk step that may
            // still fit (a cache keyed by action, valid while no release raised a permit: generation = release runs)
            int U0 = sc[RS_U0], U1 = sc[RS_U1];
            uint32_t gen = (uint32_t)sc[RS_GEN];
            uint32_t pr_rounds = 0, pr_dec = 0, pr_ovf = 0, pr_hit = 0, pr_u = 0, pr_grp = 0, pr_pass = 0, pr_alone = 0;
            u64 pr_alone_cyc = 0, pr_spec_cyc = 0, pr_val_cyc = 0;
            u64 pr_c_match = 0, pr_c_pwalk = 0, pr_c_cwalk = 0, pr_c_ins = 0, pr_c_relc = 0;
            uint32_t pr_pre = 0;
            u64 pr_hcyc = 0;  // the helper wave's concurrent walks (cycles)
            // the chunk the helper waves speculate ahead (-1 none), the plain helper's requests, and whether requests
            // may still be posted in this call
            int pre_i0 = -1;
            bool pre_live = pre_on;
            const u64 pr_stage = clock64() - t_call;  // header, staging and the range check
            u64 pr_rel = 0, pr_pub = 0;
            int32_t* out_inv = (int32_t*)(stg + s_out);  // (LDS; copied to host memory after the call)
            uint8_t* out_fl = (uint8_t*)(stg + s_ofl);
            uint8_t* rel_fl = (uint8_t*)(stg + s_orf);
            // a new (invoker, fqn) entry (lane 0): the primary while it has room, else the overflow (the engine's rule)
            auto insert = [&](uint32_t key, uint32_t nv) -> int {
                int ix = -1;
                if (used < OWGS_CT_LDS_FILL || A.ovf.cap <= 0) {
                    uint32_t h = ct_home(key);
                    for (int p = 0; p < OWGS_CTC; ++p) {
                        const uint32_t kk = ct[h].x;
                        if (kk == 0u || kk == OWGS_CT_TOMB) {
                            ct[h] = make_uint2(key, nv);
                            bf_add(bf, key);
                            used += kk == 0u;
                            tombs -= kk == OWGS_CT_TOMB;
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
            // watched-walk list -> Z marks: every entry (one lane each) marks the watched pairs of its action's key
            // at the walk steps before its deepest walk (the host's index lists a key's pairs by step in the key's
            // primary action's walk; another action of the key computes each pair's step); a mark on a pair whose
            // entry is present is never read (the entry's removal clears it)
            auto w_flush = [&]() {
                const int nl = sc[RS_WLN];
                for (int j0 = 0; j0 < nl; j0 += 64) {
                    const int j = j0 + lane;
                    uint4 e;
                    const uint2 we = j < nl ? wl[j] : make_uint2(0u, 0u);
                    const uint32_t a = we.x;
                    const int depth = (int)we.y;
                    uint2 am = make_uint2(0u, 0u);
                    uint32_t aslot = 0u;
                    if (j < nl) {
                        am = A.act_meta[a];
                        aslot = (uint32_t)A.act_slot[a];
                    }
                    if (j < nl && res_w_sfind(A, aslot, &e)) {
                        const int wpool = (am.x & OWGS_AM_POOL) ? 1 : 0;
                        const int wn = wpool ? nb : nm, wbase = wpool ? A.n_ids - nb : 0;
                        const int whome = (int)(am.x & OWGS_AM_POS_MASK), wstep = (int)((am.x >> 15) & OWGS_AM_POS_MASK);
                        const bool primary = e.w == a;
                        const int winv = (!primary && wn > 1) ? res_inv_mod(wstep % wn, wn) : 0;
                        const uint32_t kend = e.y + e.z;
                        // four pairs per round: their list entries, then their W keys, read together
                        for (uint32_t k0 = e.y; k0 < kend; k0 += 4) {
                            uint2 pe[4];
                            uint32_t key[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u)
                                pe[u] = k0 + u < kend ? A.w_list[k0 + u] : make_uint2(0u, 0x7FFFFFFFu);
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                const bool go = k0 + u < kend && (!primary || (int)pe[u].y < depth);
                                key[u] = go ? __hip_atomic_load(&A.w.keys[pe[u].x], __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_AGENT)
                                            : 0u;
                            }
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                if (key[u] == 0u || key[u] == OWGS_CT_TOMB) continue;
                                const int x = (int)(key[u] & 0x7FFFu) - 1;
                                if (x < 0 || x >= A.n_ids || !((ub[x >> 5] >> (x & 31)) & 1u)) continue;  // not tried
                                if (!primary) {
                                    const int pos = x - wbase;
                                    if (pos < 0 || pos >= wn) continue;
                                    const int st = wn > 1 ? (int)(((long long)((pos - whome + wn) % wn) * winv) % wn) : 0;
                                    if (st >= depth) continue;
                                }
                                atomicOr(&A.w.vals[pe[u].x], OWGS_W_Z);
                            }
                            if (primary && (int)pe[3].y >= depth) break;  // (the list is by step)
                        }
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                if (lane == 0) sc[RS_WLN] = 0;
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            };
            if (lane == 0) sc[RS_WLN] = 0;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            for (int r = 0; r < n_runs; ++r) {
                // ---- completions of run r (releaseInvoker SCPB:327-331 via processCompletion CLB:260-346)
                const int rb = roff[r], re = roff[r + 1];
                if (re > rb) {
                    ++gen;  // permits may rise: every walk cursor of an earlier generation is stale
                    if ((gen & 0x7FFFu) == 0u)  // the cache's generation field wraps: no entry may match again
                        for (int i = lane; i < RES_CC; i += 64) cc[i] = make_uint2(0u, 0u);
                }
                const u64 tr0 = clock64();
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
                    // concurrent: RS.release(1, true) on the entry, in queue order (NS:98-113).  Every lane looks its
                    // entry up at once; releases of different entries commute, so the primary-table entries that one
                    // lane of this group releases are updated in parallel, and entries with several releases here
                    // (and overflow entries) one release at a time in queue order
                    const u64 trc = clock64();
                    const bool cr = in && maxc > 1;
                    const uint32_t rkey = cr ? ct_key(inv, (int)(rr.z & 0x1FFFFu)) : 0u;
                    uint32_t rv = 0u;
                    int rix = -1;
                    if (cr) rix = ct_lookup2(ct, bf, A.ovf, ovf_on, rkey, &rv);
                    // a release of an fqn@version key with watched pairs: below, with the empty-entry rule
                    // (the filter may pass a key without watched pairs: the path below is releaseConcurrent's
                    // general rule, equal to the closed form for such keys)
                    const bool wat = cr && A.w.cap > 0 && wf_test(wf, rr.z & 0x1FFFFu);
                    const bool prim = cr && !wat && rix >= 0 && rix < OWGS_CTC;
                    // releases of one primary entry in this group: the j-th of them (queue order) finds the entry as
                    // the j before it leave it -- RS.release(1, true) j times from (c0, o0): c0 + j free slots, a
                    // container's memory back each time that count reaches a multiple of maxConcurrent, the entry
                    // removed when operationCount reaches 0 and every later release a NoSuchElement -- so all of them
                    // apply at once (closed form) when they agree on maxConcurrent and memory; else one at a time
                    u64 eq = 0ull, dup = 0ull;
                    const u64 pm = __ballot(prim);
                    if (pm & (pm - 1ull)) {
                        eq = pm;
                        for (int b = 0; b < 12; ++b) {
                            const bool bit = (rix >> b) & 1;
                            const u64 m = __ballot(prim && bit);
                            eq &= bit ? m : ~m;
                        }
                        if (!prim) eq = 0ull;
                        // a group whose releases disagree on maxConcurrent or memory: one at a time
                        const int lead = eq ? ffs64(eq) : 0;
                        const int lmaxc = __shfl(maxc, lead, 64), lmem = __shfl(mem, lead, 64);
                        dup = __ballot(prim && (eq & (eq - 1ull)) && (lmaxc != maxc || lmem != mem));
                        const u64 bad = dup;  // every lane of a disagreeing group goes one at a time
                        dup = 0ull;
                        for (u64 bb = bad; bb;) {
                            const int q = ffs64(bb);
                            const int rq = __builtin_amdgcn_readlane(rix, q);
                            const u64 grp = __ballot(prim && rix == rq);
                            dup |= grp;
                            bb &= ~grp;
                        }
                    } else {
                        eq = prim ? (1ull << lane) : 0ull;
                    }
                    if (cr && !wat && rix < 0) flag = OWGS_REL_NOSUCH_BIT;  // NoSuchElementException (NS:103)
                    if (prim && !((dup >> lane) & 1ull)) {
                        const int c0 = (int)(rv & OWGS_CT_C_MASK), o0 = ct_ops(rv);
                        const int j = (int)__popcll(eq & ((1ull << lane) - 1ull)), cnt = (int)__popcll(eq);
                        if (j >= o0) {
                            flag = OWGS_REL_NOSUCH_BIT;  // the entry is gone by this release (NS:103)
                        } else {
                            if ((c0 + j + 1) % maxc == 0) atomicAdd(&P[inv], mem);  // RS:45-52: a container free
                            const int jj = min(cnt, o0);
                            if (j == jj - 1) {  // the group's last release that finds the entry writes it
                                const int o1 = o0 - jj, c1 = (c0 + jj) % maxc;
                                const bool removed = o1 == 0;  // NS:109-111
                                ct[rix] = make_uint2(removed ? OWGS_CT_TOMB : rkey, removed ? 0u : ct_val(c1, o1));
                                tombs += removed;
                            }
                        }
                    }
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    u64 cm = dup | __ballot(cr && !wat && rix >= OWGS_CTC);
                    while (cm) {
                        const int q = ffs64(cm);
                        cm &= cm - 1;
                        if (lane == q) {
                            const uint32_t key = rkey;
                            uint32_t v;
                            const int ix = ct_lookup2(ct, bf, A.ovf, ovf_on, key, &v);
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
                                tombs += removed && ix < OWGS_CTC;
                            }
                        }
                        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    }
                    // releases of keys with watched pairs (after updateCluster, SCPB:561-584, discarded the entries of
                    // activations still in flight): releaseConcurrent (NS:98-113) applies RS.release(1, true) to the
                    // entry it finds -- operationCount may count below 0 -- and removes it at 0; an absent entry throws
                    // NoSuchElement (NS:103) unless the reference holds the empty entry a failed try left (Z,
                    // getOrElseUpdate NS:61-62), which then takes the release.  d (in flight - operationCount) falls
                    // only with a throw; the pair leaves W at 0.  Releases of distinct keys commute: each lane applies
                    // its own at once; a key with several releases in the group, and every release that needs the
                    // empty entry inserted, go one at a time in queue order
                    if (__ballot(wat)) {
                        u64 wdup = 0ull;
                        for (u64 bb = __ballot(wat); bb;) {
                            const int q = ffs64(bb);
                            const uint32_t kq = (uint32_t)__builtin_amdgcn_readlane((int)rkey, q);
                            const u64 g = __ballot(wat && rkey == kq);
                            if (g & (g - 1ull)) wdup |= g;
                            bb &= ~g;
                        }
                        const int wslot = (int)(rr.z & 0x1FFFFu);
                        // one RS.release(1, true) on a present entry (ix, v), or the throw / the empty entry's turn
                        auto w_apply = [&](int ix, uint32_t v, int wj, uint32_t wv) {
                            const int cc0 = (int)(v & OWGS_CT_C_MASK), o1 = ct_ops(v) - 1;
                            int c1 = cc0 + 1;
                            if (c1 % maxc == 0) {  // RS:45-52: a whole container free -> its memory
                                c1 -= maxc;
                                atomicAdd(&P[inv], mem);
                            }
                            if (o1 < -OWGS_MAX_OPS) err |= OWGS_ERR_OPS;
                            const bool removed = o1 == 0;  // NS:109-111
                            const uint32_t nk = removed ? OWGS_CT_TOMB : rkey, nv = removed ? 0u : ct_val(c1, o1);
                            if (ix < OWGS_CTC) ct[ix] = make_uint2(nk, nv);
                            else ovf_st(A.ovf.t, ix - OWGS_CTC, nk, nv);
                            tombs += removed && ix < OWGS_CTC;
                            if (removed && wj >= 0 && (wv & OWGS_W_Z))  // the removal drops the empty entry too
                                __hip_atomic_store(&A.w.vals[wj], wv & ~OWGS_W_Z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        };
                        auto w_throw = [&](int wj, uint32_t wv) {
                            flag = OWGS_REL_NOSUCH_BIT;  // NoSuchElementException (NS:103)
                            if (wj < 0) return;
                            const int d = (int)(wv & ~OWGS_W_Z) - 1;  // one in-flight activation fewer, entry absent
                            if (d <= 0) {
                                __hip_atomic_store(&A.w.vals[wj], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                __hip_atomic_store(&A.w.keys[wj], OWGS_CT_TOMB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                atomicSub(&A.w.wkey[wslot], 1);
                                atomicSub(A.w.cnt, 1);
                            } else {
                                __hip_atomic_store(&A.w.vals[wj], (uint32_t)d | (wv & OWGS_W_Z), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
                            }
                        };
                        bool wser = wat && ((wdup >> lane) & 1ull);
                        if (wat && !wser) {
                            const int wj = w_find(A.w, rkey);
                            const uint32_t wv = wj >= 0 ? __hip_atomic_load(&A.w.vals[wj], __ATOMIC_RELAXED,
                                                                             __HIP_MEMORY_SCOPE_AGENT)
                                                        : 0u;
                            if (rix >= 0) w_apply(rix, rv, wj, wv);
                            else if (wv & OWGS_W_Z) wser = true;  // the empty entry goes into the table: one at a time
                            else w_throw(wj, wv);
                        }
                        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                        for (u64 sm = __ballot(wser); sm; sm &= sm - 1ull) {
                            const int q = ffs64(sm);
                            if (lane == q) {
                                const int wj = w_find(A.w, rkey);
                                const uint32_t wv = wj >= 0 ? __hip_atomic_load(&A.w.vals[wj], __ATOMIC_RELAXED,
                                                                                 __HIP_MEMORY_SCOPE_AGENT)
                                                            : 0u;
                                uint32_t v;
                                int ix = ct_lookup2(ct, bf, A.ovf, ovf_on, rkey, &v);
                                if (ix < 0 && (wv & OWGS_W_Z)) {  // the reference's empty entry {0, 0} takes it
                                    ix = insert(rkey, 0u);
                                    v = 0u;
                                }
                                if (ix >= 0) w_apply(ix, v, wj, wv);
                                else w_throw(wj, wv);
                            }
                            used = __builtin_amdgcn_readlane(used, q);
                            ovf_on = __builtin_amdgcn_readlane((int)ovf_on, q) != 0;
                            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                        }
                    }
                    pr_c_relc += clock64() - trc;
                    if (valid) rel_fl[j] = flag;
                    // the pools' permit bounds follow what the releases raised
                    const int pn = in ? P[inv] : (int)0x80000000;
                    const int um = wave_max_i(pn < OWGS_PLIM ? pn : (int)0x80000000);
                    U0 = max(U0, um);
                    U1 = max(U1, um);
                }
                const u64 tr1 = clock64();
                pr_rel += tr1 - tr0;
                // ---- publishes of run r (SCPB:257-290 -> schedule SCPB:398-436)
                const int pb = poff[r], pe = poff[r + 1];
                const u64 tp0 = clock64();
                for (int i0 = pb; i0 < pe; i0 += 64) {
                    const int nq = min(64, pe - i0);
                    const uint4 me = lane < nq ? pub[i0 + lane] : make_uint4(0u, OWGS_AM_EMPTY, 0u, 0u);
                    const uint32_t l_act = me.w & RES_ACT_MASK;
                    const u64 myseq = has_seq ? (lane < nq ? sq[i0 + lane] : 0ull) : seq_base + (u64)(i0 + lane);
                    const uint2 mycur = lane < nq ? pcur[i0 + lane] : make_uint2(0u, 0u);  // (staged)
                    int o_v = OWGS_NONE_V, o_f = 0;
                    // per lane (decision i0 + lane): the fields of a plain decision -- maxConcurrent == 1, a pool,
                    // memory the pool's bound U does not exclude -- and where its walk may start (the HBM cursor
                    // gathered at staging, the LDS cache; a stale cursor of the same generation is still a lower bound)
                    const int l_mem = (int)(me.y & OWGS_AM_MEM_MASK);
                    const int l_pool = (me.x & OWGS_AM_POOL) ? 1 : 0;
                    const bool l_c1 = lane < nq && !(me.y & (OWGS_AM_EMPTY | OWGS_AM_THROW)) &&
                                      ((me.y >> OWGS_AM_MAXC_SHIFT) & OWGS_AM_MAXC_MASK) <= 1u;
                    const bool l_plain = l_c1 && l_mem <= (l_pool ? U1 : U0);
                    int l_sbeg = 0;
                    if (mycur.x == gen) l_sbeg = (int)mycur.y;
                    l_sbeg = max(l_sbeg, cc_get(cc, l_act, gen));

                    // one decision alone, exact against the state now: decision q of the chunk, its walk starting no
                    // earlier than step smin (the steps before smin are known to have no room for it)
                    auto decide_one = [&](int q, int smin) {
                        const u64 ta0 = clock64();
                        ++pr_alone;
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
                            const int a = __builtin_amdgcn_readlane((int)l_act, q);
                            int s_beg = 0;
                            if (maxc <= 1) {
                                const uint32_t hg = (uint32_t)__builtin_amdgcn_readlane((int)mycur.x, q);
                                const int hs = __builtin_amdgcn_readlane((int)mycur.y, q);
                                if (mem > (pool ? U1 : U0)) {
                                    s_beg = n;  // no usable invoker has mem: every walk fails
                                    ++pr_u;
                                } else {
                                    if (hg == gen) s_beg = hs;
                                    s_beg = max(s_beg, cc_get(cc, (uint32_t)a, gen));
                                    pr_hit += s_beg > 0;
                                    s_beg = max(s_beg, smin);
                                }
                            }
                            const float rn = __builtin_amdgcn_rcpf((float)n);
                            int p = mod_fast(home + (min(s_beg, n - 1) + lane) * step, n, rn);
                            const int adv = mod_fast(64 * step, n, rn);
                            int t = -1, tix = -1, tp = 0, ts = n;  // target, its map entry, its permits, its walk step
                            uint32_t tv = 0u;
                            if (maxc <= 1) {
                                // 4 probes per lane per round (256 walk steps): the 4 permit reads are in flight together
                                for (int s0 = s_beg; s0 < n; s0 += 256) {
                                    ++pr_rounds;
                                    int pk[4], vk[4];
                                    int pp = p;
#pragma unroll
                                    for (int k = 0; k < 4; ++k) {
                                        pk[k] = pp;
                                        vk[k] = P[base + pp];
                                        pp += adv;
                                        pp -= pp >= n ? n : 0;
                                    }
                                    u64 mk[4];
#pragma unroll
                                    for (int k = 0; k < 4; ++k)
                                        mk[k] = __ballot(s0 + 64 * k + lane < n && vk[k] >= mem && vk[k] < OWGS_PLIM);
                                    const int kf = mk[0] ? 0 : mk[1] ? 1 : mk[2] ? 2 : mk[3] ? 3 : 4;
                                    if (kf < 4) {
                                        const u64 m = kf == 0 ? mk[0] : kf == 1 ? mk[1] : kf == 2 ? mk[2] : mk[3];
                                        const int L = ffs64(m);
                                        const int pl = kf == 0 ? pk[0] : kf == 1 ? pk[1] : kf == 2 ? pk[2] : pk[3];
                                        const int vl = kf == 0 ? vk[0] : kf == 1 ? vk[1] : kf == 2 ? vk[2] : vk[3];
                                        t = base + __builtin_amdgcn_readlane(pl, L);
                                        tp = __builtin_amdgcn_readlane(vl, L);
                                        ts = s0 + 64 * kf + L;
                                        break;
                                    }
                                    p = pp;
                                }
                            }
                            // concurrent: every pool position once (probes n and n + 1 repeat the first two)
                            for (int s0 = s_beg; maxc > 1 && s0 < n; s0 += 64) {
                                ++pr_rounds;
                                const bool valid = s0 + lane < n;
                                const int id = base + p;
                                // the permit count, the key's filter word and its first map block, read together
                                const uint32_t key = ct_key(id, slot);
                                const uint32_t kh = ct_hash(key);
                                const uint2 fb = bf_pos_h(kh);
                                const uint32_t fh = (kh & (OWGS_CTC / CT_BLK - 1)) * CT_BLK;  // (ct_home)
                                const int pv = valid ? P[id] : OWGS_PENC;
                                const uint32_t fw = bf[fb.x];
                                const uint4 f01 = *(const uint4*)&ct[fh], f23 = *(const uint4*)&ct[fh + 2];
                                bool ok = false;
                                int ix = -1;
                                uint32_t v = 0u;
                                if (pv < OWGS_PLIM) {  // usable: a free slot of the key's container, or memory
                                    ix = (fw & fb.y) == fb.y ? ct_lookup_after(ct, key, fh, f01, f23, &v) : -1;
                                    if (ix < 0 && ovf_on) {  // (an HBM round trip: counted)
                                        ++pr_ovf;
                                        const int oj = ovf_find(A.ovf, key, &v);
                                        ix = oj >= 0 ? OWGS_CTC + oj : -1;
                                    }
                                    ok = (v & OWGS_CT_C_MASK) != 0u || pv >= mem;
                                }
                                const u64 m = __ballot(ok);
                                if (m) {
                                    const int L = ffs64(m);
                                    t = __builtin_amdgcn_readlane(id, L);
                                    ts = s0 + L;
                                    tp = __builtin_amdgcn_readlane(pv, L);
                                    tix = __builtin_amdgcn_readlane(ix, L);
                                    tv = (uint32_t)__builtin_amdgcn_readlane((int)v, L);
                                    break;
                                }
                                p += adv;
                                p -= p >= n ? n : 0;
                            }
                            if (maxc <= 1 && lane == 0) {  // the walk's steps before ts had no room for mem
                                cc_put(cc, (uint32_t)a, gen, ts);
                                if (A.cur) A.cur[a] = make_uint2(gen, (uint32_t)ts);
                            }
                            if (maxc <= 1 && t < 0) {  // a failed walk: no usable permit count reaches mem
                                if (pool) U1 = min(U1, mem - 1);
                                else U0 = min(U0, mem - 1);
                            }
                            if (t < 0) {  // overload: a random healthy invoker, forced (SCPB:417-424)
                                const int Hn = pool ? hb_e : hm_e;
                                if (Hn > 0) {
                                    const u64 sqv = (u64)__builtin_amdgcn_readlane((int)(uint32_t)myseq, q) |
                                                    ((u64)(uint32_t)__builtin_amdgcn_readlane((int)(myseq >> 32), q) << 32);
                                    const int kk = (int)rng_index(A.rng_seed, sqv, (uint32_t)Hn);
                                    t = (pool ? full_b : full_m) ? base + kk : select_usable(base, kk);
                                    if (t < 0) {
                                        err |= OWGS_ERR_INTERNAL;
                                    } else {
                                        tp = P[t];
                                        if (maxc > 1) tix = ct_lookup2(ct, bf, A.ovf, ovf_on, ct_key(t, slot), &tv);
                                    }
                                    fl = 1;
                                }
                            }
                            x = t;
                            if (t >= 0 && lane == 0) {
                                // tryAcquireConcurrent / forceAcquireConcurrent at t (NS:32-91, FS:63-110)
                                // (permit takes are LDS atomics without a return: the next decision's reads of the
                                // same wave come after them, and nothing waits for a value)
                                bool took = true;
                                if (maxc <= 1) {
                                    atomicSub(&P[t], mem);
                                } else {
                                    const int c0 = tix >= 0 ? (int)(tv & OWGS_CT_C_MASK) : 0;
                                    const int o0 = tix >= 0 ? ct_ops(tv) : 0;
                                    const bool slot_free = c0 >= 1;  // RS.tryAcquire(1) (NS:63)
                                    took = !slot_free;
                                    if (took) atomicSub(&P[t], mem);  // a new container: its memory (NS:70-79)
                                    const int c1 = slot_free ? c0 - 1 : maxc - 1;
                                    const int o1 = o0 + 1;
                                    if (o1 > OWGS_MAX_OPS) err |= OWGS_ERR_OPS;
                                    const uint32_t nv = ct_val(c1, o1);
                                    if (tix < 0) insert(ct_key(t, slot), nv);
                                    else if (tix < OWGS_CTC) ct[tix].y = nv;
                                    else ovf_st_val(A.ovf.t, tix - OWGS_CTC, nv);
                                }
                                if (took && tp - mem < -OWGS_PLIM) err |= OWGS_ERR_PERMITS;
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
                        pr_alone_cyc += clock64() - ta0;
                    };

                    if (A.spec > 0) {
                        const u64 tsp0 = clock64();
                        // ---- speculation (pspec, cspec above), then validation in stream order
                        int sp = lane < nq ? SP_STOP : SP_NONE;
                        int sp_t = -1, sp_ts = 0;  // target, its walk step (SP_FOUND, SP_FORCED), or the step to resume
                        if (lane < nq && (me.y & (OWGS_AM_EMPTY | OWGS_AM_THROW))) {
                            sp = SP_TRIV;  // None (SCPB:288-290) or the Int.MinValue throw (SCPB:266-268)
                            o_v = (me.y & OWGS_AM_EMPTY) ? OWGS_NONE_V : OWGS_THROW_V;
                        }
                        const int l_n = l_pool ? nb : nm, l_base = l_pool ? A.n_ids - nb : 0;
                        const int l_maxc = (int)((me.y >> OWGS_AM_MAXC_SHIFT) & OWGS_AM_MAXC_MASK);
                        const bool l_cc = lane < nq && !(me.y & (OWGS_AM_EMPTY | OWGS_AM_THROW)) && l_maxc > 1;
                        const int rank = l_plain ? (int)((me.w >> RES_RANK_SHIFT) & 63u) : 0;
                        // concurrent decisions (maxConcurrent > 1) walk too; a step takes one when the invoker is usable
                        // and the key's container there has a free slot or the invoker has the memory for a new one
                        // (tryAcquireConcurrent, NS:57-82).  Only decisions of the same fqn@version key change its map
                        // entries, so the k-th decision of a key in the chunk (rank k) walks past the capacity the k
                        // before it use -- free slots, then maxConcurrent per container the memory holds -- and lands
                        // where they leave it, with the entry they leave; that holds unless the decisions before took
                        // the memory it needs, or one of its key was decided alone (then the key's later ones are too)
                        int c_ix = -1;        // the target's map entry (primary index, OWGS_CTC + overflow index, -1 none)
                        uint32_t c_nv = 0u;   // the entry's value after this decision
                        bool c_take = false;  // the decision opens a container: it takes memory (NS:70-79)
                        const u64 tm1 = clock64();
                        pr_c_match += tm1 - tsp0;
                        u64 tm2 = tm1;
                        // this chunk's concurrent decisions speculated by the helper wave right after the previous
                        // chunk was decided (against this state: taken as they are unless an overflow entry appeared,
                        // whose lookups it did not make); the plain walks run here meanwhile
                        bool pre_done = false;
                        if (pre_i0 == i0) {
                            pre_i0 = -1;
                            pre_done = true;
                            pspec(me, nq, l_sbeg, U0, U1, sp, sp_t, sp_ts, pr_rounds);
                            tm2 = clock64();
                            pr_c_pwalk += tm2 - tm1;
                            bool lost = false;
                            for (int spin = 0;; ++spin) {
                                if (__hip_atomic_load(&sc[RS_HDONE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == hreq_n)
                                    break;
                                if (spin > (1 << 26)) {  // (never expected: decide here, and no further requests)
                                    lost = true;
                                    break;
                                }
                                __builtin_amdgcn_s_sleep(1);
                            }
                            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                            if (lost) pre_live = false;
                            if (!lost && !ovf_on) {
                                ++pr_pre;
                                const uint4 h0 = hx[lane], h1 = hx[64 + lane];
                                if (l_cc) {
                                    sp = (int)h0.x;
                                    sp_t = (int)h0.y;
                                    c_ix = (int)h0.z;
                                    c_nv = h0.w;
                                    c_take = h1.x != 0u;
                                }
                                err |= (int)h1.y;
                                pr_hcyc += __builtin_amdgcn_readfirstlane(h1.w);
                            } else if (__ballot(l_cc)) {
                                int e_ = 0;
                                uint32_t n_ovf = 0u;
                                cspec(me, nq, ovf_on, cb_now, sp, sp_t, c_ix, c_nv, c_take, e_, n_ovf);
                                err |= e_;
                                pr_ovf += n_ovf;
                            }
                        }
                        if (!pre_done) {
                            // the chunk's concurrent decisions go to the helper wave (their speculation reads the state
                            // only, and every earlier change of it is published by the release below)
                            const bool hreq = hsplit && !ovf_on && __ballot(l_cc) != 0ull;
                            bool hreq_lost = false;
                            if (hreq) {
                                ++hreq_n;
                                if (lane == 0) {
                                    sc[RS_HI0] = i0;
                                    sc[RS_HNQ] = nq;
                                    sc[RS_HPRE] = 0;
                                }
                                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                                if (lane == 0)
                                    __hip_atomic_store(&sc[RS_HGO], hreq_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            }
                            pspec(me, nq, l_sbeg, U0, U1, sp, sp_t, sp_ts, pr_rounds);
                            tm2 = clock64();
                            pr_c_pwalk += tm2 - tm1;
                            if (__ballot(l_cc)) {
                                if (hreq) {  // the helper wave's answer to request hreq_n
                                    for (int spin = 0;; ++spin) {
                                        if (__hip_atomic_load(&sc[RS_HDONE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) ==
                                            hreq_n * nhelp)
                                            break;
                                        if (spin > (1 << 26)) {  // (never expected: decide here instead of waiting on)
                                            hreq_lost = true;
                                            break;
                                        }
                                        __builtin_amdgcn_s_sleep(1);
                                    }
                                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                                    if (hreq_lost) pre_live = false;
                                }
                                if (hreq && !hreq_lost) {
                                    const uint4 h0 = hx[lane], h1 = hx[64 + lane];
                                    if (l_cc) {
                                        sp = (int)h0.x;
                                        sp_t = (int)h0.y;
                                        c_ix = (int)h0.z;
                                        c_nv = h0.w;
                                        c_take = h1.x != 0u;
                                    }
                                    err |= (int)h1.y;
                                    pr_hcyc += __builtin_amdgcn_readfirstlane(h1.w);
                                } else {
                                    int e_ = 0;
                                    uint32_t n_ovf = 0u;
                                    cspec(me, nq, ovf_on, cb_now, sp, sp_t, c_ix, c_nv, c_take, e_, n_ovf);
                                    err |= e_;
                                    pr_ovf += n_ovf;
                                }
                            }
                        }
                        // a failed walk bounds the pool's usable permits below its memory (U), and the fallback's
                        // healthy invoker depends on the sequence number alone: forced now, committed in order below
                        if (sp == SP_FAIL) {
                            const int Hn = l_pool ? hb_e : hm_e;
                            if (Hn > 0) {
                                const int kk = (int)rng_index(A.rng_seed, myseq, (uint32_t)Hn);
                                sp_t = (l_pool ? full_b : full_m) ? l_base + kk : select_usable(l_base, kk);
                                sp = sp_t >= 0 ? SP_FORCED : SP_TRIV;
                                o_v = OWGS_NONE_V;
                                o_f = 1;
                                if (sp_t < 0) err |= OWGS_ERR_INTERNAL;
                                else if (l_cc) {  // forceAcquireConcurrent: a free slot of the key's container there, or memory
                                    uint32_t v = 0u;
                                    c_ix = ct_lookup2(ct, bf, A.ovf, ovf_on, ct_key(sp_t, (int)me.z), &v);
                                    const int c0 = (int)(v & OWGS_CT_C_MASK), o0 = c_ix >= 0 ? ct_ops(v) : 0;
                                    c_take = c0 == 0;
                                    c_nv = ct_val(c_take ? l_maxc - 1 : c0 - 1, o0 + 1);
                                    if (o0 + 1 > OWGS_MAX_OPS) err |= OWGS_ERR_OPS;
                                }
                            } else {
                                sp = SP_TRIV;  // no healthy invoker: None
                                o_v = OWGS_NONE_V;
                            }
                            sp_ts = l_n;
                        }
                        // (a repeat's outcome holds once the repeats before it are decided, so only the first of
                        // each action proves anything about the state at the chunk's start: the bound U, the cursor)
                        {
                            const bool fl0 = l_c1 && rank == 0 && (sp == SP_FORCED || sp == SP_TRIV);
                            U0 = min(U0, wave_min_i(fl0 && !l_pool ? l_mem - 1 : 0x7FFFFFFF));
                            U1 = min(U1, wave_min_i(fl0 && l_pool ? l_mem - 1 : 0x7FFFFFFF));
                        }
                        // every first walk's cursor (the steps before it had no room then, so none now)
                        if (l_c1 && rank == 0) {
                            const int cs = sp == SP_FOUND ? sp_ts : sp == SP_STOP ? sp_ts : l_n;
                            cc_put(cc, l_act, gen, cs);
                            if (A.cur) A.cur[l_act] = make_uint2(gen, (uint32_t)cs);
                        }
                        mv[lane] = l_mem;
                        const int tbits = 32 - __clz(max(A.n_ids - 1, 1));
                        const u64 tsp1 = clock64();
                        pr_spec_cyc += tsp1 - tsp0;
                        // ---- in stream order: the longest prefix whose speculative targets still hold commits at
                        // once; the first one that does not (or a concurrent decision, or an unfinished walk) is decided
                        // alone, then the next prefix
                        const bool c_slot = l_cc && !c_take;  // takes a free slot, no memory
                        pr_c_cwalk += clock64() - tm2;
                        for (int q = 0;;) {
                            ++pr_pass;
                            const bool cand = lane >= q && (sp == SP_FOUND || sp == SP_FORCED);
                            const bool take = cand && !c_slot;
                            bool fits = true;
                            // every candidate takes its memory at once (LDS atomics); then F = the permits left at
                            // its target after all of them: the decision holds iff F plus the takes AFTER it at the
                            // same invoker is >= 0 -- always when F >= 0; only targets that went negative need the
                            // per-invoker sums (a ballot match on the target id)
                            if (take) atomicSub(&P[sp_t], l_mem);  // tryAcquire (FS:63-71) / forceAcquire (FS:102-110)
                            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // (every lane's take before the reads)
                            const int F = take ? P[sp_t] : 0;
                            if (__ballot(take && sp == SP_FOUND && F < 0)) {
                                const bool mt = take && F < 0;
                                u64 eq = __ballot(mt);
                                for (int b = 0; b < tbits; ++b) {
                                    const bool bit = (sp_t >> b) & 1;
                                    const u64 m = __ballot(mt && bit);
                                    eq &= bit ? m : ~m;
                                }
                                eq &= ~((2ull << lane) - 1ull);  // the takes after me
                                int later = 0;
                                if (mt)
                                    while (eq) {
                                        later += mv[ffs64(eq)];
                                        eq &= eq - 1ull;
                                    }
                                fits = !mt || F + later >= 0;
                            }
                            const bool ok = lane < q || sp == SP_NONE || sp == SP_TRIV || sp == SP_FORCED ||
                                            (sp == SP_FOUND && (c_slot || fits));
                            const u64 bad = __ballot(!ok);
                            const int f = bad ? ffs64(bad) : 64;
                            if (take && lane >= f) atomicAdd(&P[sp_t], l_mem);  // the takes from the first miss on: back
                            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                            if (cand && lane < f) {
                                if (take && P[sp_t] < -OWGS_PLIM) err |= OWGS_ERR_PERMITS;  // (after the takes)
                                // the key's container at the target: a slot taken, or a new one (NS:63-79); decisions of
                                // one key at one invoker leave values whose operationCount grows with each: the largest
                                // is the last one's
                                // (signed: c | operationCount << 12 as an int orders by operationCount, which a
                                // watched pair's entry may hold below 0)
                                if (l_cc && c_ix >= 0 && c_ix < OWGS_CTC) atomicMax((int*)&ct[c_ix].y, (int)c_nv);
                                else if (l_cc && c_ix >= OWGS_CTC) atomicMax((int*)&A.ovf.t[c_ix - OWGS_CTC].y, (int)c_nv);
                                o_v = sp_t;
                                o_f = sp == SP_FORCED ? 1 : 0;
                            }
                            // entries absent at the chunk's start, one at a time in stream order (lane 0): the first
                            // decision of a key at an invoker inserts it, the later ones find it
                            const u64 ti0 = clock64();
                            u64 insm = __ballot(cand && lane < f && l_cc && c_ix < 0);
                            if (insm && !ovf_on && used + (int)__popcll(insm) < OWGS_CT_LDS_FILL) {
                                // all at once while the primary has room for every one of them: each lane walks its
                                // key's chain from its home and claims the first empty or deleted entry by CAS; lanes
                                // of one key race for the same entry, the losers find the key there and merge their
                                // value (operationCount order: atomicMax), lanes of other keys move on
                                bool fresh = false;
                                if ((insm >> lane) & 1ull) {
                                    const uint32_t key = ct_key(sp_t, (int)me.z);
                                    uint32_t h = ct_home(key);
                                    for (int p = 0; p < OWGS_CTC;) {
                                        const uint32_t k = ct[h].x;
                                        if (k == key) {
                                            atomicMax((int*)&ct[h].y, (int)c_nv);
                                            break;
                                        }
                                        if (k == 0u || k == OWGS_CT_TOMB) {
                                            const uint32_t old = atomicCAS((uint32_t*)&ct[h].x, k, key);
                                            if (old == k) {
                                                atomicMax((int*)&ct[h].y, (int)c_nv);  // (a free entry holds 0)
                                                bf_add(bf, key);
                                                fresh = k == 0u;
                                                tombs -= k == OWGS_CT_TOMB;
                                                break;
                                            }
                                            continue;  // lost the entry: read it again
                                        }
                                        h = (h + 1) & (OWGS_CTC - 1);
                                        ++p;
                                    }
                                }
                                used = __builtin_amdgcn_readfirstlane(used) + (int)__popcll(__ballot(fresh));
                                insm = 0ull;
                                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                            }
                            for (u64 ins = insm; ins; ins &= ins - 1ull) {
                                const int j = ffs64(ins);
                                const uint32_t key = ct_key(__builtin_amdgcn_readlane(sp_t, j),
                                                            __builtin_amdgcn_readlane((int)me.z, j));
                                const uint32_t nvj = (uint32_t)__builtin_amdgcn_readlane((int)c_nv, j);
                                if (lane == 0) {
                                    uint32_t v0;
                                    const int ix = ct_lookup2(ct, bf, A.ovf, ovf_on, key, &v0);
                                    const uint32_t mv0 = (uint32_t)max((int)v0, (int)nvj);  // (signed, as above)
                                    if (ix < 0) insert(key, nvj);
                                    else if (ix < OWGS_CTC) ct[ix].y = mv0;
                                    else ovf_st_val(A.ovf.t, ix - OWGS_CTC, mv0);
                                }
                                used = __builtin_amdgcn_readfirstlane(used);
                                ovf_on = __builtin_amdgcn_readfirstlane((int)ovf_on) != 0;
                                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                            }
                            pr_c_ins += clock64() - ti0;
                            pr_grp += (uint32_t)__popcll(__ballot(cand && lane < f));
                            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                            // this chunk decided: the concurrent decisions of the run's next chunk to the helper wave,
                            // which walks them against the state they will find (nothing changes it before their
                            // validation) while wave 0 writes this chunk's outputs and walks the next chunk's others
                            if (f >= nq && pre_live && i0 + 64 < pe && !ovf_on) {
                                const int ni0 = i0 + 64, nnq = min(64, pe - ni0);
                                const uint32_t ny = lane < nnq ? pub[ni0 + lane].y : OWGS_AM_EMPTY;
                                const bool ncc = !(ny & (OWGS_AM_EMPTY | OWGS_AM_THROW)) &&
                                                 ((ny >> OWGS_AM_MAXC_SHIFT) & OWGS_AM_MAXC_MASK) > 1u;
                                if (__ballot(ncc)) {
                                    ++hreq_n;
                                    if (lane == 0) {
                                        sc[RS_HI0] = ni0;
                                        sc[RS_HNQ] = nnq;
                                        sc[RS_HPRE] = 1;
                                    }
                                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                                    if (lane == 0)
                                        __hip_atomic_store(&sc[RS_HGO], hreq_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                                    pre_i0 = ni0;
                                }
                            }
                            if (f >= nq) {
                                pr_val_cyc += clock64() - tsp1;
                                break;
                            }
                            decide_one(f, __builtin_amdgcn_readlane(sp_ts, f));
                            if (__builtin_amdgcn_readlane((int)l_cc, f)) {  // the key's later decisions assumed its
                                const uint32_t zf = (uint32_t)__builtin_amdgcn_readlane((int)me.z, f);  // prediction
                                if (lane > f && l_cc && me.z == zf) sp = SP_STOP;
                            }
                            q = f + 1;
                        }
                    } else {
                        for (int q = 0; q < nq; ++q) {
                            // ---- up to 4 consecutive plain decisions walk together, 16 lanes each (4 probes per lane:
                            // 64 walk steps per round), against the state before all of them; then in stream order
                            // each is exact unless an earlier one of the group took the room at its target (permits
                            // only fall inside a run, so every step a walk passed is still full).  The first one that
                            // is not exact, and every fallback, goes to the single-decision path.
                            const u64 npm = ~(__ballot(l_plain) >> q);
                            const int g = npm ? min(__builtin_ctzll(npm), 4) : 4;
                            if (g >= 2) {
                                const int grp = lane >> 4, u = lane & 15;
                                const bool gact = grp < g;
                                const int dq = q + (gact ? grp : 0);
                                const uint32_t gmx = (uint32_t)__shfl((int)me.x, dq, 64);
                                const int gmem = __shfl(l_mem, dq, 64), gsb = __shfl(l_sbeg, dq, 64);
                                const int ghome = (int)(gmx & OWGS_AM_POS_MASK), gstep = (int)((gmx >> 15) & OWGS_AM_POS_MASK);
                                const int gpool = (gmx & OWGS_AM_POOL) ? 1 : 0;
                                const int gn = gpool ? nb : nm, gbase = gpool ? A.n_ids - nb : 0;
                                const float grn = __builtin_amdgcn_rcpf((float)gn);
                                int gp = mod_fast(ghome + (gsb + u) * gstep, gn, grn);
                                const int gadv = mod_fast(16 * gstep, gn, grn);
                                int gs = gsb, gt = -1, gts = gn, gpv = 0;
                                bool gdone = !gact || gs >= gn;
                                while (__ballot(!gdone)) {
                                    ++pr_rounds;
                                    int pk[4], vk[4];
                                    int pp = gp;
#pragma unroll
                                    for (int k = 0; k < 4; ++k) {
                                        pk[k] = pp;
                                        vk[k] = P[gbase + pp];
                                        pp += gadv;
                                        pp -= pp >= gn ? gn : 0;
                                    }
                                    u64 B[4];
#pragma unroll
                                    for (int k = 0; k < 4; ++k)
                                        B[k] = __ballot(!gdone & (gs + 16 * k + u < gn) & (vk[k] >= gmem) & (vk[k] < OWGS_PLIM));
                                    int kf = 4, L = 0, sp = pk[0], sv = vk[0];
#pragma unroll
                                    for (int k = 3; k >= 0; --k) {  // this group's first hit in walk order (k, then lane)
                                        const uint32_t m = (uint32_t)(B[k] >> (16 * grp)) & 0xFFFFu;
                                        if (m) {
                                            kf = k;
                                            L = __builtin_ctz(m);
                                            sp = pk[k];
                                            sv = vk[k];
                                        }
                                    }
                                    const int src = (grp << 4) + L;
                                    const int hp = __shfl(sp, src, 64), hv = __shfl(sv, src, 64);
                                    if (!gdone) {
                                        if (kf < 4) {
                                            gt = gbase + hp;
                                            gpv = hv;
                                            gts = gs + 16 * kf + L;
                                            gdone = true;
                                        } else {
                                            gs += 64;
                                            gp = pp;
                                            gdone = gs >= gn;  // every pool position probed: the walk failed
                                        }
                                    }
                                }
                                // in stream order: accept while exact
                                int ge = 0, at0 = -1, at1 = -1, at2 = -1, am0 = 0, am1 = 0, am2 = 0;
#pragma unroll
                                for (int k = 0; k < 4; ++k) {
                                    if (k >= g || ge < k) break;
                                    const int tk = __builtin_amdgcn_readlane(gt, 16 * k);
                                    const int pvk = __builtin_amdgcn_readlane(gpv, 16 * k);
                                    const int tsk = __builtin_amdgcn_readlane(gts, 16 * k);
                                    const int memk = __builtin_amdgcn_readlane(l_mem, q + k);
                                    const int ak = __builtin_amdgcn_readlane((int)l_act, q + k);
                                    const int pk_ = (__builtin_amdgcn_readlane((int)me.x, q + k) & OWGS_AM_POOL) ? 1 : 0;
                                    if (tk < 0) {  // no room anywhere for memk (then, so now): cursor past the pool, U below memk
                                        const int nk = pk_ ? nb : nm;
                                        if (lane == 0) cc_put(cc, (uint32_t)ak, gen, nk);
                                        if (pk_) U1 = min(U1, memk - 1);
                                        else U0 = min(U0, memk - 1);
                                        break;
                                    }
                                    int room = pvk;
                                    if (k > 0 && at0 == tk) room -= am0;
                                    if (k > 1 && at1 == tk) room -= am1;
                                    if (k > 2 && at2 == tk) room -= am2;
                                    if (room < memk) break;  // an earlier decision of the group took it: decide again
                                    if (k == 0) { at0 = tk; am0 = memk; }
                                    if (k == 1) { at1 = tk; am1 = memk; }
                                    if (k == 2) { at2 = tk; am2 = memk; }
                                    if (lane == 0) {
                                        atomicSub(&P[tk], memk);  // tryAcquire (FS:63-71)
                                        cc_put(cc, (uint32_t)ak, gen, tsk);
                                        if (A.cur) A.cur[ak] = make_uint2(gen, (uint32_t)tsk);
                                    }
                                    if (lane == q + k) {
                                        o_v = tk;
                                        o_f = 0;
                                    }
                                    ++ge;
                                }
                                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                                if (ge > 0) {
                                    pr_grp += ge;
                                    q += ge - 1;
                                    continue;
                                }
                            }
                            decide_one(q, 0);
                        }
                    }
                    pr_dec += nq;
                    if (lane < nq) {
                        out_inv[i0 + lane] = o_v;
                        out_fl[i0 + lane] = (uint8_t)o_f;
                    }
                    // Z marks (watched pairs): a concurrent decision's walk tried every usable invoker before the step
                    // it took -- all of them before an overload fallback -- and a failed try leaves the reference an
                    // empty entry (getOrElseUpdate, NS:61-62).  Per action its deepest walk of the run goes into the
                    // watched-walk list (wl); at the run's end (w_flush, before the next run's releases) every entry
                    // marks the watched pairs of its key at the steps before
                    if (A.w.cap > 0) {
                        const int wmx = (int)((me.y >> OWGS_AM_MAXC_SHIFT) & OWGS_AM_MAXC_MASK);
                        const bool wd = lane < nq && !(me.y & (OWGS_AM_EMPTY | OWGS_AM_THROW)) && wmx > 1 && o_v >= 0 &&
                                        wf_test(wf, me.z & 0x1FFFFu);
                        if (__ballot(wd)) {
                            int depth = 0;
                            if (wd) {
                                const int wpool = (me.x & OWGS_AM_POOL) ? 1 : 0;
                                const int wn = wpool ? nb : nm, wbase = wpool ? A.n_ids - nb : 0;
                                const int whome = (int)(me.x & OWGS_AM_POS_MASK), wstep = (int)((me.x >> 15) & OWGS_AM_POS_MASK);
                                if (o_f & 1) {
                                    depth = 0x7FFFFFFF;  // n + 2 failed probes, then the forced acquire (SCPB:417-424)
                                } else if (wn > 1) {
                                    const int d = (o_v - wbase - whome + wn) % wn;
                                    depth = (int)(((long long)d * res_inv_mod(wstep % wn, wn)) % wn);
                                }
                            }
                            for (u64 bb = __ballot(wd && depth > 0); bb;) {  // one entry per action: its deepest walk
                                const int q = ffs64(bb);
                                const uint32_t aq = (uint32_t)__builtin_amdgcn_readlane((int)l_act, q);
                                const bool in_g = wd && depth > 0 && l_act == aq;
                                const int dd = wave_max_i(in_g ? depth : -1);
                                bb &= ~__ballot(in_g);
                                const int nl = sc[RS_WLN];
                                const u64 hit = __ballot((lane < nl && wl[lane].x == aq) ||
                                                         (lane + 64 < nl && wl[lane + 64].x == aq));
                                if (hit) {
                                    const int h = ffs64(hit);
                                    const int j = wl[h].x == aq ? h : h + 64;
                                    if (lane == 0) wl[j].y = (uint32_t)max((int)wl[j].y, dd);
                                } else {
                                    if (nl >= RES_WL) {
                                        w_flush();
                                    }
                                    if (lane == 0) {
                                        const int j = sc[RS_WLN];
                                        wl[j] = make_uint2(aq, (uint32_t)dd);
                                        sc[RS_WLN] = j + 1;
                                    }
                                }
                                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                            }
                        }
                    }
                }
                if (A.w.cap > 0) w_flush();
                pr_pub += clock64() - tp0;
            }
            // the call's releases may have raised permits: the range bound grows by what they returned at most
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) err |= __shfl_xor(err, d, 64);
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) pr_ovf += __shfl_xor(pr_ovf, d, 64);
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) tombs += __shfl_xor(tombs, d, 64);
            if (lane == 0 && !smode) {
                int32_t* pr = A.ctl + OWGS_RES_PROF;
                st_sys(pr + 0, (int)pr_rounds);
                st_sys(pr + 1, (int)pr_dec);
                st_sys(pr + 2, (int)min(pr_stage, (u64)0x7FFFFFFF));
                st_sys(pr + 3, (int)min(pr_rel, (u64)0x7FFFFFFF));
                st_sys(pr + 4, (int)min(pr_pub, (u64)0x7FFFFFFF));
                st_sys(pr + 5, (int)pr_ovf);
                st_sys(pr + 6, (int)pr_hit);
                st_sys(pr + 7, (int)pr_u);
                st_sys(pr + 8, (int)pr_grp);
                st_sys(pr + 9, (int)pr_pass);
                st_sys(pr + 10, (int)pr_alone);
                st_sys(pr + 11, (int)min(pr_alone_cyc, (u64)0x7FFFFFFF));
                st_sys(pr + 12, (int)min(pr_spec_cyc, (u64)0x7FFFFFFF));
                st_sys(pr + 13, (int)min(pr_val_cyc, (u64)0x7FFFFFFF));
                st_sys(pr + 14, (int)min(pr_c_match, (u64)0x7FFFFFFF));
                st_sys(pr + 15, (int)min(pr_c_pwalk, (u64)0x7FFFFFFF));
                st_sys(pr + 16, (int)min(pr_c_cwalk, (u64)0x7FFFFFFF));
                st_sys(pr + 17, (int)min(pr_c_ins, (u64)0x7FFFFFFF));
                st_sys(pr + 18, (int)min(pr_c_relc, (u64)0x7FFFFFFF));
                st_sys(pr + 19, (int)pr_pre);
                st_sys(pr + 20, (int)min(pr_hcyc, (u64)0x7FFFFFFF));
                st_sys(&A.ctl[OWGS_RES_GEN], (int)gen);
            } else if (lane == 0 && A.s_stats) {  // stream mode: summed over the launch (owgs_resident_stats' order)
                A.s_stats[0] += pr_rounds;
                A.s_stats[1] += pr_dec;
                A.s_stats[2] += pr_stage;
                A.s_stats[3] += pr_rel;
                A.s_stats[4] += pr_pub;
                A.s_stats[5] += (uint32_t)pr_ovf;
                A.s_stats[6] += pr_hit;
                A.s_stats[7] += pr_u;
                A.s_stats[8] += pr_grp;
                A.s_stats[9] += pr_pass;
                A.s_stats[10] += pr_alone;
                A.s_stats[11] += pr_alone_cyc;
                A.s_stats[12] += pr_spec_cyc;
                A.s_stats[13] += pr_val_cyc;
                A.s_stats[14] += pr_c_match;
                A.s_stats[15] += pr_c_pwalk;
                A.s_stats[16] += pr_c_cwalk;
                A.s_stats[17] += pr_c_ins;
                A.s_stats[18] += pr_c_relc;
                A.s_stats[19] += pr_pre;
                A.s_stats[20] += pr_hcyc;
            }
            if (lane == 0) {
                sc[RS_USED] = used;
                sc[RS_TOMB] += tombs;
                sc[RS_U0] = U0;
                sc[RS_U1] = U1;
                sc[RS_GEN] = gen;
                const long long mp = (long long)sc[RS_MAXP] + (long long)rsum;
                sc[RS_MAXP] = (int)min(mp, (long long)0x7FFFFFFF);
                if (err) atomicOr(&sc[RS_ERR], err);
            }
            if (hsplit) {  // the call's decisions are done: the helper wave leaves its loop
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                if (lane == 0) __hip_atomic_store(&sc[RS_HGO], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        } else if (bail == 0 && wave >= 1 && wave <= nhelp) {
            // ---- helper wave: speculates the concurrent decisions of the chunk wave 0 posts (request k), answers k
            for (int expect = 1;; ++expect) {
                int go = 0;
                for (int spin = 0;; ++spin) {
                    go = __hip_atomic_load(&sc[RS_HGO], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (go < 0 || go >= expect) break;
                    if (spin > (1 << 26)) {  // (bounded: wave 0 decides by itself past its own bound)
                        go = -2;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (go < 0) break;
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                const int hi0 = sc[RS_HI0], hnq = sc[RS_HNQ];
                const bool mine = lane % max(nhelp, 1) == wave - 1;  // (the lanes of the other helper waves: skipped)
                const uint4 me = lane < hnq && mine ? pub[hi0 + lane] : make_uint4(0u, OWGS_AM_EMPTY, 0u, 0u);
                int sp = SP_STOP, sp_t = -1, c_ix = -1, e_ = 0;
                uint32_t c_nv = 0u, n_ovf = 0u;
                bool c_take = false;
                const u64 th0 = clock64();
                cspec(me, hnq, false, sc[RS_HPRE] ? cb_pre : cb_now, sp, sp_t, c_ix, c_nv, c_take, e_, n_ovf);
                const uint32_t th = (uint32_t)min(clock64() - th0, (u64)0x7FFFFFFF);  // (its walk's cycles)
                if (mine) {
                    hx[lane] = make_uint4((uint32_t)sp, (uint32_t)sp_t, (uint32_t)c_ix, c_nv);
                    hx[64 + lane] = make_uint4(c_take ? 1u : 0u, (uint32_t)e_, n_ovf, th);
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                if (lane == 0) atomicAdd(&sc[RS_HDONE], 1);  // (wave 0 waits for nhelp answers per request)
            }
        }
        __syncthreads();
        // ---- primary-table cleanup between calls: deleted entries keep chains long and fill the primary
        if (sc[RS_USED] > RES_CLEAN_USED && sc[RS_TOMB] >= RES_CLEAN_TOMBS) {  // (uniform) enough deleted entries
            {
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
                const int nlive = sc[RS_LIVE];
                for (int i = tid; i < OWGS_CTC; i += 256) ct[i] = make_uint2(0u, 0u);
                for (int i = tid; i < RES_BF; i += 256) bf[i] = 0u;
                __syncthreads();
                for (int j = tid; j < nlive; j += 256) {  // distinct keys into an empty table: claim by CAS
                    const uint32_t kk = A.ct_tmp[2 * j], vv = A.ct_tmp[2 * j + 1];
                    uint32_t h = ct_home(kk);
                    for (int p = 0; p < OWGS_CTC; ++p) {
                        if (atomicCAS((uint32_t*)&ct[h], 0u, kk) == 0u) {
                            ct[h].y = vv;
                            bf_add(bf, kk);
                            break;
                        }
                        h = (h + 1) & (OWGS_CTC - 1);
                    }
                }
                if (tid == 0) {
                    sc[RS_USED] = nlive;
                    sc[RS_TOMB] = 0;
                }
                __syncthreads();
            }
        }
        if (smode) {  // ---- stream mode: the outputs into the stream's arrays; an error or a refusal ends the replay
            if (bail == 0) {
                const int32_t* oi = (const int32_t*)(stg + s_out);
                for (int i = tid; i < NP; i += 256) {
                    A.s_out_inv[s_first + i] = oi[i];
                    A.s_out_fl[s_first + i] = (uint8_t)stg[s_ofl + i];
                }
                if (A.s_rel_fl)
                    for (int j = tid; j < NR; j += 256) A.s_rel_fl[s_first + j] = (uint8_t)stg[s_orf + j];
            }
            __threadfence();  // (the next piece's releases read these decisions through L2)
            __syncthreads();
            const int e = sc[RS_ERR] | (bail ? OWGS_ERR_RELRISK : 0);
            __syncthreads();
            if (e) {
                if (tid == 0) atomicOr(A.err, e);
                break;
            }
            continue;
        }
        // ---- answer: the outputs to host memory (16-byte stores), then the result and the done word
        if (bail == 0) {
            for (uint32_t o = 16u * tid; o < s_end - s_out; o += 16u * 256u)
                *(uint4*)(A.out + o) = *(const uint4*)(stg + s_out + o);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // every wave's output stores are done (system scope) ...
        __syncthreads();                               // ... before thread 0 answers
        if (tid == 0) {
            const int e = sc[RS_ERR];  // (reported in the result word, not the context's error word)
            sc[RS_ERR] = 0;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            st_sys(&A.ctl[OWGS_RES_RESULT], bail | (e << 8));
            st_sys(&A.ctl[OWGS_RES_USED], sc[RS_USED]);
            st_sys(&A.ctl[OWGS_RES_TOMBS], sc[RS_TOMB]);
            if (A.w.cap > 0)
                st_sys(&A.ctl[OWGS_RES_WLIVE], __hip_atomic_load(A.w.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
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
    if (tid == 0 && !smode) {
        st_sys(&A.ctl[OWGS_RES_WHY], why);
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
        hipError_t e = hipFuncSetAttribute((const void*)owgs_resident_kernel<false>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, OWGS_LDS_BYTES);
        if (e == hipSuccess)
            e = hipFuncSetAttribute((const void*)owgs_resident_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    OWGS_LDS_BYTES);
        if (e != hipSuccess) return e;
        attr = true;
    }
    if (lds_bytes > OWGS_LDS_BYTES || a->n_slots > OWGS_MAX_SLOTS_CT) return hipErrorInvalidValue;
    if (a->smode) hipLaunchKernelGGL(owgs_resident_kernel<true>, dim3(1), dim3(256), lds_bytes, s, *a);
    else hipLaunchKernelGGL(owgs_resident_kernel<false>, dim3(1), dim3(256), lds_bytes, s, *a);
    return hipGetLastError();
}
