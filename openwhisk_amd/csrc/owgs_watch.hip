// owgs_watch.hip -- the reference's empty NestedSemaphore entries after a slot-state reset.
//
// NestedSemaphore.tryOrForceAcquireConcurrent (NestedSemaphore.scala:57-82) runs getOrElseUpdate (:61-62) before
// its tryAcquire, so a failed concurrent try leaves an entry {permits 0, operationCount 0} behind.  The engine
// creates entries only when an acquisition succeeds.  An empty entry and an absent one acquire alike; they differ
// only for a release that finds no entry of its own acquisition: the reference's releaseConcurrent (NS:98-113)
// applies RS.release(1, true) to the empty entry (no memory back, one free container slot, operationCount -1), where
// an absent entry throws NoSuchElementException (NS:103).  Such releases exist only after updateCluster
// (SCPB:561-584) threw away the entries of activations still in flight.  So the engine tracks exactly those pairs:
//
//   d[p] = in-flight activations of (invoker, fqn) p - operationCount of p's entry (0 when absent), W = {p : d > 0}
//
// d changes at a reset (d = ops + d_old for every pair; owgs_w_rebuild_kernel) and when a release of a watched pair
// throws NoSuchElement (d - 1; owgs_release_seq_kernel).  Z[p] (the reference holds an empty entry for p) is set
// after each publish run for watched pairs absent from the table whose invoker a decision of their fqn tried and
// failed (its walk passed the usable invoker before the step it took; every step before an overload fallback:
// owgs_w_depth/list/mark kernels), and cleared when p's entry is removed.  tests/watch_model.py restates the rules;
// tests/test_watch_model.py checks them against the literal oracle.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "owgs_internal.h"
#include "owgs_table.h"

// ------------------------------------------------------------------------------------------------ reset
// one thread per candidate: primary entries [0, CTC), overflow entries [CTC, CTC + ovf.cap), old watched pairs after
__global__ __launch_bounds__(256) void owgs_w_rebuild_kernel(OwgsWRebuildArgs a) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t n_ovf = a.ovf.cap > 0 ? a.ovf.cap : 0;
    uint32_t key = 0u;
    int t = 0;
    if (i < OWGS_CTC + n_ovf) {
        uint32_t v;
        if (i < OWGS_CTC) {
            key = a.ct_keys[i];
            v = a.ct_vals[i];
        } else {
            const uint2 e = ovf_ld(a.ovf.t, (int)(i - OWGS_CTC));
            key = e.x;
            v = e.y;
        }
        if (key == 0u || key == OWGS_CT_TOMB) return;
        const int wj = w_find(a.old_w, key);
        t = ct_ops(v) + (wj >= 0 ? (int)(a.old_w.vals[wj] & ~OWGS_W_Z) : 0);  // in flight = ops + d
    } else {
        const int64_t j = i - OWGS_CTC - n_ovf;
        if (j >= a.old_w.cap) return;
        key = a.old_w.keys[j];
        if (key == 0u || key == OWGS_CT_TOMB) return;
        // pairs with an entry were counted above
        if (ct_find(a.ct_keys, key) >= 0) return;
        uint32_t v;
        if (a.ovf.cap > 0 && ovf_find(a.ovf, key, &v) >= 0) return;
        t = (int)(a.old_w.vals[j] & ~OWGS_W_Z);
    }
    if (t <= 0) return;
    if (w_insert(a.new_w, key, (uint32_t)t) >= 0) {
        atomicAdd(a.new_w.cnt, 1);
        atomicAdd(&a.new_w.wkey[key >> OWGS_CT_SLOT_SHIFT], 1);
    }
}

// ------------------------------------------------------------------------------------------------ publish runs
__device__ __forceinline__ int gcd_i(int a, int b) {
    while (b) {
        const int t = a % b;
        a = b;
        b = t;
    }
    return a;
}
// x^-1 mod n for gcd(x, n) == 1 (extended Euclid)
__device__ __forceinline__ int inv_mod(int x, int n) {
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

struct WalkRef {
    int pool, home, step, n;
};
__device__ __forceinline__ WalkRef walk_of(const OwgsWUpdateArgs& A, uint32_t mx) {
    WalkRef w;
    w.pool = (int)((mx >> 30) & 1u);
    w.home = (int)(mx & OWGS_AM_POS_MASK);
    w.step = (int)((mx >> 15) & OWGS_AM_POS_MASK);
    w.n = w.pool ? A.nb : A.nm;
    return w;
}
// pool word at position pos: id (usable), OWGS_PW_UNUSABLE, OWGS_PW_BADID
__device__ __forceinline__ int pool_word(const OwgsWUpdateArgs& A, int pool, int pos) {
    return A.pool_words[pool ? A.nm + pos : pos];
}
// walk step at which the walk first reaches a usable position holding invoker `inv` (n + 2 when it never does)
__device__ int step_of(const OwgsWUpdateArgs& A, const WalkRef& w, int inv) {
    if (w.n <= 0) return 0x7FFFFFFF;
    if (A.pool_mode == 0) {  // identity pools: position p holds id p (managed) or n_ids - nb + p (blackbox)
        const int pos = w.pool ? inv - (A.n_ids - A.nb) : inv;
        if (pos < 0 || pos >= w.n) return 0x7FFFFFFF;
        if (!((A.usable[inv >> 5] >> (inv & 31)) & 1u)) return 0x7FFFFFFF;
        const int st = w.step % w.n;
        if (gcd_i(st == 0 ? w.n : st, w.n) == 1) {
            const int d = (pos - w.home + w.n) % w.n;
            return (int)(((long long)d * inv_mod(st, w.n)) % w.n);
        }
    }
    int idx = w.home;  // explicit pools (ids may repeat) or a step that shares a factor with n: scan the walk
    if (A.pool_mode == 0) {
        // identity pools: position -> id is arithmetic and usability is the bitmap (kept current by
        // owgs_update_health_device, which does not rebuild pool_words on this path)
        const int pos = w.pool ? inv - (A.n_ids - A.nb) : inv;
        for (int s = 0; s < w.n + 2; ++s) {
            if (idx == pos) return s;
            idx = (int)(((long long)idx + w.step) % w.n);
        }
        return 0x7FFFFFFF;
    }
    for (int s = 0; s < w.n + 2; ++s) {
        if (pool_word(A, w.pool, idx) == inv) return s;
        idx = (int)(((long long)idx + w.step) % w.n);
    }
    return 0x7FFFFFFF;
}

// per decision of a watched fqn: how deep its walk tried and failed (SCPB:398-436): the step it took (every earlier
// usable step failed a try), n + 2 for an overload fallback, the throwing step for an id outside the slots
__global__ __launch_bounds__(256) void owgs_w_depth_kernel(OwgsWUpdateArgs A) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= A.n) return;
    const int a = A.act ? A.act[i] : -1;
    const uint2 m = A.act ? A.act_meta[a] : A.xmeta[i];
    const int slot = A.act ? A.act_slot[a] : A.xslot[i];
    const int maxc = (int)((m.y >> OWGS_AM_MAXC_SHIFT) & OWGS_AM_MAXC_MASK);
    if (maxc <= 1 || (m.y & (OWGS_AM_THROW | OWGS_AM_EMPTY))) return;  // no concurrency map / no try at all
    if (A.w.wkey[slot] <= 0) return;
    const int out = A.out_inv[i];
    const WalkRef w = walk_of(A, m.x);
    int depth;
    if (A.out_flags[i] & 1u) {
        depth = w.n + 2;  // n + 2 failed probes, then the forced acquire (SCPB:417-424)
    } else if (out >= 0) {
        depth = step_of(A, w, out) + 1;
        if (depth > w.n + 2) depth = w.n + 2;
    } else if (out == OWGS_THROW_V) {  // explicit pools: the first usable id outside invokerSlots (SCPB:413)
        depth = w.n + 2;
        int idx = w.home;
        for (int s = 0; s < w.n + 2; ++s) {
            if (pool_word(A, w.pool, idx) == OWGS_PW_BADID) {
                depth = s;
                break;
            }
            idx = (int)(((long long)idx + w.step) % w.n);
        }
    } else {
        return;  // None: no usable invoker was tried
    }
    if (depth <= 0) return;
    if (A.act) {
        if (atomicMax(&A.D[a], depth) == 0) A.L[atomicAdd(&A.Lcnt[0], 1)] = a;
    } else {
        A.L2[atomicAdd(&A.Lcnt[1], 1)] = make_uint4(m.x, (uint32_t)slot, (uint32_t)depth, 0u);
    }
}

// registered actions: one walk per listed action at its deepest step; D back to zero
__global__ __launch_bounds__(256) void owgs_w_list_kernel(OwgsWUpdateArgs A) {
    const int n = A.Lcnt[0];
    for (int j = blockIdx.x * 256 + threadIdx.x; j < n; j += gridDim.x * 256) {
        const int a = A.L[j];
        A.L2[j] = make_uint4(A.act_meta[a].x, (uint32_t)A.act_slot[a], (uint32_t)A.D[a], 0u);
        A.D[a] = 0;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) A.Lcnt[1] = n;
}

// per watched pair, absent from the table and without Z: did a listed walk of its fqn pass its invoker?
__global__ __launch_bounds__(256) void owgs_w_mark_kernel(OwgsWUpdateArgs A) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= A.w.cap) return;
    const uint32_t key = A.w.keys[j];
    if (key == 0u || key == OWGS_CT_TOMB) return;
    const uint32_t v = A.w.vals[j];
    if (v & OWGS_W_Z) return;
    if (ct_find(A.ct_keys, key) >= 0) return;  // an entry exists: Z is irrelevant until it is removed
    uint32_t ov;
    if (A.ovf.cap > 0 && ovf_find(A.ovf, key, &ov) >= 0) return;
    const int inv = (int)(key & 0x7FFFu) - 1, slot = (int)(key >> OWGS_CT_SLOT_SHIFT);
    const int nl = A.Lcnt[1];
    for (int q = 0; q < nl; ++q) {
        const uint4 e = A.L2[q];
        if ((int)e.y != slot) continue;
        const WalkRef w = walk_of(A, e.x);
        if (step_of(A, w, inv) < (int)e.z) {
            A.w.vals[j] = v | OWGS_W_Z;
            return;
        }
    }
}

// releases of one batch of a replay in watch mode: (invoker, limits, key) of each released activation
__global__ __launch_bounds__(256) void owgs_w_relgather_kernel(const int64_t* rel_aid, int32_t n, const int32_t* out_inv,
                                                               const int32_t* act, const int32_t* act_mem,
                                                               const int32_t* act_maxc, const int32_t* act_slot,
                                                               int32_t* inv, int32_t* mem, int32_t* maxc, int32_t* slot) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    const int64_t aid = rel_aid[r];
    const int a = act[aid];
    inv[r] = out_inv[aid];
    mem[r] = act_mem[a];
    maxc[r] = act_maxc[a];
    slot[r] = act_slot[a];
}

// ------------------------------------------------------------------------------------------------ launchers
extern "C" hipError_t owgs_launch_w_rebuild(const OwgsWRebuildArgs* a, hipStream_t s) {
    const int64_t n = (int64_t)OWGS_CTC + (a->ovf.cap > 0 ? a->ovf.cap : 0) + (a->old_w.cap > 0 ? a->old_w.cap : 0);
    hipLaunchKernelGGL(owgs_w_rebuild_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, *a);
    return hipGetLastError();
}

extern "C" hipError_t owgs_launch_w_update(const OwgsWUpdateArgs* a, hipStream_t s) {
    if (a->n <= 0 || a->w.cap <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(a->Lcnt, 0, 2 * sizeof(int32_t), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(owgs_w_depth_kernel, dim3((unsigned)((a->n + 255) / 256)), dim3(256), 0, s, *a);
    if (a->act) hipLaunchKernelGGL(owgs_w_list_kernel, dim3(std::min(64, (a->n + 255) / 256)), dim3(256), 0, s, *a);
    hipLaunchKernelGGL(owgs_w_mark_kernel, dim3((unsigned)((a->w.cap + 255) / 256)), dim3(256), 0, s, *a);
    return hipGetLastError();
}

extern "C" hipError_t owgs_launch_w_relgather(const int64_t* rel_aid, int32_t n, const int32_t* out_inv,
                                              const int32_t* act, const int32_t* act_mem, const int32_t* act_maxc,
                                              const int32_t* act_slot, int32_t* inv, int32_t* mem, int32_t* maxc,
                                              int32_t* slot, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(owgs_w_relgather_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, rel_aid, n, out_inv,
                       act, act_mem, act_maxc, act_slot, inv, mem, maxc, slot);
    return hipGetLastError();
}
