// owgs_state.hip -- device side of the shard-state updates.
//
// updateInvokers (SCPB:512-551) and updateCluster (SCPB:561-584) rebuild the per-pool step-size tables and the slot
// permits.  The reference recomputes pairwiseCoprimeNumbersUntil (SCPB:379-384) with an O(x * k) fold of gcds
// (x = 9000 managed invokers -> 1115 kept values, ~10M gcds) whenever the invoker count changes, and re-creates
// every NestedSemaphore with getInvokerSlot(userMemory).toMB (SCPB:485-499) on a cluster-size change.  Here:
//
//   owgs_coprime_kernel  one workgroup per pool.  The greedy fold keeps exactly {1} and the primes p <= x with
//                        p !| x: a kept composite would share its smallest prime factor q < c with a kept q, or
//                        (q | x) fail gcd(c, x) == 1; a prime p passes the pairwise test because every kept value
//                        below it is 1 or a smaller prime, and passes gcd(p, x) == 1 iff p !| x.  So the kernel
//                        sieves [2, x] in LDS (one bit per number, 64 KB: pools up to 524,287 positions; multiples of
//                        every prime <= sqrt(x) marked by all threads with LDS atomics), keeps c == 1 or (prime,
//                        x % c != 0), and compacts in ascending order with a
//                        block scan -- the fold's output order.  The restatement the tests compare against is the
//                        literal fold (oracle/owsched_oracle.c:owo_pairwise_coprime).
//   owgs_slots_kernel    permits[i] = toMB(max(MIN_MEMORY, userMemory_i / clusterSize)) for i in [from, n)
//                        (Size.scala:70, 97-99: integer byte division, then bytes / 2^20), one thread per invoker.
//   owgs_usable_kernel   the usable bitmap (InvokerState.isUsable, ISUP:54-59: only Healthy) from the status bytes,
//                        one thread per 32-bit word.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "owgs_internal.h"

#define CP_TPB 1024
#define CP_MAX 524287  // LDS flag bits (64 KB): the on-chip engines take pools up to 32767 positions, the large-state
                      // engine (owgs_seq.hip) the rest

__global__ __launch_bounds__(CP_TPB) void owgs_coprime_kernel(const int32_t* xs, int32_t* out, int32_t out_stride,
                                                              int32_t* counts) {
    __shared__ uint32_t comp[(CP_MAX + 1) / 32];  // bit c: c is composite
    __shared__ int32_t wsum[CP_TPB / 64];
    const int x = xs[blockIdx.x];
    int32_t* o = out + (size_t)blockIdx.x * out_stride;
    const int t = threadIdx.x;
    if (x <= 0) {  // (1 to x) is empty
        if (t == 0) counts[blockIdx.x] = 0;
        return;
    }
    for (int i = t; i <= (x >> 5); i += CP_TPB) comp[i] = 0u;
    __syncthreads();
    // mark composites: every prime p <= sqrt(x) (found by trial division, uniform over the block) strikes its
    // multiples from p * p; concurrent stores write the same value
    for (int p = 2; p * p <= x; ++p) {
        bool prime = true;
        for (int d = 2; d * d <= p; ++d)
            if (p % d == 0) {
                prime = false;
                break;
            }
        if (!prime) continue;
        for (int m = p * p + t * p; m <= x; m += CP_TPB * p) atomicOr(&comp[m >> 5], 1u << (m & 31));
    }
    __syncthreads();
    // each thread owns a contiguous run of candidates so the block scan yields ascending output positions
    const int per = (x + CP_TPB - 1) / CP_TPB;
    const int lo = 1 + t * per;
    const int hi = min(x, lo + per - 1);
    int cnt = 0;
    auto keep = [&](int c) { return c == 1 || (!((comp[c >> 5] >> (c & 31)) & 1u) && x % c != 0); };
    for (int c = lo; c <= hi; ++c) cnt += keep(c);
    // block exclusive scan of cnt
    int v = cnt;
    const int lane = t & 63, w = t >> 6;
    for (int d = 1; d < 64; d <<= 1) {
        int u = __shfl_up(v, d, 64);
        if (lane >= d) v += u;
    }
    if (lane == 63) wsum[w] = v;
    __syncthreads();
    if (w == 0) {
        int s = lane < CP_TPB / 64 ? wsum[lane] : 0;
        for (int d = 1; d < CP_TPB / 64; d <<= 1) {
            int u = __shfl_up(s, d, 64);
            if (lane >= d) s += u;
        }
        if (lane < CP_TPB / 64) wsum[lane] = s;  // inclusive wave totals
    }
    __syncthreads();
    int pos = v - cnt + (w ? wsum[w - 1] : 0);
    for (int c = lo; c <= hi; ++c)
        if (keep(c)) o[pos++] = c;
    if (t == CP_TPB - 1) counts[blockIdx.x] = pos;
}

__global__ __launch_bounds__(256) void owgs_slots_kernel(const int64_t* mem_bytes, int32_t from, int32_t n,
                                                         int32_t cluster, int64_t min_bytes, int32_t* permits) {
    const int i = from + blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    int64_t shard = mem_bytes[i] / cluster;  // ByteSize./ (Size.scala:70): integer bytes
    if (shard < min_bytes) shard = min_bytes;  // getInvokerSlot: below MIN_MEMORY -> MIN_MEMORY (SCPB:490-497)
    permits[i] = (int32_t)(shard / (1024 * 1024));  // .toMB (Size.scala:97-99)
}

__global__ __launch_bounds__(256) void owgs_usable_kernel(const uint8_t* status, int32_t n, uint32_t* bits,
                                                          int32_t n_words) {
    const int wd = blockIdx.x * 256 + threadIdx.x;
    if (wd >= n_words) return;
    uint32_t b = 0;
    for (int k = 0; k < 32; ++k) {
        const int i = wd * 32 + k;
        if (i < n && status[i] == 0) b |= 1u << k;  // OWGS_HEALTHY
    }
    bits[wd] = b;
}

// the usable bitmap of every row of a [rows][stride] status matrix (one row per batch: the health each batch of a group
// replay applies before its releases, owgs_replay_device_group) into bits[row * n_words ..]
__global__ __launch_bounds__(256) void owgs_usable_rows_kernel(const uint8_t* status, int64_t stride, int32_t n,
                                                               uint32_t* bits, int32_t n_words) {
    const int wd = blockIdx.x * 256 + threadIdx.x, row = blockIdx.y;
    if (wd >= n_words) return;
    const uint8_t* st = status + (int64_t)row * stride;
    uint32_t b = 0;
    for (int k = 0; k < 32; ++k) {
        const int i = wd * 32 + k;
        if (i < n && st[i] == 0) b |= 1u << k;  // OWGS_HEALTHY
    }
    bits[(int64_t)row * n_words + wd] = b;
}

extern "C" hipError_t owgs_launch_usable_rows(const uint8_t* status, int64_t stride, int32_t n, int32_t rows,
                                              uint32_t* bits, int32_t n_words, hipStream_t s) {
    if (rows <= 0 || n_words <= 0) return hipSuccess;
    hipLaunchKernelGGL(owgs_usable_rows_kernel, dim3((unsigned)((n_words + 255) / 256), (unsigned)rows), dim3(256), 0, s,
                       status, stride, n, bits, n_words);
    return hipGetLastError();
}

extern "C" int32_t owgs_coprime_max(void) { return CP_MAX; }

// xs[0..n_pools) on the device; out[p * out_stride ..] receives pool p's list, counts[p] its length.
extern "C" hipError_t owgs_launch_coprime(const int32_t* xs, int32_t n_pools, int32_t* out, int32_t out_stride,
                                          int32_t* counts, hipStream_t s) {
    if (n_pools <= 0) return hipSuccess;
    hipLaunchKernelGGL(owgs_coprime_kernel, dim3(n_pools), dim3(CP_TPB), 0, s, xs, out, out_stride, counts);
    return hipGetLastError();
}

extern "C" hipError_t owgs_launch_slots(const int64_t* mem_bytes, int32_t from, int32_t n, int32_t cluster,
                                       int64_t min_bytes, int32_t* permits, hipStream_t s) {
    if (n <= from) return hipSuccess;
    hipLaunchKernelGGL(owgs_slots_kernel, dim3((n - from + 255) / 256), dim3(256), 0, s, mem_bytes, from, n, cluster,
                       min_bytes, permits);
    return hipGetLastError();
}

extern "C" hipError_t owgs_launch_usable(const uint8_t* status, int32_t n, uint32_t* bits, int32_t n_words,
                                        hipStream_t s) {
    if (n_words <= 0) return hipSuccess;
    hipLaunchKernelGGL(owgs_usable_kernel, dim3((n_words + 255) / 256), dim3(256), 0, s, status, n, bits, n_words);
    return hipGetLastError();
}

// Key recycling (owgs_release_actions): cand = bitmap over fqn@version slot ids that no live action handle names; the
// bit of every slot still held by a NestedSemaphore entry (primary table, HBM overflow: key = (invoker + 1) | slot << 15)
// or by a watched pair (its table and its per-key count) is cleared.  What stays set is free (NestedSemaphore.scala:
// 109-111 drops an entry at operationCount 0; nothing else on the device is keyed by slot).
__global__ __launch_bounds__(256) void owgs_slot_scan_kernel(const uint32_t* ct_keys, const uint2* ovf, int32_t ovf_cap,
                                                             const uint32_t* w_keys, int32_t w_cap, const int32_t* wkey,
                                                             uint32_t* cand) {
    const int64_t n_keys = (int64_t)OWGS_MAX_SLOTKEYS + 1;
    const int64_t total = (int64_t)OWGS_CTC + ovf_cap + w_cap + (wkey ? n_keys : 0);
    auto drop = [&](uint32_t s) {
        if (s < (uint32_t)n_keys && ((cand[s >> 5] >> (s & 31)) & 1u)) atomicAnd(&cand[s >> 5], ~(1u << (s & 31)));
    };
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        uint32_t key = 0u;
        if (i < OWGS_CTC) {
            key = ct_keys[i];
        } else if (i < (int64_t)OWGS_CTC + ovf_cap) {
            key = ovf[i - OWGS_CTC].x;
        } else if (i < (int64_t)OWGS_CTC + ovf_cap + w_cap) {
            key = w_keys[i - OWGS_CTC - ovf_cap];
        } else {
            const int64_t s = i - OWGS_CTC - ovf_cap - w_cap;
            if (wkey[s] > 0) drop((uint32_t)s);
            continue;
        }
        if (key != 0u && key != OWGS_CT_TOMB) drop(key >> OWGS_CT_SLOT_SHIFT);
    }
}

extern "C" hipError_t owgs_launch_slot_scan(const uint32_t* ct_keys, const uint2* ovf, int32_t ovf_cap,
                                           const uint32_t* w_keys, int32_t w_cap, const int32_t* wkey, uint32_t* cand,
                                           hipStream_t s) {
    hipLaunchKernelGGL(owgs_slot_scan_kernel, dim3(512), dim3(256), 0, s, ct_keys, ovf, ovf_cap, w_keys, w_cap, wkey,
                       cand);
    return hipGetLastError();
}
