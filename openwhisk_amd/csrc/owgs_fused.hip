// owgs_fused.hip -- owgs_process_batch: one drained batch of the shim's batching thread in one launch chain.
//
// The shim drains its queue into runs of completions followed by publishes (GpuShardingContainerPoolBalancer.scala
// runBatch; CommonLoadBalancer.processCompletion -> releaseInvoker, SCPB:327-331, then publish, SCPB:257-290).
// owgs_stage_releases_kernel turns each run's completions -- (invoker, action handle) pairs from the caller's
// ActivationEntry -- into the engine's release records, so ONE engine launch replays the whole drained batch as a
// stream of batches (releases of run r, then its publishes), exactly like a replay whose releases name activations
// of earlier calls.  The records of a run are split by class (maxConcurrent == 1 and no-op records first, concurrent
// ones after, stream order inside a class); rel_src maps a record back to the caller's release for its flags.
#include <hip/hip_runtime.h>

#include "owgs_internal.h"

// one workgroup per run: class counts, then stable placement by ballot ranks
__global__ __launch_bounds__(256) void owgs_stage_releases_kernel(OwgsStageArgs a) {
    const int run = blockIdx.x;
    const bool span = a.rel_off == nullptr;
    const int64_t cb = span ? 0 : a.rel_off[run], ce = span ? a.span_nrel : a.rel_off[run + 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ int t0[4], t1[4];
    if (span && tid == 0) {
        a.span_off[0] = 0;
        a.span_off[1] = a.span_npub;
        a.span_off[2] = 0;
        a.span_off[3] = a.span_nrel;
    }
    auto inv_of = [&](int64_t i) { return span ? a.dec_inv[a.rel_aid[i]] : a.rel_inv[i]; };
    auto act_of = [&](int64_t i) { return span ? a.dec_act[a.rel_aid[i]] : a.rel_act[i]; };
    auto first_class = [&](int64_t i) {
        const int inv = inv_of(i);
        return inv < 0 || inv >= a.n_slots || a.act_maxc[act_of(i)] == 1;
    };
    int n0 = 0;
    for (int64_t c = cb; c < ce; c += 256) {
        const int64_t i = c + tid;
        n0 += __syncthreads_count(i < ce && first_class(i));
    }
    const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    int base0 = 0, base1 = 0;
    for (int64_t c = cb; c < ce; c += 256) {
        const int64_t i = c + tid;
        const bool valid = i < ce;
        const bool f = valid && first_class(i);
        const unsigned long long b0 = __ballot(f), b1 = __ballot(valid && !f);
        if (lane == 0) {
            t0[wave] = __popcll(b0);
            t1[wave] = __popcll(b1);
        }
        __syncthreads();
        int o0 = base0, o1 = base1, s0 = 0, s1 = 0;
        for (int w = 0; w < 4; ++w) {
            if (w < wave) {
                o0 += t0[w];
                o1 += t1[w];
            }
            s0 += t0[w];
            s1 += t1[w];
        }
        if (valid) {
            const int inv = inv_of(i), act = act_of(i);
            const bool in = inv >= 0 && inv < a.n_slots;
            const int64_t pos = f ? cb + o0 + __popcll(b0 & lt) : cb + n0 + o1 + __popcll(b1 & lt);
            const uint32_t inv15 = in ? (uint32_t)inv : OWGS_RR_NOINV;  // no-op: invokerSlots.lift (SCPB:329)
            a.rel_rec[pos] = make_uint2(inv15 | ((uint32_t)a.act_mem[act] << 15),
                                        (uint32_t)a.act_slot[act] | ((uint32_t)a.act_maxc[act] << 17));
            a.rel_src[pos] = (int32_t)i;
            a.rel_flags[i] = inv < 0 ? OWGS_REL_NOENTRY_BIT : 0;  // no ActivationEntry (CLB:278-279)
            // what the releases can return per slot at most (every release its memory: a concurrent one returns it
            // when its container empties): the engine refuses the call when a slot could leave its LDS range
            if (a.bound && in) atomicAdd(&a.bound[inv], (unsigned long long)a.act_mem[act]);
        }
        base0 += s0;
        base1 += s1;
        __syncthreads();
    }
    if (tid == 0) {
        a.relcnt[2 * run] = n0;
        a.relcnt[2 * run + 1] = (int32_t)(ce - cb) - n0;
    }
}

// Span mode with many releases (owgs_replay_device_span: a whole batch of a replay): the same stable split by class
// over tiles of OWGS_STAGE_TILE records, one workgroup each -- count the first class per tile, then every tile places
// its records after the first-class records of the tiles before it (and the second class after all first-class ones).
__device__ __forceinline__ bool stage_first_class(const OwgsStageArgs& a, int64_t i) {
    const int inv = a.dec_inv[a.rel_aid[i]];
    return inv < 0 || inv >= a.n_slots || a.act_maxc[a.dec_act[a.rel_aid[i]]] == 1;
}

__global__ __launch_bounds__(256) void owgs_stage_count_kernel(OwgsStageArgs a) {
    const int64_t t0 = (int64_t)blockIdx.x * OWGS_STAGE_TILE;
    int n = 0;
    for (int k = 0; k < OWGS_STAGE_TILE; k += 256) {
        const int64_t i = t0 + k + threadIdx.x;
        n += __syncthreads_count(i < a.span_nrel && stage_first_class(a, i));
    }
    if (threadIdx.x == 0) a.tile_cnt[blockIdx.x] = n;
}

__global__ __launch_bounds__(256) void owgs_stage_place_kernel(OwgsStageArgs a, int32_t n_tiles) {
    const int tile = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ int sb, st, t0[4], t1[4];
    if (tid == 0) sb = st = 0;
    __syncthreads();
    int before = 0, total = 0;
    for (int j = tid; j < n_tiles; j += 256) {
        const int v = a.tile_cnt[j];
        total += v;
        before += j < tile ? v : 0;
    }
    atomicAdd(&sb, before);
    atomicAdd(&st, total);
    __syncthreads();
    const int64_t nr = a.span_nrel, tb = (int64_t)tile * OWGS_STAGE_TILE;
    const int64_t n0 = st;
    int64_t base0 = sb, base1 = tb - sb;  // records of each class in the tiles before this one
    if (tile == 0 && tid == 0) {
        a.relcnt[0] = (int32_t)n0;
        a.relcnt[1] = (int32_t)(nr - n0);
        a.span_off[0] = 0;
        a.span_off[1] = a.span_npub;
        a.span_off[2] = 0;
        a.span_off[3] = nr;
    }
    const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (int k = 0; k < OWGS_STAGE_TILE; k += 256) {
        const int64_t i = tb + k + tid;
        const bool valid = i < nr;
        const bool f = valid && stage_first_class(a, i);
        const unsigned long long b0 = __ballot(f), b1 = __ballot(valid && !f);
        if (lane == 0) {
            t0[wave] = __popcll(b0);
            t1[wave] = __popcll(b1);
        }
        __syncthreads();
        int64_t o0 = base0, o1 = base1;
        int s0 = 0, s1 = 0;
        for (int w = 0; w < 4; ++w) {
            if (w < wave) {
                o0 += t0[w];
                o1 += t1[w];
            }
            s0 += t0[w];
            s1 += t1[w];
        }
        if (valid) {
            const int inv = a.dec_inv[a.rel_aid[i]], act = a.dec_act[a.rel_aid[i]];
            const bool in = inv >= 0 && inv < a.n_slots;
            const int64_t pos = f ? o0 + __popcll(b0 & lt) : n0 + o1 + __popcll(b1 & lt);
            const uint32_t inv15 = in ? (uint32_t)inv : OWGS_RR_NOINV;
            a.rel_rec[pos] = make_uint2(inv15 | ((uint32_t)a.act_mem[act] << 15),
                                        (uint32_t)a.act_slot[act] | ((uint32_t)a.act_maxc[act] << 17));
            a.rel_src[pos] = (int32_t)i;
            a.rel_flags[i] = inv < 0 ? OWGS_REL_NOENTRY_BIT : 0;
        }
        base0 += s0;
        base1 += s1;
        __syncthreads();
    }
}

// (invoker, action handle) -> the release kernels' (invoker, memory, maxConcurrent, slot key) arrays
__global__ __launch_bounds__(256) void owgs_relmeta_kernel(int32_t n, const int32_t* act, const int32_t* act_mem,
                                                           const int32_t* act_maxc, const int32_t* act_slot,
                                                           int32_t* mem, int32_t* maxc, int32_t* slot) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int a = act[i];
    mem[i] = act_mem[a];
    maxc[i] = act_maxc[a];
    slot[i] = act_slot[a];
}

extern "C" hipError_t owgs_launch_stage_releases(const OwgsStageArgs* a, hipStream_t s) {
    if (a->n_runs <= 0) return hipSuccess;
    if (a->rel_off == nullptr && a->span_nrel > OWGS_STAGE_TILE && a->tile_cnt) {
        const int32_t nt = (int32_t)((a->span_nrel + OWGS_STAGE_TILE - 1) / OWGS_STAGE_TILE);
        hipLaunchKernelGGL(owgs_stage_count_kernel, dim3((unsigned)nt), dim3(256), 0, s, *a);
        hipLaunchKernelGGL(owgs_stage_place_kernel, dim3((unsigned)nt), dim3(256), 0, s, *a, nt);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(owgs_stage_releases_kernel, dim3((unsigned)a->n_runs), dim3(256), 0, s, *a);
    return hipGetLastError();
}

extern "C" hipError_t owgs_launch_relmeta(int32_t n, const int32_t* act, const int32_t* act_mem,
                                          const int32_t* act_maxc, const int32_t* act_slot, int32_t* mem,
                                          int32_t* maxc, int32_t* slot, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(owgs_relmeta_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, act, act_mem,
                       act_maxc, act_slot, mem, maxc, slot);
    return hipGetLastError();
}
