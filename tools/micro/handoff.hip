// Microbenchmark: cross-CU hand-off latency on MI355X, the price a multi-CU split of one shard's decision stream would
// pay per dependency edge.  Two workgroups of one launch ping-pong a counter: block 0 publishes
// k (optionally with a 1 KB payload tagged k), block `partner` waits for it, checks the payload and answers k; block 0
// waits for the answer.  partner = 8: same XCD under round-robin placement (checked with HW_REG_XCC_ID); partner = 1:
// another XCD.  Every store is a vector `sc1` store (agent-scope relaxed atomic), every poll an `sc1` load; polls are
// bounded (no hang if a block is never scheduled).
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/handoff tools/micro/handoff.hip && /tmp/handoff
#include <hip/hip_runtime.h>

#include <cstdio>

#define SPIN_MAX (1 << 24)
#define LINE 64  // ints: flags on separate 256-byte lines

__device__ __forceinline__ int ld(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ int xcc_id() {
    int v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 0xF;
}

// wait until *p == want (lane 0 polls, the wave learns the result); false after SPIN_MAX polls
__device__ __forceinline__ bool wait_eq(const int* p, int want) {
    int ok = 0;
    if (threadIdx.x == 0) {
        for (int s = 0; s < SPIN_MAX; ++s) {
            if (ld(p) == want) {
                ok = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    return __shfl(ok, 0, 64) != 0;
}

__global__ __launch_bounds__(64) void pingpong(int* buf, int partner, int iters, int payload, int* out) {
    const int b = blockIdx.x, lane = threadIdx.x;
    if (b != 0 && b != partner) return;
    int* ping = buf;
    int* pong = buf + LINE;
    int* data = buf + 2 * LINE;  // 64 lanes x 4 ints = 1 KB
    if (lane == 0) out[b == 0 ? 0 : 1] = xcc_id();
    int stale = 0, timeouts = 0;
    for (int k = 1; k <= iters; ++k) {
        if (b == 0) {
            if (payload) {
#pragma unroll
                for (int q = 0; q < 4; ++q) st(&data[4 * lane + q], k * 4 + q);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            if (lane == 0) st(ping, k);
            if (!wait_eq(pong, k)) {
                ++timeouts;
                break;
            }
        } else {
            if (!wait_eq(ping, k)) {
                ++timeouts;
                break;
            }
            if (payload) {
#pragma unroll
                for (int q = 0; q < 4; ++q) stale += ld(&data[4 * lane + q]) != k * 4 + q;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) st(pong, k);
        }
    }
    for (int d = 32; d >= 1; d >>= 1) stale += __shfl_xor(stale, d, 64);
    if (lane == 0) {
        atomicAdd(&out[2], stale);
        atomicAdd(&out[3], timeouts);
    }
}

int main() {
    int *buf, *out;
    hipMalloc(&buf, 8192);
    hipMalloc(&out, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("{\"handoff\": [\n");
    bool first = true;
    for (int payload = 0; payload < 2; ++payload)
        for (int partner : {8, 1}) {
            float ms[2];
            int h[4];
            const int its[2] = {10, 10010};
            for (int r = 0; r < 2; ++r) {
                hipMemset(buf, 0, 8192);
                hipMemset(out, 0, 64);
                hipDeviceSynchronize();
                hipEventRecord(e0);
                hipLaunchKernelGGL(pingpong, dim3(16), dim3(64), 0, 0, buf, partner, its[r], payload, out);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                hipEventElapsedTime(&ms[r], e0, e1);
                hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
            }
            const double rt_us = (ms[1] - ms[0]) * 1000.0 / (its[1] - its[0]);
            printf("%s  {\"partner_block\": %d, \"xcc\": [%d, %d], \"payload_bytes\": %d, \"round_trip_us\": %.3f, "
                   "\"one_way_us\": %.3f, \"stale_words\": %d, \"timeouts\": %d}",
                   first ? "" : ",\n", partner, h[0], h[1], payload ? 1024 : 0, rt_us, rt_us / 2, h[2], h[3]);
            first = false;
        }
    printf("\n]}\n");
    return 0;
}
