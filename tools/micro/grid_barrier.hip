// Microbenchmark: one grid-wide barrier over every CU of the MI355X, the per-round floor of a batch-scope fixpoint
// engine (profiles/r05_batch_fixpoint_sim.txt): G workgroups of one launch (G = the CU count, one
// wave each, all resident), R barriers in a row.  Arrival: one agent-scope atomic add per workgroup on a counter; the
// last arrival of round r publishes r in a flag word; the others poll it (`sc1` loads, s_sleep 1 between polls).  Polls
// are bounded and any workgroup that gives up raises an abort word every other workgroup also polls, so the launch
// always drains.  Prints microseconds per barrier for G = 8 (one per XCD), 64 and all CUs.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/grid_barrier tools/micro/grid_barrier.hip && /tmp/grid_barrier
#include <hip/hip_runtime.h>

#include <cstdio>

#define SPIN_MAX (1 << 22)
#define LINE 64  // ints: words on separate 256-byte lines

__device__ __forceinline__ int ld(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

__global__ __launch_bounds__(64) void barriers(int* buf, int rounds, int* out) {
    int* cnt = buf;
    int* flag = buf + LINE;
    int* abort_w = buf + 2 * LINE;
    const int G = (int)gridDim.x;
    int ok = 1;
    for (int r = 1; r <= rounds && ok; ++r) {
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old == r * G - 1) {
                st(flag, r);  // last arrival of round r
            } else {
                int s = 0;
                for (; s < SPIN_MAX; ++s) {
                    if (ld(flag) >= r) break;
                    if (ld(abort_w)) {
                        s = SPIN_MAX;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (s == SPIN_MAX) {
                    ok = 0;
                    st(abort_w, 1);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        ok = __shfl(ok, 0, 64);
    }
    if (threadIdx.x == 0 && !ok) atomicAdd(out, 1);
}

int main() {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
    const int cus = p.multiProcessorCount;
    int *buf, *out;
    if (hipMalloc(&buf, 4 * LINE * sizeof(int)) != hipSuccess || hipMalloc(&out, sizeof(int)) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int gs[3] = {8, 64, cus};
    printf("{\"cus\": %d, \"barriers\": [", cus);
    for (int gi = 0; gi < 3; ++gi) {
        const int G = gs[gi];
        for (int rep = 0; rep < 2; ++rep) {  // (first: warm-up)
            const int rounds = 20000;
            (void)hipMemset(buf, 0, 4 * LINE * sizeof(int));
            (void)hipMemset(out, 0, sizeof(int));
            (void)hipEventRecord(e0, 0);
            hipLaunchKernelGGL(barriers, dim3(G), dim3(64), 0, 0, buf, rounds, out);
            (void)hipEventRecord(e1, 0);
            if (hipEventSynchronize(e1) != hipSuccess) return 2;
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            int bad = 0;
            (void)hipMemcpy(&bad, out, sizeof(int), hipMemcpyDeviceToHost);
            if (rep == 1)
                printf("%s{\"workgroups\": %d, \"rounds\": %d, \"us_per_barrier\": %.3f, \"timeouts\": %d}", gi ? ", " : "",
                       G, rounds, ms * 1e3f / rounds, bad);
        }
    }
    printf("]}\n");
    return 0;
}
