// Microbenchmark: dependent-load latency of one wave on MI355X for the large-state engine's access pattern
// (owgs_seq.hip): a pointer chase over a 1 MB array (beyond L1, inside one XCD's L2) with plain loads, with
// agent-scope relaxed atomic loads (`sc1`), and each hop followed by a store and a wait for it (vmcnt(0)).  Prints
// cycles per hop (s_memtime) for each, as JSON.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/load_lat tools/micro/load_lat.hip && /tmp/load_lat
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ __launch_bounds__(64) void chase(const int* next, int* sink, int hops, int mode, long long* out) {
    if (threadIdx.x != 0) return;
    int p = 0;
    const long long t0 = clock64();
    for (int h = 0; h < hops; ++h) {
        if (mode == 0) {
            p = next[p];
        } else {
            p = __hip_atomic_load(&next[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (mode == 2) {
            sink[p & 1023] = h;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    const long long t1 = clock64();
    out[0] = t1 - t0;
    out[1] = p;
}

int main() {
    const int n = 1 << 18;  // 1 MB of ints
    std::vector<int> perm(n), next(n);
    for (int i = 0; i < n; ++i) perm[i] = i;
    unsigned s = 12345u;
    for (int i = n - 1; i > 0; --i) {  // a random cycle through every element
        s = s * 1664525u + 1013904223u;
        const int j = (int)(s % (unsigned)(i + 1));
        const int t = perm[i];
        perm[i] = perm[j];
        perm[j] = t;
    }
    for (int i = 0; i < n; ++i) next[perm[i]] = perm[(i + 1) % n];
    int *d_next, *d_sink;
    long long* d_out;
    if (hipMalloc(&d_next, n * sizeof(int)) != hipSuccess || hipMalloc(&d_sink, 4096 * sizeof(int)) != hipSuccess ||
        hipMalloc(&d_out, 2 * sizeof(long long)) != hipSuccess)
        return 1;
    if (hipMemcpy(d_next, next.data(), n * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) return 1;
    const char* names[3] = {"plain", "agent_atomic_load", "agent_load_then_store_wait"};
    printf("{\"array_bytes\": %d, \"cycles_per_hop\": {", n * 4);
    for (int mode = 0; mode < 3; ++mode) {
        long long h[2] = {0, 0};
        for (int rep = 0; rep < 2; ++rep) {  // (first: warms L2 with the array)
            hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, d_next, d_sink, n, mode, d_out);
            if (hipDeviceSynchronize() != hipSuccess) return 2;
            if (hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
        }
        printf("%s\"%s\": %.1f", mode ? ", " : "", names[mode], (double)h[0] / n);
    }
    printf("}}\n");
    return 0;
}
