// Microbenchmark: dependent LDS read latency (random 4-byte gathers) vs. resident waves in one workgroup.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void lat(int nwaves, int iters, unsigned long long* out, int mode) {
    extern __shared__ int lds[];
    const int N = 32768;  // 128 KB
    for (int i = threadIdx.x; i < N; i += blockDim.x) lds[i] = (int)((i * 2654435761u + 12345u) & (N - 1));
    __syncthreads();
    const int w = threadIdx.x >> 6;
    if (w >= nwaves) return;
    int p = (threadIdx.x * 977) & (N - 1);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    int acc = 0;
    for (int k = 0; k < iters; ++k) {
        if (mode == 0) {
            p = lds[p];  // dependent chain
        } else {
            // 8 independent reads per step, then combine
            int a0 = lds[p], a1 = lds[(p + 4099) & (N - 1)], a2 = lds[(p + 8191) & (N - 1)], a3 = lds[(p + 12289) & (N - 1)];
            int a4 = lds[(p + 16411) & (N - 1)], a5 = lds[(p + 20483) & (N - 1)], a6 = lds[(p + 24593) & (N - 1)], a7 = lds[(p + 28687) & (N - 1)];
            p = (a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) & (N - 1);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    acc += p;
    if ((threadIdx.x & 63) == 0) out[w] = (t1 - t0);
    if (acc == -1) out[63] = acc;
}
int main() {
    unsigned long long* d;
    hipMalloc(&d, 64 * 8);
    hipFuncSetAttribute((const void*)lat, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int mode = 0; mode < 2; ++mode)
        for (int nw : {1, 2, 4, 8, 9, 16}) {
            const int iters = 2000;
            hipLaunchKernelGGL(lat, dim3(1), dim3(64 * (nw < 9 ? 9 : nw)), 131072, 0, nw, iters, d, mode);
            hipDeviceSynchronize();
            std::vector<unsigned long long> h(64);
            hipMemcpy(h.data(), d, 64 * 8, hipMemcpyDeviceToHost);
            unsigned long long mx = 0;
            for (int i = 0; i < nw; ++i) mx = h[i] > mx ? h[i] : mx;
            printf("mode %s waves %2d: %.1f cycles per step\n", mode ? "8-indep" : "chain", nw, (double)mx / iters);
        }
    return 0;
}
