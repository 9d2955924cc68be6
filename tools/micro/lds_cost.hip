// Microbenchmark: LDS cost per wave instruction for the access patterns of the engine (9 waves, one workgroup).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define N 32768
template <int MODE>
__global__ void k(int nwaves, int iters, unsigned long long* out) {
    extern __shared__ int lds[];
    for (int i = threadIdx.x; i < N; i += blockDim.x) lds[i] = (int)((i * 2654435761u + 12345u) & (N - 1));
    __syncthreads();
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (w >= nwaves) return;
    int p = (int)(((unsigned)threadIdx.x * 2654435761u) >> 17) & (N - 1);
    int acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        int a[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            int q;
            if (MODE == 0) q = (w * 64 + lane + j * 576) & (N - 1);                       // linear
            else if (MODE == 1) q = (p + j * 4099) & (N - 1);                              // random b32
            else if (MODE == 2) q = (p + j * 4099) & (N - 2);                              // random b64
            else if (MODE == 3) q = (w * 7 + j * 4099 + (p & 0)) & (N - 1);                // broadcast
            else if (MODE == 4) q = (p + j * 4099) & (N - 1);                              // random atomic
            else q = ((p & 63) * 16 + j * 4099 + (lane >> 4)) & (N - 1);                   // 16 lanes share a word group
            if (MODE == 2) {
                const int2 v = *(const int2*)&lds[q];
                a[j] = v.x ^ v.y;
            } else if (MODE == 4) {
                atomicAdd(&lds[q], 1);
                a[j] = 0;
            } else {
                a[j] = lds[q];
            }
        }
        int x = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) x ^= a[j];
        p = (p + x + 1) & (N - 1);
        acc += x;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[w] = t1 - t0;
    if (acc == 0x7fffffff) out[63] = acc;
}
template <int MODE>
void run(const char* name, unsigned long long* d) {
    hipFuncSetAttribute((const void*)k<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int nw : {1, 9}) {
        const int iters = 1000;
        hipLaunchKernelGGL(k<MODE>, dim3(1), dim3(64 * 9), 131072, 0, nw, iters, d);
        hipDeviceSynchronize();
        std::vector<unsigned long long> h(64);
        hipMemcpy(h.data(), d, 64 * 8, hipMemcpyDeviceToHost);
        unsigned long long mx = 0;
        for (int i = 0; i < nw; ++i) mx = h[i] > mx ? h[i] : mx;
        printf("%-22s waves %d: %6.1f cycles per 8 ops per wave -> %5.2f cycles per wave-op at the LDS\n", name, nw,
               (double)mx / iters, (double)mx / iters / (8.0 * nw));
    }
}
int main() {
    unsigned long long* d;
    (void)hipMalloc(&d, 64 * 8);
    run<0>("linear b32", d);
    run<1>("random b32", d);
    run<2>("random b64", d);
    run<3>("broadcast b32", d);
    run<4>("random atomic add", d);
    run<5>("16-lane groups b32", d);
    return 0;
}
