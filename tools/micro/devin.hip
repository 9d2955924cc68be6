// Microbenchmark: where a resident kernel should read a call's input block from.  The host writes an 8 KB block and
// rings a doorbell (pinned word); the resident kernel (one workgroup) reads the block, writes a checksum answer, and
// the host spins on it.  Block placement:
//   pinned      hipHostMalloc(coherent) host memory: the kernel's reads cross PCIe (today's resident engine)
//   devfine     hipExtMallocWithFlags(hipDeviceMallocFinegrained) device memory written by the host through its
//               mapping (if the allocation has a host pointer: large-BAR systems); the kernel reads HBM
// Prints p50 / p90 round trips (us) and the host's copy time; exits on its own.
//   hipcc -O3 --offload-arch=gfx950 -o tools/micro/devin tools/micro/devin.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)

__device__ __forceinline__ int ld_sys(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }
__device__ __forceinline__ void st_sys(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }

__global__ __launch_bounds__(256) void resident_k(int* ctl, const uint4* in, int n16, long long idle_ticks) {
    __shared__ int s_k;
    __shared__ unsigned s_sum;
    int last = 0;
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (threadIdx.x == 0) {
            int k;
            for (;;) {
                k = ld_sys(ctl);
                if (k != last) break;
                if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > idle_ticks) {
                    k = -1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            s_k = k;
            s_sum = 0;
        }
        __syncthreads();
        const int k = s_k;
        if (k < 0) break;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        unsigned x = 0;
        for (int i = threadIdx.x; i < n16; i += 256) {
            const uint4 v = in[i];
            x += v.x ^ v.y ^ v.z ^ v.w;
        }
        atomicAdd(&s_sum, x);
        __syncthreads();
        if (threadIdx.x == 0) {
            st_sys(ctl + 16, (int)s_sum);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            st_sys(ctl + 32, k);
        }
        last = k;
        t0 = __builtin_amdgcn_s_memrealtime();
    }
}

static int run(const char* name, int* ctl, uint4* dev_in, void* host_view, int n16, int calls) {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    volatile int* c = ctl;
    c[0] = 0;
    c[32] = 0;
    hipLaunchKernelGGL(resident_k, dim3(1), dim3(256), 0, s, ctl, dev_in, n16, 100LL * 200000);  // 200 ms idle
    CK(hipGetLastError());
    std::vector<uint4> src(n16);
    std::vector<double> rt, cp;
    for (int k = 1; k <= calls; ++k) {
        for (int i = 0; i < n16; ++i) src[i] = make_uint4(k, i, k ^ i, 7);
        const auto t0 = std::chrono::steady_clock::now();
        memcpy(host_view, src.data(), (size_t)n16 * 16);
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        const auto t1 = std::chrono::steady_clock::now();
        __atomic_store_n(&ctl[0], k, __ATOMIC_RELEASE);
        while (__atomic_load_n(&ctl[32], __ATOMIC_ACQUIRE) != k) __builtin_ia32_pause();
        const auto t2 = std::chrono::steady_clock::now();
        unsigned want = 0;
        for (int i = 0; i < n16; ++i) want += src[i].x ^ src[i].y ^ src[i].z ^ src[i].w;
        if ((unsigned)ctl[16] != want) {
            fprintf(stderr, "%s: checksum mismatch at call %d\n", name, k);
            __atomic_store_n(&ctl[0], -1, __ATOMIC_RELEASE);
            hipStreamSynchronize(s);
            return 1;
        }
        if (k > 50) {
            cp.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            rt.push_back(std::chrono::duration<double, std::micro>(t2 - t0).count());
        }
    }
    __atomic_store_n(&ctl[0], -1, __ATOMIC_RELEASE);
    CK(hipStreamSynchronize(s));
    std::sort(rt.begin(), rt.end());
    std::sort(cp.begin(), cp.end());
    printf("{\"case\": \"%s\", \"bytes\": %d, \"p50_us\": %.2f, \"p90_us\": %.2f, \"host_copy_p50_us\": %.2f}\n", name,
           n16 * 16, rt[rt.size() / 2], rt[rt.size() * 9 / 10], cp[cp.size() / 2]);
    CK(hipStreamDestroy(s));
    return 0;
}

int main() {
    const int n16 = 8192 / 16, calls = 2000;
    int* ctl;
    CK(hipHostMalloc((void**)&ctl, 4096, hipHostMallocCoherent));
    memset(ctl, 0, 4096);
    uint4* pin;
    CK(hipHostMalloc((void**)&pin, 65536, hipHostMallocCoherent));
    if (run("pinned", ctl, pin, pin, n16, calls)) return 1;
    uint4* dev = nullptr;
    if (hipExtMallocWithFlags((void**)&dev, 65536, hipDeviceMallocFinegrained) != hipSuccess) {
        printf("{\"case\": \"devfine\", \"error\": \"hipExtMallocWithFlags(fine-grained) failed\"}\n");
        return 0;
    }
    hipPointerAttribute_t at;
    void* hv = nullptr;
    if (hipPointerGetAttributes(&at, dev) == hipSuccess) hv = at.hostPointer;
    if (!hv) {
        printf("{\"case\": \"devfine\", \"error\": \"no host mapping of fine-grained device memory\"}\n");
        return 0;
    }
    return run("devfine", ctl, dev, hv, n16, calls);
}
