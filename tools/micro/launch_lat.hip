// Microbenchmark: the fixed costs of one shim call (owgs_process_batch) on MI355X -- what a drained batch of 64 jobs
// pays before any scheduling work.  Each case is timed over many calls from the host (wall clock, p50):
//   launch1     one empty kernel + hipStreamSynchronize
//   launch4     four dependent empty kernels (the stage / chunks / pre-pass / engine chain) + sync
//   copies      H2D 1 KB (pinned) + kernel + D2H 1 KB (pinned) + sync (today's staging)
//   zerocopy    one kernel that reads its 1 KB input from pinned host memory and writes its output there + sync
//   doorbell    a resident kernel (one workgroup) polling a doorbell word in pinned host memory: the host writes the
//               call number, the kernel answers in another pinned word; host spins (no HIP call per round trip)
//   doorbell_io the same, the kernel also reads 1 KB of input from pinned memory and writes 1 KB back per round trip
// The resident kernel exits on a stop word or after a bounded number of idle polls.
//   hipcc -O3 --offload-arch=gfx950 -o tools/micro/launch_lat tools/micro/launch_lat.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)

__global__ void empty_k(int* p) {
    if (threadIdx.x == 0 && p) p[0] += 1;
}

__global__ void io_k(const int* in, int* out, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = in[i] + 1;
}

__device__ __forceinline__ int ld_sys(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }
__device__ __forceinline__ void st_sys(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }

// resident: ctl[0] = doorbell (call number from the host, -1 = stop), ctl[64] = answer, ctl[32] = 1 once started,
// ctl[96] = polls done (written at exit); exits after idle_ticks (s_memrealtime, 100 MHz) without a new call
__global__ __launch_bounds__(256) void resident_k(int* ctl, const int* in, int* out, int n, long long idle_ticks) {
    __shared__ int s_k;
    int last = 0, polls = 0;
    if (threadIdx.x == 0) st_sys(ctl + 32, 1);
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (threadIdx.x == 0) {
            int k;
            for (;;) {
                k = ld_sys(ctl);
                ++polls;
                if (k != last) break;
                if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > idle_ticks) {
                    k = -1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            s_k = k;
        }
        __syncthreads();
        const int k = s_k;
        __syncthreads();
        if (k < 0) break;
        last = k;
        if (n > 0) {
            for (int i = threadIdx.x; i < n; i += blockDim.x) {
                const int v = ld_sys(in + i);
                st_sys(out + i, v + k);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: outputs visible before the answer
            __syncthreads();
        }
        if (threadIdx.x == 0) st_sys(ctl + 64, k);
        t0 = __builtin_amdgcn_s_memrealtime();
    }
    if (threadIdx.x == 0) st_sys(ctl + 96, polls);
}

static double p50(std::vector<double>& v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}
static double p99(std::vector<double>& v) {
    std::sort(v.begin(), v.end());
    return v[(size_t)(v.size() * 0.99)];
}
using clk = std::chrono::steady_clock;
static double us_since(clk::time_point t0) { return std::chrono::duration<double, std::micro>(clk::now() - t0).count(); }

int main() {
    const int N = 2000, W = 200, NI = 256;  // calls, warmup, ints of I/O (1 KB)
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int *d, *din, *dout, *hin, *hout, *ctl;
    CK(hipMalloc(&d, 4096));
    CK(hipMalloc(&din, NI * 4));
    CK(hipMalloc(&dout, NI * 4));
    CK(hipHostMalloc(&hin, NI * 4, hipHostMallocDefault));
    CK(hipHostMalloc(&hout, NI * 4, hipHostMallocDefault));
    CK(hipHostMalloc(&ctl, 4096, hipHostMallocCoherent));
    for (int i = 0; i < NI; ++i) hin[i] = i;
    printf("{\"launch_latency_us\": {");
    auto report = [](const char* name, std::vector<double>& v, bool first) {
        const double a = p50(v), b = p99(v);
        printf("%s\"%s\": {\"p50\": %.2f, \"p99\": %.2f}", first ? "" : ", ", name, a, b);
        fflush(stdout);
    };
    std::vector<double> t;
    // launch1
    t.clear();
    for (int i = 0; i < N + W; ++i) {
        auto t0 = clk::now();
        hipLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, s, d);
        CK(hipStreamSynchronize(s));
        if (i >= W) t.push_back(us_since(t0));
    }
    report("launch1", t, true);
    t.clear();
    for (int i = 0; i < N + W; ++i) {
        auto t0 = clk::now();
        for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(empty_k, dim3(k == 3 ? 1 : 64), dim3(256), 0, s, d);
        CK(hipStreamSynchronize(s));
        if (i >= W) t.push_back(us_since(t0));
    }
    report("launch4", t, false);
    t.clear();
    for (int i = 0; i < N + W; ++i) {
        auto t0 = clk::now();
        CK(hipMemcpyAsync(din, hin, NI * 4, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(io_k, dim3(1), dim3(256), 0, s, din, dout, NI);
        CK(hipMemcpyAsync(hout, dout, NI * 4, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        if (i >= W) t.push_back(us_since(t0));
    }
    report("copies", t, false);
    t.clear();
    for (int i = 0; i < N + W; ++i) {
        auto t0 = clk::now();
        hipLaunchKernelGGL(io_k, dim3(1), dim3(256), 0, s, hin, hout, NI);
        CK(hipStreamSynchronize(s));
        if (i >= W) t.push_back(us_since(t0));
    }
    report("zerocopy", t, false);
    // resident kernel round trips; every wait is bounded by wall-clock time
    for (int mode = 0; mode < 3; ++mode) {  // 0: doorbell, 1: + 1 KB in/out, 2: doorbell after a hipStreamQuery flush
        const int io = mode == 1;
        const char* name = mode == 0 ? "doorbell" : mode == 1 ? "doorbell_io" : "doorbell_flushed";
        volatile int* vc = ctl;
        vc[0] = 0;
        vc[32] = 0;
        vc[64] = 0;
        vc[96] = 0;
        auto tl = clk::now();
        hipLaunchKernelGGL(resident_k, dim3(1), dim3(256), 0, s, ctl, hin, hout, io ? NI : 0, 20000000ll);  // 200 ms idle
        if (mode == 2) (void)hipStreamQuery(s);
        bool alive = false;
        while (us_since(tl) < 2e6) {
            if (__atomic_load_n(&ctl[32], __ATOMIC_ACQUIRE) == 1) {
                alive = true;
                break;
            }
        }
        const double t_alive = us_since(tl);
        t.clear();
        int served = 0;
        for (int i = 1; i <= N + W && alive; ++i) {
            auto t0 = clk::now();
            __atomic_store_n(&ctl[0], i, __ATOMIC_RELEASE);
            bool ok = false;
            while (us_since(t0) < 100000) {
                if (__atomic_load_n(&ctl[64], __ATOMIC_ACQUIRE) == i) {
                    ok = true;
                    break;
                }
            }
            if (!ok || (io && hout[NI - 1] != NI - 1 + i)) break;
            ++served;
            if (i > W) t.push_back(us_since(t0));
        }
        __atomic_store_n(&ctl[0], -1, __ATOMIC_RELEASE);
        CK(hipStreamSynchronize(s));
        printf(", \"%s\": {\"start_us\": %.1f, \"served\": %d, \"polls\": %d", name, t_alive, served, ctl[96]);
        if (t.size() > 10) {
            const double a = p50(t), b = p99(t);
            printf(", \"p50\": %.2f, \"p99\": %.2f", a, b);
        }
        printf("}");
        fflush(stdout);
    }
    printf("}}\n");
    return 0;
}
