// owgs_health.hip -- invoker health supervision on the device.
//
// Replaces, for a batch of supervision events in mailbox order (pings from the `health` topic, InvocationFinished
// results from processCompletion, CLB:316-343):
//   InvokerPool.receive / registerInvoker / padToIndexed     InvokerSupervision.scala (ISUP) 119-150, 180-199
//   InvokerActor FSM: Offline/Unhealthy/Unresponsive/Healthy, state timeout 10 s, 1-minute Tick while pinging,
//   handleCompletionMessage with a ring buffer of 10 results and tolerance 3      ISUP:285-440
// The status vector it produces is CurrentInvokerPoolState (ISUP:156-160), which the balancer's monitor turns into
// updateInvokers (SCPB:226-227) -- owgs_health_events(apply = 1) does exactly that on the same context.
//
// Layout (HBM, SoA by invoker id): st u8 (InvokerState, 254 = padded entry without an actor, 255 = outside the
// status vector), ring u32 (2 bits per result, oldest first, | count << 20), last i64 (when the state timeout was
// armed), tick i64 (next Tick), mem i64 (userMemory of the instance in the status vector), tests i32.
//
// Kernels (every one is a plain grid over events or invoker ids, no inter-workgroup hand-off):
//   hipcub radix sort of (invoker, event index)    stable grouping of the batch by invoker (mailbox order kept)
//   owgs_health_segments_kernel                    [begin, end) of each invoker's events in the sorted order
//   owgs_health_regfirst_kernel                    first ping of each invoker without an actor (registration)
//   owgs_health_padmin_kernel                      suffix minimum of registration indices: which registration
//                                                  padded each new status entry (its userMemory)
//   owgs_health_fsm_kernel                         one lane per invoker: its events in order, due timers between
//                                                  them and up to `now` (akka FSM rules restated in the header of
//                                                  oracle/owhealth_oracle.c, which the parity tests compare with)
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdint.h>

#define H_HEALTHY 0
#define H_UNHEALTHY 1
#define H_UNRESPONSIVE 2
#define H_OFFLINE 3
#define H_PADDED 254
#define H_ABSENT 255
#define EV_PING 0
#define EV_SUCCESS 1
#define EV_SYSTEM_ERROR 2
#define EV_TIMEOUT 3
#define EV_STATE_TIMEOUT 4
#define STATE_TIMEOUT_MS 10000  // healthyTimeout, ISUP:298
#define TICK_MS 60000           // setTimer(InvokerActor.timerName, Tick, 1.minute, repeat = true), ISUP:360
#define RING 10                 // InvokerActor.bufferSize, ISUP:437
#define TOLERANCE 3             // InvokerActor.bufferErrorTolerance, ISUP:438
#define NEVER INT64_MAX
#define NO_EVENT 0x7FFFFFFF

struct HealthArgs {
    // persistent state
    uint8_t* st;
    uint32_t* ring;
    int64_t* last;
    int64_t* tick;
    int64_t* mem;
    int32_t* tests;
    // batch
    const int32_t* ev_inv;    // sorted keys
    const int32_t* ev_idx;    // event index of each sorted position
    const int64_t* ev_packed; // t << 3 | kind of each sorted position (gathered once, read sequentially)
    const uint8_t* ev_kind;   // by event index
    const int64_t* ev_t;
    const int64_t* ev_mem;
    const int32_t* seg_beg;   // per invoker, valid where seg_end > seg_beg
    const int32_t* seg_end;
    const int32_t* reg_first;
    const int32_t* pad_src;
    int32_t old_size, new_size;
    int64_t now;
};

struct Inv {
    int st;
    uint32_t ring;
    int64_t last, tick;
    int tests;
};

__device__ __forceinline__ bool has_timeout(int st) { return st <= H_UNRESPONSIVE; }
__device__ __forceinline__ void arm(Inv& a, int64_t t) { a.last = has_timeout(a.st) ? t : NEVER; }

// goto(to): onTransition handlers in registration order (ISUP:339-365): Unhealthy's, then Unresponsive's
__device__ __forceinline__ void go(Inv& a, int to, int64_t t) {
    if (to != a.st) {
        const int from = a.st;
        if (to == H_UNHEALTHY) { a.tests++; a.tick = t + TICK_MS; }
        else if (from == H_UNHEALTHY) a.tick = NEVER;
        if (to == H_UNRESPONSIVE) { a.tests++; a.tick = t + TICK_MS; }
        else if (from == H_UNRESPONSIVE) a.tick = NEVER;
        a.st = to;
    }
    arm(a, t);
}

__device__ __forceinline__ void fire_due(Inv& a, int64_t t) {
    for (;;) {
        const int64_t ds = a.last == NEVER ? NEVER : a.last + STATE_TIMEOUT_MS;
        if (ds <= t && ds <= a.tick) {
            go(a, H_OFFLINE, ds);  // StateTimeout -> goto(Offline)
        } else if (a.tick <= t) {  // Tick -> invokeTestAction(); stay
            const int64_t dt = a.tick;
            a.tests++;
            a.tick = dt + TICK_MS;
            arm(a, dt);
        } else {
            return;
        }
    }
}

// handleCompletionMessage (ISUP:383-410) on the packed ring: add, then count system errors / timeouts
__device__ __forceinline__ void completion(Inv& a, int result, int64_t t) {
    uint32_t cnt = a.ring >> 20, bits = a.ring & 0xFFFFFu;
    if (cnt == RING) { bits >>= 2; cnt--; }
    bits |= (uint32_t)result << (2 * cnt);
    cnt++;
    a.ring = bits | cnt << 20;
    if (result == EV_SUCCESS && a.st == H_UNHEALTHY) a.tests++;
    if ((a.st == H_HEALTHY && result == EV_SUCCESS) || a.st == H_OFFLINE) {
        arm(a, t);
        return;
    }
    // count 2-bit fields equal to SYSTEM_ERROR (10b) and TIMEOUT (11b): hi & ~lo, hi & lo over the valid fields
    const uint32_t hi = (bits >> 1) & 0x55555u, lo = bits & 0x55555u;
    const int se = __popc(hi & ~lo), to = __popc(hi & lo);
    go(a, se > TOLERANCE ? H_UNHEALTHY : to > TOLERANCE ? H_UNRESPONSIVE : H_HEALTHY, t);
}

__global__ __launch_bounds__(256) void owgs_health_init_kernel(uint8_t* st, uint32_t* ring, int64_t* last,
                                                               int64_t* tick, int64_t* mem, int32_t* tests,
                                                               int32_t from, int32_t to) {
    const int32_t k = from + blockIdx.x * 256 + threadIdx.x;
    if (k >= to) return;
    st[k] = H_ABSENT;
    ring[k] = 0;
    last[k] = NEVER;
    tick[k] = NEVER;
    mem[k] = 0;
    tests[k] = 0;
}

__global__ __launch_bounds__(256) void owgs_health_iota_kernel(int32_t* v, int32_t n) {
    const int32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) v[i] = i;
}

// segment bounds + the sorted event record t << 3 | kind (times are >= 0 and below 2^60 ms)
__global__ __launch_bounds__(256) void owgs_health_segments_kernel(const int32_t* key, const int32_t* idx,
                                                                   const uint8_t* kind, const int64_t* t, int32_t n,
                                                                   int32_t size, int32_t* beg, int32_t* end,
                                                                   int64_t* packed) {
    const int32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int32_t e = idx[i];
    packed[i] = t[e] << 3 | kind[e];
    const int32_t k = key[i];
    if (k >= size) return;
    if (i == 0 || key[i - 1] != k) beg[k] = i;
    if (i == n - 1 || key[i + 1] != k) end[k] = i + 1;
}

// first ping of each invoker that has no actor yet (registerInvoker), else NO_EVENT
__global__ __launch_bounds__(256) void owgs_health_regfirst_kernel(HealthArgs A) {
    const int32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= A.new_size) return;
    int32_t r = NO_EVENT;
    if (A.st[k] >= H_PADDED) {
        for (int32_t p = A.seg_beg[k]; p < A.seg_end[k]; ++p) {
            if ((A.ev_packed[p] & 7) == EV_PING) { r = A.ev_idx[p]; break; }
        }
    }
    ((int32_t*)A.reg_first)[k] = r;
}

// pad_src[k] = min over j > k of reg_first[j]: the registration that first grew the vector past k.  One workgroup,
// tiles of 1024 ids from the top down, a reverse inclusive min-scan per tile in LDS carried across tiles.
__global__ __launch_bounds__(1024) void owgs_health_padmin_kernel(const int32_t* reg_first, int32_t* pad_src,
                                                                  int32_t n) {
    __shared__ int32_t s[1024];
    __shared__ int32_t carry;
    const int tid = threadIdx.x;
    if (tid == 0) carry = NO_EVENT;
    __syncthreads();
    for (int32_t top = n; top > 0; top -= 1024) {
        const int32_t k = top - 1 - tid;  // tid 0 = highest id of the tile
        s[tid] = k >= 0 ? reg_first[k] : NO_EVENT;
        __syncthreads();
        for (int off = 1; off < 1024; off <<= 1) {  // inclusive min over tids <= tid, i.e. ids >= k
            const int32_t v = tid >= off ? s[tid - off] : NO_EVENT;
            __syncthreads();
            s[tid] = min(s[tid], v);
            __syncthreads();
        }
        const int32_t c = carry;
        // exclusive: ids > k = inclusive of tid - 1, plus the carry from higher tiles
        const int32_t excl = min(c, tid ? s[tid - 1] : NO_EVENT);
        if (k >= 0) pad_src[k] = excl;
        __syncthreads();
        if (tid == 0) carry = min(c, s[1023]);
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void owgs_health_fsm_kernel(HealthArgs A) {
    const int32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= A.new_size) return;
    Inv a;
    a.st = A.st[k];
    a.ring = A.ring[k];
    a.last = A.last[k];
    a.tick = A.tick[k];
    a.tests = 0;
    int64_t mem = A.mem[k];
    if (a.st == H_ABSENT) {  // inside the new status vector: padded by the registration that grew it past k
        const int32_t src = A.pad_src[k];
        if (src != NO_EVENT) {
            a.st = H_PADDED;
            mem = A.ev_mem[src];
        }
    }
    const int32_t e0 = A.seg_beg[k], e1 = A.seg_end[k];
    // the invoker's events in blocks of 8: the block's loads issue together, then the FSM steps through them (the
    // userMemory of the status entry is the last ping's, read once at the end)
    int32_t last_ping = -1;
    for (int32_t p0 = e0; p0 < e1; p0 += 8) {
        int64_t wv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) wv[u] = p0 + u < e1 ? A.ev_packed[p0 + u] : -1;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t w = wv[u];
            if (w < 0) break;
            const int kind = (int)(w & 7);
            const int64_t t = w >> 3;
            if (a.st < H_PADDED) fire_due(a, t);
            if (kind == EV_PING) {
                if (a.st >= H_PADDED) {  // registerInvoker: new actor, startWith(Unhealthy) + initialize() handlers
                    a.ring = 0;
                    a.st = H_UNHEALTHY;
                    a.tests++;
                    a.tick = t + TICK_MS;
                }
                last_ping = p0 + u;
                if (a.st == H_OFFLINE) go(a, H_UNHEALTHY, t);
                else arm(a, t);
            } else if (a.st < H_PADDED) {
                if (kind == EV_STATE_TIMEOUT) {
                    if (has_timeout(a.st)) go(a, H_OFFLINE, t);
                    else arm(a, t);
                } else {
                    completion(a, kind, t);
                }
            }
        }
    }
    if (last_ping >= 0) mem = A.ev_mem[A.ev_idx[last_ping]];
    if (a.st < H_PADDED) fire_due(a, A.now);
    A.st[k] = (uint8_t)a.st;
    A.ring[k] = a.ring;
    A.last[k] = a.last;
    A.tick[k] = a.tick;
    A.mem[k] = mem;
    A.tests[k] = a.tests;
}

#define GRID(n) dim3((unsigned)(((n) + 255) / 256)), dim3(256), 0, st

extern "C" hipError_t owgs_launch_health_init(uint8_t* s, uint32_t* ring, int64_t* last, int64_t* tick, int64_t* mem,
                                              int32_t* tests, int32_t from, int32_t to, hipStream_t st) {
    if (to <= from) return hipSuccess;
    hipLaunchKernelGGL(owgs_health_init_kernel, GRID(to - from), s, ring, last, tick, mem, tests, from, to);
    return hipGetLastError();
}

// temp bytes for the sort of n (key, value) pairs
extern "C" size_t owgs_health_sort_bytes(int32_t n, int32_t bits) {
    size_t b = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                       (const int32_t*)nullptr, (int32_t*)nullptr, n, 0, bits);
    return b;
}

// keys: ev_inv (input), sorted into key_out; values: event indices sorted into idx_out (idx_in = scratch)
extern "C" hipError_t owgs_launch_health_batch(const int32_t* ev_inv, const uint8_t* ev_kind, const int64_t* ev_t,
                                               const int64_t* ev_mem, int32_t n, int32_t bits, void* temp,
                                               size_t temp_bytes, int32_t* key_out, int32_t* idx_in,
                                               int32_t* idx_out, int64_t* packed, int32_t* seg_beg, int32_t* seg_end,
                                               int32_t* reg_first, int32_t* pad_src, uint8_t* s, uint32_t* ring,
                                               int64_t* last, int64_t* tick, int64_t* mem, int32_t* tests,
                                               int32_t old_size, int32_t new_size, int64_t now, hipStream_t st) {
    hipError_t e;
    if (new_size <= 0) return hipSuccess;
    e = hipMemsetAsync(seg_beg, 0, (size_t)new_size * 4, st);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(seg_end, 0, (size_t)new_size * 4, st);
    if (e != hipSuccess) return e;
    if (n > 0) {
        hipLaunchKernelGGL(owgs_health_iota_kernel, GRID(n), idx_in, n);
        size_t tb = temp_bytes;
        e = hipcub::DeviceRadixSort::SortPairs(temp, tb, (const uint32_t*)ev_inv, (uint32_t*)key_out, idx_in, idx_out,
                                               n, 0, bits, st);  // ids are >= 0: unsigned keys, LSD = stable
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(owgs_health_segments_kernel, GRID(n), key_out, idx_out, ev_kind, ev_t, n, new_size, seg_beg,
                           seg_end, packed);
    }
    HealthArgs A;
    A.st = s;
    A.ring = ring;
    A.last = last;
    A.tick = tick;
    A.mem = mem;
    A.tests = tests;
    A.ev_inv = key_out;
    A.ev_idx = idx_out;
    A.ev_packed = packed;
    A.ev_kind = ev_kind;
    A.ev_t = ev_t;
    A.ev_mem = ev_mem;
    A.seg_beg = seg_beg;
    A.seg_end = seg_end;
    A.reg_first = reg_first;
    A.pad_src = pad_src;
    A.old_size = old_size;
    A.new_size = new_size;
    A.now = now;
    hipLaunchKernelGGL(owgs_health_regfirst_kernel, GRID(new_size), A);
    hipLaunchKernelGGL(owgs_health_padmin_kernel, dim3(1), dim3(1024), 0, st, reg_first, pad_src, new_size);
    hipLaunchKernelGGL(owgs_health_fsm_kernel, GRID(new_size), A);
    return hipGetLastError();
}
