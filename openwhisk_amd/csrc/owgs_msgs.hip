// owgs_msgs.hip -- ActivationMessage serialisation and per-invoker topic fan-out on the device (SURVEY.md §8(f)
// row 4): the output side of publish.
//
// Replaces, for a batch of scheduled activations:
//   ActivationMessage.serialize = serdes.write(this).compactPrint    Message.scala:51-70, 170-175 (jsonFormat11)
//   sendActivationToInvoker: topic "invoker<N>", one send per activation in publish order    CLB:175-198
// The invariant members are printed once per (action, identity) by the caller as templates (part A = "action",
// "revision", "user" members; part B = the initArgs array) and the rootControllerIndex once per context; content and
// traceContext arrive printed.  The device formats the per-activation members (transid with spray-json string
// escaping, the epoch-ms number, the 128-bit activation id and cause as 32 lowercase hex digits, blocking) and lays
// every topic's messages out contiguously in publish order, so each topic is one producer batch.
//
// Kernels (HBM-bound byte work; no MFMA):
//   owgs_msg_size_kernel     one thread per activation: validity, message length (escaped transaction id), topic key
//   hipcub radix sort        (topic, activation) -> stable order by topic
//   owgs_msg_gather_kernel   lengths in output order (for the byte-offset scan) + per-topic counts
//   hipcub exclusive sums    byte offsets of the messages, message ranges of the topics
//   owgs_msg_write_kernel    one wave per message: pieces copied by the 64 lanes; the transaction id is escaped
//                            cooperatively (per-lane unit lengths, wave prefix sum, scattered writes)
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdint.h>

#include "owgs_internal.h"

#define F_BLOCKING 1
#define F_EXTRA 2
#define F_CONTENT 4
#define F_CAUSE 8
#define F_TRACE 16

// spray-json string escaping of one UTF-16 unit: printed length
__device__ __forceinline__ int unit_len(unsigned u) {
    if (u == '"' || u == '\\' || u == '\b' || u == '\f' || u == '\n' || u == '\r' || u == '\t') return 2;
    return (u >= 0x20 && u < 0x7F) ? 1 : 6;
}

// decode the UTF-8 sequence starting at s[i] (i < n): code point, byte count; cp = -1 if malformed
__device__ __forceinline__ int utf8_at(const uint8_t* s, int64_t i, int64_t n, int* nb) {
    const unsigned c = s[i];
    if (c < 0x80) { *nb = 1; return (int)c; }
    unsigned cp, need;
    if ((c & 0xE0) == 0xC0) { cp = c & 0x1F; need = 1; }
    else if ((c & 0xF0) == 0xE0) { cp = c & 0x0F; need = 2; }
    else if ((c & 0xF8) == 0xF0) { cp = c & 0x07; need = 3; }
    else { *nb = 1; return -1; }
    for (unsigned k = 1; k <= need; ++k) {
        if (i + k >= n || (s[i + k] & 0xC0) != 0x80) { *nb = 1; return -1; }
        cp = cp << 6 | (s[i + k] & 0x3F);
    }
    *nb = (int)need + 1;
    if ((need == 1 && cp < 0x80) || (need == 2 && cp < 0x800) || (need == 3 && cp < 0x10000) || cp > 0x10FFFF ||
        (cp >= 0xD800 && cp <= 0xDFFF))
        return -1;
    return (int)cp;
}

// printed length of a code point (one or two UTF-16 units)
__device__ __forceinline__ int cp_len(int cp) { return cp >= 0x10000 ? 12 : unit_len((unsigned)cp); }

__constant__ unsigned long long POW10[20] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull,
    10000000ull, 100000000ull, 1000000000ull, 10000000000ull, 100000000000ull, 1000000000000ull, 10000000000000ull,
    100000000000000ull, 1000000000000000ull, 10000000000000000ull, 100000000000000000ull, 1000000000000000000ull,
    10000000000000000000ull};

__device__ __forceinline__ uint64_t magnitude(int64_t v) { return v < 0 ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v; }

// decimal digits of |v| (+1 for the sign): t = floor(bit length * log10(2)) is the digit count or one less
__device__ __forceinline__ int digits(int64_t v) {
    const uint64_t u = magnitude(v);
    const int t = ((64 - __clzll(u | 1)) * 1233) >> 12;
    return max(t + (u >= POW10[t] ? 1 : 0), 1) + (v < 0);
}

// decimal digit of u at power r (0 = units): u split into three base-1e9 limbs by two constant divisions, then one
// 32-bit division
__device__ __forceinline__ int digit_at(uint64_t u, int r) {
    const uint64_t q = u / 1000000000ull;
    const uint32_t lo = (uint32_t)(u - q * 1000000000ull);
    const uint64_t q2 = q / 1000000000ull;
    const uint32_t mid = (uint32_t)(q - q2 * 1000000000ull), top = (uint32_t)q2;
    const uint32_t x = r < 9 ? lo : r < 18 ? mid : top;
    const uint32_t p = (uint32_t)POW10[r < 9 ? r : r < 18 ? r - 9 : r - 18];
    return (int)((x / p) % 10u);
}

#define LIT(s) (int64_t)(sizeof(s) - 1)
#define P_TRANSID "{\"transid\":["
#define P_AID ",\"activationId\":"
#define P_RCI ",\"rootControllerIndex\":"
#define P_BLOCK_T ",\"blocking\":true"
#define P_BLOCK_F ",\"blocking\":false"
#define P_CONTENT ",\"content\":"
#define P_INIT ",\"initArgs\":"
#define P_CAUSE ",\"cause\":"
#define P_TRACE ",\"traceContext\":"

__global__ __launch_bounds__(256) void owgs_msg_size_kernel(OwgsMsgArgs A) {
    const int32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= A.n) return;
    const int32_t inv = A.invoker[i];
    if (inv < 0) {
        A.key[i] = (uint32_t)A.n_topics;  // no message: sorts after every topic
        A.len[i] = 0;
        return;
    }
    const int32_t t = A.tmpl[i];
    if (inv >= A.n_topics || t < 0 || t >= A.n_templates) {
        atomicOr(A.bad, 1);
        A.key[i] = (uint32_t)A.n_topics;
        A.len[i] = 0;
        return;
    }
    const uint8_t f = A.flags[i];
    const uint8_t* s = (const uint8_t*)A.tid;
    const int64_t b = A.tid_off[i], e = A.tid_off[i + 1];
    int64_t tl = 0;
    for (int64_t p = b; p < e;) {
        int nb;
        const int cp = utf8_at(s, p, e, &nb);
        if (cp < 0) { atomicOr(A.bad, 2); break; }
        tl += cp_len(cp);
        p += nb;
    }
    int64_t L = LIT(P_TRANSID) + 2 + tl + 1 + digits(A.tid_start[i]) + ((f & F_EXTRA) ? 5 : 0) + 2;
    L += A.ta_off[t + 1] - A.ta_off[t];
    L += LIT(P_AID) + 34 + LIT(P_RCI) + A.rci_len + ((f & F_BLOCKING) ? LIT(P_BLOCK_T) : LIT(P_BLOCK_F));
    if (f & F_CONTENT) L += LIT(P_CONTENT) + A.content_off[i + 1] - A.content_off[i];
    L += LIT(P_INIT) + A.tb_off[t + 1] - A.tb_off[t];
    if (f & F_CAUSE) L += LIT(P_CAUSE) + 34;
    if (f & F_TRACE) L += LIT(P_TRACE) + A.trace_off[i + 1] - A.trace_off[i];
    L += 1;
    A.key[i] = (uint32_t)inv;
    A.len[i] = L;
}

__global__ __launch_bounds__(256) void owgs_msg_iota_kernel(int32_t* v, int32_t n) {
    const int32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) v[i] = i;
}

// lengths in output order (len_sorted[m] = 0 for the total) and topic counts
__global__ __launch_bounds__(256) void owgs_msg_gather_kernel(const int32_t* order, const int64_t* len,
                                                              const uint32_t* key_sorted, int32_t n, int32_t n_topics,
                                                              int64_t* len_sorted, int32_t* cnt) {
    const int32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    const uint32_t k = key_sorted[j];
    len_sorted[j] = k < (uint32_t)n_topics ? len[order[j]] : 0;
    if (k < (uint32_t)n_topics) atomicAdd(&cnt[k], 1);
}

// wave-cooperative copy of len bytes
__device__ __forceinline__ void wcopy(char* dst, const char* src, int64_t len, int lane) {
    const int n = (int)len;  // a piece of one message: < 2^31 bytes
    for (int j = lane; j < n; j += 64) dst[j] = src[j];
}
__device__ __forceinline__ void wlit(char* dst, const char* lit, int len, int lane) {
    if (lane < len) dst[lane] = lit[lane];
}

__device__ __forceinline__ void put_hex_unit(char* d, unsigned u) {
    const char* H = "0123456789abcdef";
    d[0] = '\\';
    d[1] = 'u';
    d[2] = H[(u >> 12) & 15];
    d[3] = H[(u >> 8) & 15];
    d[4] = H[(u >> 4) & 15];
    d[5] = H[u & 15];
}
__device__ __forceinline__ void put_unit(char* d, unsigned u) {
    switch (u) {
        case '"': d[0] = '\\'; d[1] = '"'; return;
        case '\\': d[0] = '\\'; d[1] = '\\'; return;
        case '\b': d[0] = '\\'; d[1] = 'b'; return;
        case '\f': d[0] = '\\'; d[1] = 'f'; return;
        case '\n': d[0] = '\\'; d[1] = 'n'; return;
        case '\r': d[0] = '\\'; d[1] = 'r'; return;
        case '\t': d[0] = '\\'; d[1] = 't'; return;
        default: break;
    }
    if (u >= 0x20 && u < 0x7F) d[0] = (char)u;
    else put_hex_unit(d, u);
}

// 32 lowercase hex digits of a 128-bit id, quoted; lanes 0..33 each write one char
__device__ __forceinline__ void wput_aid(char* d, ulonglong2 id, int lane) {
    if (lane == 0 || lane == 33) d[lane] = '"';
    else if (lane < 33) {
        const int k = lane - 1;
        const unsigned long long w = k < 16 ? id.x : id.y;
        const int sh = 60 - 4 * (k & 15);
        d[lane] = "0123456789abcdef"[(w >> sh) & 15];
    }
}

// grid over all n activations; the number of messages m = topic_start[n_topics] is read on the device, and nothing
// is written when the batch does not fit (out_off[n] = total bytes > cap: flag 4 for the host)
__global__ __launch_bounds__(256) void owgs_msg_write_kernel(OwgsMsgArgs A) {
    const int32_t j = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (j >= A.topic_start[A.n_topics] || *A.bad) return;
    if (A.out_off[A.n] > A.cap) {
        if (j == 0 && lane == 0) atomicOr(A.bad, 4);
        return;
    }
    const int32_t i = A.order[j];
    char* d = A.out + A.out_off[j];
    const int32_t t = A.tmpl[i];
    const uint8_t f = A.flags[i];
    int64_t o = 0;
    wlit(d + o, P_TRANSID, LIT(P_TRANSID), lane);
    o += LIT(P_TRANSID);
    if (lane == 0) d[o] = '"';
    o += 1;
    // transaction id: per-lane code points of a 64-byte window, printed lengths, wave prefix sum
    {
        const uint8_t* s = (const uint8_t*)A.tid;
        const int64_t b = A.tid_off[i], e = A.tid_off[i + 1];
        for (int64_t w = b; w < e; w += 64) {
            const int64_t p = w + lane;
            int cp = -2, nb = 0, pl = 0;
            // a lane prints the code point that starts at its byte (continuation bytes print nothing)
            if (p < e && (s[p] & 0xC0) != 0x80) {
                cp = utf8_at(s, p, e, &nb);
                pl = cp < 0 ? 0 : cp_len(cp);
            }
            int incl = pl;
            for (int off = 1; off < 64; off <<= 1) {
                const int v = __shfl_up(incl, off, 64);
                if (lane >= off) incl += v;
            }
            char* q = d + o + (incl - pl);
            if (pl) {
                if (cp >= 0x10000) {
                    put_hex_unit(q, 0xD800 + ((cp - 0x10000) >> 10));
                    put_hex_unit(q + 6, 0xDC00 + ((cp - 0x10000) & 0x3FF));
                } else {
                    put_unit(q, (unsigned)cp);
                }
            }
            o += __shfl(incl, 63, 64);
        }
    }
    if (lane == 0) { d[o] = '"'; d[o + 1] = ','; }
    o += 2;
    {
        const int64_t v = A.tid_start[i];
        const int nd = digits(v);
        if (lane < nd) {  // lane k writes character k from the left
            if (v < 0 && lane == 0) d[o] = '-';
            else d[o + lane] = (char)('0' + digit_at(magnitude(v), nd - 1 - lane));
        }
        o += nd;
    }
    if (f & F_EXTRA) { wlit(d + o, ",true", 5, lane); o += 5; }
    wlit(d + o, "],", 2, lane);
    o += 2;
    {
        const int64_t a0 = A.ta_off[t], al = A.ta_off[t + 1] - a0;
        wcopy(d + o, A.ta + a0, al, lane);
        o += al;
    }
    wlit(d + o, P_AID, LIT(P_AID), lane);
    o += LIT(P_AID);
    wput_aid(d + o, A.aid[i], lane);
    o += 34;
    wlit(d + o, P_RCI, LIT(P_RCI), lane);
    o += LIT(P_RCI);
    wcopy(d + o, A.rci, A.rci_len, lane);
    o += A.rci_len;
    if (f & F_BLOCKING) { wlit(d + o, P_BLOCK_T, LIT(P_BLOCK_T), lane); o += LIT(P_BLOCK_T); }
    else { wlit(d + o, P_BLOCK_F, LIT(P_BLOCK_F), lane); o += LIT(P_BLOCK_F); }
    if (f & F_CONTENT) {
        wlit(d + o, P_CONTENT, LIT(P_CONTENT), lane);
        o += LIT(P_CONTENT);
        const int64_t c0 = A.content_off[i], cl = A.content_off[i + 1] - c0;
        wcopy(d + o, A.content + c0, cl, lane);
        o += cl;
    }
    wlit(d + o, P_INIT, LIT(P_INIT), lane);
    o += LIT(P_INIT);
    {
        const int64_t b0 = A.tb_off[t], bl = A.tb_off[t + 1] - b0;
        wcopy(d + o, A.tb + b0, bl, lane);
        o += bl;
    }
    if (f & F_CAUSE) {
        wlit(d + o, P_CAUSE, LIT(P_CAUSE), lane);
        o += LIT(P_CAUSE);
        wput_aid(d + o, A.cause[i], lane);
        o += 34;
    }
    if (f & F_TRACE) {
        wlit(d + o, P_TRACE, LIT(P_TRACE), lane);
        o += LIT(P_TRACE);
        const int64_t r0 = A.trace_off[i], rl = A.trace_off[i + 1] - r0;
        wcopy(d + o, A.trace + r0, rl, lane);
        o += rl;
    }
    if (lane == 0) d[o] = '}';
}

#define GRID(n) dim3((unsigned)(((n) + 255) / 256)), dim3(256), 0, st

extern "C" size_t owgs_msg_scratch_bytes(int32_t n, int32_t n_topics, int32_t bits) {
    size_t a = 0, b = 0, c = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, n, 0, bits);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const int64_t*)nullptr, (int64_t*)nullptr, n + 1);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, c, (const int32_t*)nullptr, (int32_t*)nullptr, n_topics + 1);
    return a > b ? (a > c ? a : c) : (b > c ? b : c);
}

// phase 1: sizes, sort, offsets.  Leaves out_off[0..n], topic_start[0..n_topics] and order on the device; the caller
// reads the total (out_off[m], m = topic_start[n_topics]) before phase 2.
extern "C" hipError_t owgs_launch_msg_plan(const OwgsMsgArgs* a, int32_t bits, void* temp, size_t temp_bytes,
                                           uint32_t* key_sorted, int32_t* iota, int64_t* len_sorted, int32_t* cnt,
                                           hipStream_t st) {
    const OwgsMsgArgs& A = *a;
    hipError_t e;
    hipLaunchKernelGGL(owgs_msg_size_kernel, GRID(A.n), A);
    hipLaunchKernelGGL(owgs_msg_iota_kernel, GRID(A.n), iota, A.n);
    size_t tb = temp_bytes;
    e = hipcub::DeviceRadixSort::SortPairs(temp, tb, A.key, key_sorted, iota, A.order, A.n, 0, bits, st);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(cnt, 0, (size_t)(A.n_topics + 1) * 4, st);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(len_sorted + A.n, 0, 8, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(owgs_msg_gather_kernel, GRID(A.n), A.order, A.len, key_sorted, A.n, A.n_topics, len_sorted,
                       cnt);
    tb = temp_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(temp, tb, len_sorted, A.out_off, A.n + 1, st);
    if (e != hipSuccess) return e;
    tb = temp_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(temp, tb, cnt, A.topic_start, A.n_topics + 1, st);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

extern "C" hipError_t owgs_launch_msg_write(const OwgsMsgArgs* a, hipStream_t st) {
    if (a->n <= 0) return hipSuccess;
    hipLaunchKernelGGL(owgs_msg_write_kernel, dim3((unsigned)((a->n + 3) / 4)), dim3(256), 0, st, *a);
    return hipGetLastError();
}
