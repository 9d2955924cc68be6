// owgs_acks.hip -- completion-ack path on the device.
//
// Replaces, for a batch of raw ack messages from the feed (LB:94-108: the activeAck topic, 128-message batches):
//   CommonLoadBalancer.processAcknowledgement   CLB:205-232   AcknowledegmentMessage.parse (Message.scala:224-256)
//   CommonLoadBalancer.processCompletion        CLB:260-346   activationSlots.remove + outcome + releaseInvoker
// and, at publish time, the activationSlots.getOrElseUpdate of setupActivation (CLB:148-166).
//
// Kernels
//   owgs_ack_parse_kernel    one thread per message: an iterative JSON scanner (explicit bit stack of containers,
//                            16-byte vector reads through a per-thread window) that validates the whole message
//                            (RFC 8259 grammar, as spray-json 1.3.5 parses it) and records the last occurrence of
//                            the top-level members transid / activationId / isSystemError / invoker / response;
//                            then converts the members CompletionMessage needs (jsonFormat4, Message.scala:204-216):
//                            ActivationId.parse (32 chars [0-9a-f] -> 128-bit key), InvokerInstanceId.instance
//                            (BigDecimal.intValue), userMemory (ByteSize regex + toLong), uniqueName/displayedName
//                            (Option[String]), isSystemError (Option[Boolean]), transid == invokerHealth.
//   owgs_act_*_kernel        activationSlots as an open-addressing table in HBM: key = 128-bit activation id,
//                            value = {action handle, caller ticket}.  Inserts claim an empty slot by 64-bit CAS;
//                            same-key inserts of one batch resolve to the lowest batch index (getOrElseUpdate in
//                            array order); removals of one batch resolve to the lowest message index
//                            (activationSlots.remove in array order: later duplicates see None).
//   owgs_ack_resolve_kernel  processCompletion outcome per message + the release record of releaseInvoker
//                            (SCPB:327-331: invokerSlots.lift(invoker.toInt) -- out-of-range ids are no-ops),
//                            applied in message order by owgs_release_seq_kernel (owgs_kernels.hip).
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "owgs_internal.h"

typedef unsigned long long u64;

// ------------------------------------------------------------------------------------------ byte window
// Reads the message through aligned 16-byte loads; the host pads the byte buffer by 16 bytes so the last block is
// readable.  at(i) returns -1 outside [b, e).
struct Win {
    const uint4* base;
    int64_t b, e, blk;
    uint4 v;
    __device__ Win(const uint8_t* bytes, int64_t b_, int64_t e_) : base((const uint4*)bytes), b(b_), e(e_), blk(-1) {}
    __device__ __forceinline__ int at(int64_t i) {
        if (i >= e || i < b) return -1;
        const int64_t k = i >> 4;
        if (k != blk) {
            v = base[k];
            blk = k;
        }
        const int q = (int)(i >> 2) & 3;
        const uint32_t w = q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w;
        return (int)((w >> ((i & 3) * 8)) & 0xFFu);
    }
};

__device__ __forceinline__ bool is_ws(int c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
__device__ __forceinline__ int hex_val(int c) {
    return (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10 : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : -1;
}

// one decoded UTF-16 code unit of a validated JSON string at i (i points inside the quotes); advances i.
// -1 at the closing quote; non-ASCII bytes decode to 0x10000 (never equal to an ASCII unit)
__device__ __forceinline__ int unit_at(Win& W, int64_t& i) {
    const int c = W.at(i);
    if (c == '"') return -1;
    if (c == '\\') {
        const int e = W.at(i + 1);
        if (e == 'u') {
            const int u = (hex_val(W.at(i + 2)) << 12) | (hex_val(W.at(i + 3)) << 8) | (hex_val(W.at(i + 4)) << 4) |
                          hex_val(W.at(i + 5));
            i += 6;
            return u;
        }
        i += 2;
        return e == 'b' ? 8 : e == 'f' ? 12 : e == 'n' ? 10 : e == 'r' ? 13 : e == 't' ? 9 : e;
    }
    i += 1;
    return c >= 0x80 ? 0x10000 : c;
}

// member names the path reads; decoded name compared against each (key at k = its opening quote)
#define K_AID 0
#define K_INV 1
#define K_SYS 2
#define K_RESP 3
#define K_TID 4
#define K_INSTANCE 5
#define K_UNIQUE 6
#define K_DISPLAYED 7
#define K_USERMEM 8
__constant__ char k_names[9][16] = {"activationId", "invoker", "isSystemError", "response", "transid",
                                    "instance",     "uniqueName", "displayedName", "userMemory"};
__constant__ int k_len[9] = {12, 7, 13, 8, 7, 8, 10, 13, 10};

// bitmask of the candidate names (lo..hi) the decoded key equals
__device__ __forceinline__ int key_match(Win& W, int64_t k, int lo, int hi) {
    int64_t i = k + 1;
    uint32_t alive = ((1u << (hi + 1)) - 1u) & ~((1u << lo) - 1u);
    int n = 0;
    for (;;) {
        const int u = unit_at(W, i);
        if (u < 0) break;
        for (int c = lo; c <= hi; ++c)
            if (((alive >> c) & 1u) && (n >= k_len[c] || u != k_names[c][n])) alive &= ~(1u << c);
        ++n;
        if (!alive) return -1;
    }
    for (int c = lo; c <= hi; ++c)
        if (((alive >> c) & 1u) && n == k_len[c]) return c;
    return -1;
}

#define EV_ERR 1
#define EV_UNSUP 2

// string starting at i (the opening quote); returns the index after the closing quote, or -1 on a grammar error
__device__ __forceinline__ int64_t scan_string(Win& W, int64_t i) {
    ++i;
    for (;;) {
        const int c = W.at(i);
        if (c < 0x20) return -1;  // end of message (-1) or a raw control character
        if (c == '"') return i + 1;
        if (c == '\\') {
            const int e = W.at(i + 1);
            if (e == 'u') {
                if (hex_val(W.at(i + 2)) < 0 || hex_val(W.at(i + 3)) < 0 || hex_val(W.at(i + 4)) < 0 ||
                    hex_val(W.at(i + 5)) < 0)
                    return -1;
                i += 6;
            } else if (e == '"' || e == '\\' || e == '/' || e == 'b' || e == 'f' || e == 'n' || e == 'r' || e == 't') {
                i += 2;
            } else {
                return -1;
            }
        } else {
            ++i;
        }
    }
}

// number at i; returns the index after it, -1 on a grammar error, -2 for an exponent of more than 9 digits
__device__ __forceinline__ int64_t scan_number(Win& W, int64_t i) {
    if (W.at(i) == '-') ++i;
    int c = W.at(i);
    if (c == '0') ++i;
    else if (c >= '1' && c <= '9') {
        while ((c = W.at(i)) >= '0' && c <= '9') ++i;
    } else return -1;
    if (W.at(i) == '.') {
        ++i;
        const int64_t f = i;
        while ((c = W.at(i)) >= '0' && c <= '9') ++i;
        if (i == f) return -1;
    }
    c = W.at(i);
    if (c == 'e' || c == 'E') {
        ++i;
        c = W.at(i);
        if (c == '+' || c == '-') ++i;
        const int64_t f = i;
        while ((c = W.at(i)) >= '0' && c <= '9') ++i;
        if (i == f) return -1;
        if (i - f > 9) return -2;
    }
    return i;
}

// low 64 bits of the integer part of a validated number literal (BigDecimal -> BigInteger.longValue), significant
// digit count in *sig
__device__ __forceinline__ u64 number_bits(Win& W, int64_t i, int* sig) {
    bool neg = false;
    if (W.at(i) == '-') neg = true, ++i;
    const int64_t ib = i;
    int c;
    while ((c = W.at(i)) >= '0' && c <= '9') ++i;
    const int64_t ie = i;
    int64_t fb = i, fe = i;
    if (W.at(i) == '.') {
        fb = ++i;
        while ((c = W.at(i)) >= '0' && c <= '9') ++i;
        fe = i;
    }
    int64_t ex = 0;
    c = W.at(i);
    if (c == 'e' || c == 'E') {
        ++i;
        bool en = false;
        c = W.at(i);
        if (c == '+') ++i;
        else if (c == '-') en = true, ++i;
        while ((c = W.at(i)) >= '0' && c <= '9') ex = ex * 10 + (c - '0'), ++i;
        if (en) ex = -ex;
    }
    const int64_t ni = ie - ib, nf = fe - fb, nd = ni + nf;
    const int64_t shift = ex - nf;
    const int64_t keep = shift >= 0 ? nd : nd + shift;
    u64 v = 0;
    int s = 0;
    bool started = false;
    for (int64_t k = 0; k < nd; ++k) {
        const int d = W.at(k < ni ? ib + k : fb + (k - ni)) - '0';
        started |= d != 0;
        s += started;
        if (k < keep) v = v * 10ull + (u64)d;
    }
    if (shift > 0 && keep > 0)
        for (int64_t k = 0; k < shift && k < 64; ++k) v *= 10ull;
    *sig = s;
    return neg ? 0ull - v : v;
}

// skip one validated value at i (containers by depth counting, strings by scan_string)
__device__ __forceinline__ int64_t skip_value(Win& W, int64_t i) {
    int depth = 0;
    for (;;) {
        const int c = W.at(i);
        if (c == '"') i = scan_string(W, i);
        else if (c == '{' || c == '[') ++depth, ++i;
        else if (c == '}' || c == ']') --depth, ++i;
        else if (c == '-' || (c >= '0' && c <= '9')) i = scan_number(W, i);
        else if (c == 't' || c == 'n') i += 4;
        else if (c == 'f') i += 5;
        else ++i;  // ',' ':' whitespace inside a container
        if (depth == 0) return i;
    }
}

// ByteSize.fromString over the decoded string at a (Size.scala:119-138)
__device__ __forceinline__ bool bytesize_ok(Win& W, int64_t a) {
    int64_t i = a + 1;
    int st = 0;
    u64 val = 0;
    bool ovf = false;
    for (;;) {
        const int u = unit_at(W, i);
        if (u < 0) break;
        const bool ws = u == ' ' || u == '\t' || u == '\n' || u == 0x0B || u == '\f' || u == '\r';
        const bool dg = u >= '0' && u <= '9';
        const int U = (u >= 'a' && u <= 'z') ? u - 32 : u;
        const bool gmk = U == 'G' || U == 'M' || U == 'K';
        switch (st) {
            case 0: st = ws ? 1 : dg ? 2 : 9; if (dg) val = (u64)(u - '0'); break;
            case 1: st = dg ? 2 : 9; if (dg) val = (u64)(u - '0'); break;
            case 2:
                if (dg) {
                    if (val > (u64)(0x7FFFFFFFFFFFFFFFull - (u64)(u - '0')) / 10ull) ovf = true;
                    else val = val * 10ull + (u64)(u - '0');
                } else st = ws ? 3 : gmk ? 4 : U == 'B' ? 5 : 9;
                break;
            case 3: st = gmk ? 4 : U == 'B' ? 5 : 9; break;
            case 4: st = U == 'B' ? 5 : ws ? 6 : 9; break;
            case 5: st = ws ? 6 : 9; break;
            default: st = 9;
        }
        if (st == 9) return false;
    }
    return (st == 4 || st == 5 || st == 6) && !ovf;
}

__device__ __forceinline__ bool num_start(int c) { return c == '-' || (c >= '0' && c <= '9'); }

__global__ __launch_bounds__(256) void owgs_ack_parse_kernel(OwgsAckParseArgs A) {
    const int m = blockIdx.x * 256 + threadIdx.x;
    if (m >= A.n) return;
    const int64_t b = A.off[m], e = A.off[m + 1];
    Win W(A.bytes, b, e);
    int kind = OWGS_ACK_FAIL, inst = -1, sys = 0, health = 0;
    u64 hi = 0, lo = 0;
    // U+FFFF (EF BF BF) reads as spray-json's end-of-input marker: left to the JVM
    bool ffff = false;
    for (int64_t i = b; i + 2 < e && !ffff; ++i)
        ffff = W.at(i) == 0xEF && W.at(i + 1) == 0xBF && W.at(i + 2) == 0xBF;
    if (ffff) {
        kind = OWGS_ACK_UNSUPPORTED;
    } else {
        // ---------------------------------------------------------------- phase 1: grammar, top-level members
        u64 stk = 0;  // bit d-1: container at depth d is an object
        int d = 0, ev = 0;
        int64_t v[5] = {-1, -1, -1, -1, -1};
        int64_t i = b;
        while (is_ws(W.at(i))) ++i;
        const bool top_obj = W.at(i) == '{';
        enum { VALUE, KEY, AFTER } st = VALUE;
        for (;;) {
            if (st == VALUE) {
                const int c = W.at(i);
                if (c == '{' || c == '[') {
                    if (d == 64) { ev = EV_UNSUP; break; }
                    stk = (stk & ~(1ull << d)) | ((u64)(c == '{') << d);
                    ++d;
                    ++i;
                    while (is_ws(W.at(i))) ++i;
                    const int c2 = W.at(i);
                    if (c2 == (c == '{' ? '}' : ']')) { --d; ++i; st = AFTER; }
                    else st = c == '{' ? KEY : VALUE;
                    continue;
                }
                int64_t j;
                if (c == '"') j = scan_string(W, i);
                else if (num_start(c)) j = scan_number(W, i);
                else if (c == 't') j = (W.at(i + 1) == 'r' && W.at(i + 2) == 'u' && W.at(i + 3) == 'e') ? i + 4 : -1;
                else if (c == 'f') j = (W.at(i + 1) == 'a' && W.at(i + 2) == 'l' && W.at(i + 3) == 's' && W.at(i + 4) == 'e') ? i + 5 : -1;
                else if (c == 'n') j = (W.at(i + 1) == 'u' && W.at(i + 2) == 'l' && W.at(i + 3) == 'l') ? i + 4 : -1;
                else j = -1;
                if (j == -2) { ev = EV_UNSUP; break; }
                if (j < 0) { ev = EV_ERR; break; }
                i = j;
                st = AFTER;
            } else if (st == KEY) {
                if (W.at(i) != '"') { ev = EV_ERR; break; }
                const int64_t k = i;
                i = scan_string(W, i);
                if (i < 0) { ev = EV_ERR; break; }
                while (is_ws(W.at(i))) ++i;
                if (W.at(i) != ':') { ev = EV_ERR; break; }
                ++i;
                while (is_ws(W.at(i))) ++i;
                if (d == 1) {
                    const int id = key_match(W, k, K_AID, K_TID);
#pragma unroll
                    for (int q = 0; q < 5; ++q)  // constant indices: v stays in registers (no scratch)
                        if (id == q) v[q] = i;
                }
                st = VALUE;
            } else {  // AFTER a value
                while (is_ws(W.at(i))) ++i;
                if (d == 0) {
                    if (i != e) ev = EV_ERR;
                    break;
                }
                const int c = W.at(i);
                const bool obj = (stk >> (d - 1)) & 1ull;
                if (c == ',') {
                    ++i;
                    while (is_ws(W.at(i))) ++i;
                    st = obj ? KEY : VALUE;
                } else if (c == (obj ? '}' : ']')) {
                    --d;
                    ++i;
                } else {
                    ev = EV_ERR;
                    break;
                }
            }
        }
        if (ev == EV_UNSUP) kind = OWGS_ACK_UNSUPPORTED;
        else if (ev == EV_ERR || !top_obj) kind = OWGS_ACK_FAIL;
        else if (v[K_RESP] >= 0) kind = OWGS_ACK_JVM;
        else if (v[K_INV] < 0) kind = OWGS_ACK_FAIL;
        else {
            // ------------------------------------------------------------ phase 2: CompletionMessage members
            bool fail = v[K_TID] < 0 || v[K_AID] < 0, unsup = false;
            if (v[K_AID] >= 0) {
                const int64_t a = v[K_AID];
                const int c = W.at(a);
                if (c == '"') {
                    int64_t j = a + 1;
                    int len = 0;
                    bool bad = false, nonascii = false;
                    for (;;) {
                        const int u = unit_at(W, j);
                        if (u < 0) break;
                        nonascii |= u >= 0x80;
                        const int h = (u >= '0' && u <= '9') ? u - '0' : (u >= 'a' && u <= 'f') ? u - 'a' + 10 : -1;
                        if (h < 0) bad = true;
                        else if (len < 16) hi = (hi << 4) | (u64)h;
                        else if (len < 32) lo = (lo << 4) | (u64)h;
                        ++len;
                    }
                    if (nonascii) unsup = true;
                    else if (len != 32 || bad) fail = true;
                } else if (num_start(c)) {
                    unsup = true;
                } else {
                    fail = true;
                }
            }
            if (v[K_SYS] >= 0) {
                const int c = W.at(v[K_SYS]);
                if (c == 't') sys = 1;
                else if (c != 'f' && c != 'n') fail = true;
            }
            {
                const int64_t a = v[K_INV];
                if (W.at(a) != '{') fail = true;
                else {
                    int64_t w[4] = {-1, -1, -1, -1};
                    int64_t j = a + 1;
                    while (is_ws(W.at(j))) ++j;
                    if (W.at(j) != '}') {
                        for (;;) {
                            while (is_ws(W.at(j))) ++j;
                            const int64_t k = j;
                            j = scan_string(W, j);
                            while (is_ws(W.at(j))) ++j;
                            ++j;  // ':'
                            while (is_ws(W.at(j))) ++j;
                            const int id = key_match(W, k, K_INSTANCE, K_USERMEM);
#pragma unroll
                            for (int q = 0; q < 4; ++q)  // constant indices: w stays in registers
                                if (id - K_INSTANCE == q) w[q] = j;
                            j = skip_value(W, j);
                            while (is_ws(W.at(j))) ++j;
                            if (W.at(j) != ',') break;
                            ++j;
                        }
                    }
                    if (w[0] < 0 || !num_start(W.at(w[0]))) fail = true;
                    else {
                        int sg;
                        inst = (int32_t)(uint32_t)number_bits(W, w[0], &sg);
                        if (sg > 34) unsup = true;
                    }
                    for (int q = 1; q <= 2; ++q)
                        if (w[q] >= 0 && W.at(w[q]) != '"' && W.at(w[q]) != 'n') fail = true;
                    if (w[3] < 0 || W.at(w[3]) != '"' || !bytesize_ok(W, w[3])) fail = true;
                }
            }
            if (v[K_TID] >= 0 && W.at(v[K_TID]) == '[') {
                int64_t el[3] = {-1, -1, -1};
                int ne = 0;
                int64_t j = v[K_TID] + 1;
                while (is_ws(W.at(j))) ++j;
                if (W.at(j) != ']') {
                    for (;;) {
                        while (is_ws(W.at(j))) ++j;
#pragma unroll
                        for (int q = 0; q < 3; ++q)  // constant indices: el stays in registers
                            if (ne == q) el[q] = j;
                        ++ne;
                        j = skip_value(W, j);
                        while (is_ws(W.at(j))) ++j;
                        if (W.at(j) != ',') break;
                        ++j;
                    }
                }
                if ((ne == 2 || ne == 3) && W.at(el[0]) == '"' && num_start(W.at(el[1])) &&
                    (ne == 2 || W.at(el[2]) == 't' || W.at(el[2]) == 'f')) {
                    // "sid_invokerHealth"
                    int64_t q = el[0] + 1;
                    const char* H = "sid_invokerHealth";
                    bool eq = true;
                    int n = 0;
                    for (;;) {
                        const int u = unit_at(W, q);
                        if (u < 0) break;
                        if (n >= 17 || u != H[n]) eq = false;
                        ++n;
                    }
                    if (eq && n == 17) {
                        int sg;
                        const u64 s0 = number_bits(W, el[1], &sg);
                        if (sg > 34) unsup = true;
                        health = ((int64_t)s0 == A.health_start_ms) && (ne == 2 || W.at(el[2]) == 'f');
                    }
                }
            }
            kind = fail ? OWGS_ACK_FAIL : unsup ? OWGS_ACK_UNSUPPORTED : OWGS_ACK_COMPLETION;
        }
    }
    if (kind != OWGS_ACK_COMPLETION) sys = health = 0;  // only a parsed CompletionMessage carries them
    A.key[m] = make_ulonglong2(hi, lo);
    A.inst[m] = inst;
    A.info[m] = (uint8_t)(kind | (sys << 4) | (health << 5) | (A.forced ? (A.forced[m] & 1) << 6 : 0));
}

// 32 hex chars per id (caller-side ActivationId strings) -> 128-bit keys; ids that are not 32 x [0-9a-f] get
// info = OWGS_ACK_FAIL (the caller's bug: ActivationId guarantees the format)
__global__ __launch_bounds__(256) void owgs_aid_decode_kernel(const char* aid32, int32_t n, const uint8_t* cflags,
                                                              ulonglong2* key, uint8_t* info, int32_t* inst,
                                                              const int32_t* inv) {
    const int m = blockIdx.x * 256 + threadIdx.x;
    if (m >= n) return;
    u64 hi = 0, lo = 0;
    bool bad = false;
    for (int k = 0; k < 32; ++k) {
        const int c = (uint8_t)aid32[(size_t)m * 32 + k];
        const int h = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10 : -1;
        bad |= h < 0;
        if (k < 16) hi = (hi << 4) | (u64)(h & 15);
        else lo = (lo << 4) | (u64)(h & 15);
    }
    key[m] = make_ulonglong2(hi, lo);
    if (info) {
        const uint8_t f = cflags ? cflags[m] : 0;  // bit0 forced, bit1 isSystemError, bit2 transid == invokerHealth
        info[m] = (uint8_t)((bad ? OWGS_ACK_FAIL : OWGS_ACK_COMPLETION) | ((f >> 1) & 1) << 4 | ((f >> 2) & 1) << 5 |
                            (f & 1) << 6);
        inst[m] = inv[m];
    }
}

// ------------------------------------------------------------------------------------------ activation table
__device__ __forceinline__ u64 aid_hash(ulonglong2 k) {
    u64 x = k.x * 0x9E3779B97F4A7C15ull ^ k.y;
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    return x;
}
__device__ __forceinline__ bool keq(ulonglong2 a, ulonglong2 b) { return a.x == b.x && a.y == b.y; }

#define TW_EMPTY 0ull
#define TW_READY 1ull
#define TW_TOMB 2ull
#define TW_CLAIM (1ull << 63)

// track step 1: find or claim a slot for every id of the batch
__global__ __launch_bounds__(256) void owgs_act_claim_kernel(OwgsActTable T, const ulonglong2* key, int32_t n,
                                                             const uint8_t* info, int32_t* slot, uint8_t* state) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    if (info && (info[i] & 7) != OWGS_ACK_COMPLETION) {
        slot[i] = -1;
        state[i] = 3;
        return;
    }
    const ulonglong2 k = key[i];
    const u64 mask = (u64)T.cap - 1;
    u64 s = aid_hash(k) & mask;
    for (u64 probes = 0; probes <= mask; ++probes) {
        u64 w = __hip_atomic_load(&T.tw[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (w == TW_EMPTY) {
            const u64 old = atomicCAS(&T.tw[s], TW_EMPTY, TW_CLAIM | (u64)i);
            if (old == TW_EMPTY) {
                slot[i] = (int32_t)s;
                state[i] = 0;  // claimed in this batch
                atomicMin(&T.owner[s], i);
                return;
            }
            w = old;
        }
        if (w == TW_READY) {
            if (keq(T.tk[s], k)) {
                slot[i] = (int32_t)s;
                state[i] = 1;  // existed before the batch
                return;
            }
        } else if (w & TW_CLAIM) {
            const int j = (int)(w & 0x7FFFFFFFull);
            if (keq(key[j], k)) {
                slot[i] = (int32_t)s;
                state[i] = 0;
                atomicMin(&T.owner[s], i);
                return;
            }
        }
        s = (s + 1) & mask;
    }
    slot[i] = -1;  // table full: the host keeps the load under one half, so this is unreachable
    state[i] = 3;
}

// track step 2: the lowest batch index of each claimed slot writes the entry (getOrElseUpdate in array order)
__global__ __launch_bounds__(256) void owgs_act_fill_kernel(OwgsActTable T, const ulonglong2* key, int32_t n,
                                                            const int32_t* action, const int32_t* ticket,
                                                            const int32_t* slot, const uint8_t* state,
                                                            int32_t* out_ticket, uint8_t* out_existed,
                                                            unsigned long long* counters) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int s = slot[i];
    if (s < 0) {
        out_existed[i] = 2;
        out_ticket[i] = -1;
        return;
    }
    if (state[i] == 1) {
        out_existed[i] = 1;
        out_ticket[i] = T.tv[s].y;
        return;
    }
    const int o = T.owner[s];
    if (o == i) {
        T.tk[s] = key[i];
        T.tv[s] = make_int2(action[i], ticket[i]);
        out_existed[i] = 0;
        out_ticket[i] = ticket[i];
        atomicAdd(&counters[0], 1ull);
    } else {
        out_existed[i] = 1;
        out_ticket[i] = ticket[o];
    }
}

// track step 3: publish the claimed slots and reset the owner words
__global__ __launch_bounds__(256) void owgs_act_publish_kernel(OwgsActTable T, int32_t n, const int32_t* slot,
                                                               const uint8_t* state) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int s = slot[i];
    if (s < 0 || state[i] != 0 || T.owner[s] != i) return;
    T.tw[s] = TW_READY;
    T.owner[s] = 0x7FFFFFFF;
}

// completion step 1: find each message's entry; the lowest message index of an entry removes it
__global__ __launch_bounds__(256) void owgs_act_find_kernel(OwgsActTable T, const ulonglong2* key, int32_t n,
                                                            const uint8_t* info, int32_t* slot) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    int r = -1;
    if ((info[i] & 7) == OWGS_ACK_COMPLETION) {
        const ulonglong2 k = key[i];
        const u64 mask = (u64)T.cap - 1;
        u64 s = aid_hash(k) & mask;
        for (u64 probes = 0; probes <= mask; ++probes) {
            const u64 w = T.tw[s];
            if (w == TW_EMPTY) break;
            if (w == TW_READY && keq(T.tk[s], k)) {
                r = (int)s;
                atomicMin(&T.owner[s], i);
                break;
            }
            s = (s + 1) & mask;
        }
    }
    slot[i] = r;
}

// completion step 2: processCompletion outcome + releaseInvoker record (CLB:286-345, SCPB:327-331)
__global__ __launch_bounds__(256) void owgs_ack_resolve_kernel(OwgsActTable T, int32_t n, const uint8_t* info,
                                                               const int32_t* inst, const int32_t* slot,
                                                               const int32_t* act_mem, const int32_t* act_maxc,
                                                               const int32_t* act_slot, int32_t n_slots,
                                                               int32_t* r_inv, int32_t* r_mem, int32_t* r_maxc,
                                                               int32_t* r_slot, uint8_t* out_kind,
                                                               int32_t* out_ticket, unsigned long long* counters) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int k = info[i] & 7;
    const int s = slot[i];
    int outk = k, tk = -1, ri = 0x7FFFFFFF, rm = 1, rc = 1, rs = 0;
    if (k == OWGS_ACK_COMPLETION) {
        if (s >= 0 && T.owner[s] == i) {
            const int2 v = T.tv[s];
            outk = OWGS_ACK_RELEASED;
            tk = v.y;
            const int inv = inst[i];
            ri = (inv >= 0 && inv < n_slots) ? inv : 0x7FFFFFFF;  // invokerSlots.lift(invoker.toInt)
            rm = act_mem[v.x];
            rc = act_maxc[v.x];
            rs = act_slot[v.x];
            atomicAdd(&counters[1], 1ull);
        } else if ((info[i] >> 5) & 1) {
            outk = OWGS_ACK_HEALTH;  // None if tid == TransactionId.invokerHealth (CLB:320-328)
        } else {
            outk = ((info[i] >> 6) & 1) ? OWGS_ACK_FORCED_NOENTRY : OWGS_ACK_NOENTRY;  // CLB:329-345
        }
    }
    r_inv[i] = ri;
    r_mem[i] = rm;
    r_maxc[i] = rc;
    r_slot[i] = rs;
    out_kind[i] = (uint8_t)outk;
    out_ticket[i] = tk;
}

// completion step 3: tombstone removed entries, reset owner words
__global__ __launch_bounds__(256) void owgs_act_remove_kernel(OwgsActTable T, int32_t n, const int32_t* slot) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int s = slot[i];
    if (s < 0 || T.owner[s] != i) return;
    T.tw[s] = TW_TOMB;
    T.owner[s] = 0x7FFFFFFF;
}

// out_flags = isSystemError | release flags << 1
__global__ __launch_bounds__(256) void owgs_ack_flags_kernel(int32_t n, const uint8_t* info, const uint8_t* rflags,
                                                             const uint8_t* out_kind, uint8_t* out_flags) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const bool rel = out_kind[i] == OWGS_ACK_RELEASED;
    out_flags[i] = (uint8_t)(((info[i] >> 4) & 1) | (rel ? (rflags[i] & 3) << 1 : 0));
}

// rehash live entries into a fresh table (all keys distinct: plain CAS insertion)
__global__ __launch_bounds__(256) void owgs_act_rehash_kernel(OwgsActTable O, OwgsActTable T) {
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= O.cap || O.tw[s] != TW_READY) return;
    const ulonglong2 k = O.tk[s];
    const u64 mask = (u64)T.cap - 1;
    u64 t = aid_hash(k) & mask;
    for (;;) {
        if (atomicCAS(&T.tw[t], TW_EMPTY, TW_READY) == TW_EMPTY) {
            T.tk[t] = k;
            T.tv[t] = O.tv[s];
            return;
        }
        t = (t + 1) & mask;
    }
}

__global__ __launch_bounds__(256) void owgs_act_init_kernel(OwgsActTable T) {
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= T.cap) return;
    T.tw[s] = TW_EMPTY;
    T.owner[s] = 0x7FFFFFFF;
}

// ------------------------------------------------------------------------------------------ launchers
#define GRID(n) dim3((unsigned)(((n) + 255) / 256)), dim3(256), 0, st

extern "C" hipError_t owgs_launch_ack_parse(const OwgsAckParseArgs* a, hipStream_t st) {
    if (a->n <= 0) return hipSuccess;
    hipLaunchKernelGGL(owgs_ack_parse_kernel, GRID(a->n), *a);
    return hipGetLastError();
}

extern "C" hipError_t owgs_launch_aid_decode(const char* aid32, int32_t n, const uint8_t* cflags, ulonglong2* key,
                                             uint8_t* info, int32_t* inst, const int32_t* inv, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(owgs_aid_decode_kernel, GRID(n), aid32, n, cflags, key, info, inst, inv);
    return hipGetLastError();
}

extern "C" hipError_t owgs_launch_act_init(const OwgsActTable* T, hipStream_t st) {
    hipLaunchKernelGGL(owgs_act_init_kernel, GRID(T->cap), *T);
    return hipGetLastError();
}

extern "C" hipError_t owgs_launch_act_rehash(const OwgsActTable* O, const OwgsActTable* T, hipStream_t st) {
    hipLaunchKernelGGL(owgs_act_rehash_kernel, GRID(O->cap), *O, *T);
    return hipGetLastError();
}

extern "C" hipError_t owgs_launch_act_track(const OwgsActTable* T, const ulonglong2* key, int32_t n,
                                            const int32_t* action, const int32_t* ticket, int32_t* slot,
                                            uint8_t* state, int32_t* out_ticket, uint8_t* out_existed,
                                            unsigned long long* counters, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(owgs_act_claim_kernel, GRID(n), *T, key, n, (const uint8_t*)nullptr, slot, state);
    hipLaunchKernelGGL(owgs_act_fill_kernel, GRID(n), *T, key, n, action, ticket, slot, state, out_ticket,
                       out_existed, counters);
    hipLaunchKernelGGL(owgs_act_publish_kernel, GRID(n), *T, n, slot, state);
    return hipGetLastError();
}

// find + resolve: afterwards r_* hold the release records for owgs_release_seq_kernel (message order)
extern "C" hipError_t owgs_launch_ack_complete(const OwgsActTable* T, const OwgsAckCompleteArgs* a, hipStream_t st) {
    if (a->n <= 0) return hipSuccess;
    hipLaunchKernelGGL(owgs_act_find_kernel, GRID(a->n), *T, a->key, a->n, a->info, a->slot);
    hipLaunchKernelGGL(owgs_ack_resolve_kernel, GRID(a->n), *T, a->n, a->info, a->inst, a->slot, a->act_mem,
                       a->act_maxc, a->act_slot, a->n_slots, a->r_inv, a->r_mem, a->r_maxc, a->r_slot, a->out_kind,
                       a->out_ticket, a->counters);
    hipLaunchKernelGGL(owgs_act_remove_kernel, GRID(a->n), *T, a->n, a->slot);
    return hipGetLastError();
}

extern "C" hipError_t owgs_launch_ack_flags(int32_t n, const uint8_t* info, const uint8_t* rflags,
                                            const uint8_t* out_kind, uint8_t* out_flags, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(owgs_ack_flags_kernel, GRID(n), n, info, rflags, out_kind, out_flags);
    return hipGetLastError();
}
