/*
 * owack_oracle.c -- TEST INFRASTRUCTURE (CPU oracle): restatement of the completion-ack path for the parity tests.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it; the product path never does.
 *
 * Follows, in the reference repository:
 *   CommonLoadBalancer.processAcknowledgement   core/controller/.../loadBalancer/CommonLoadBalancer.scala:205-232
 *   CommonLoadBalancer.processCompletion        CommonLoadBalancer.scala:260-346 (activationSlots.remove, outcomes)
 *   CommonLoadBalancer.setupActivation          CommonLoadBalancer.scala:148-166 (activationSlots.getOrElseUpdate)
 *   AcknowledegmentMessage.serdes.read          common/scala/.../core/connector/Message.scala:237-256
 *   CompletionMessage.serdes (jsonFormat4)      Message.scala:204-216; fields transid, activationId, isSystemError,
 *                                               invoker (Message.scala:85-100)
 *   InvokerInstanceId.serdes (jsonFormat4)      common/scala/.../core/entity/InstanceId.scala:31-49
 *   ByteSize.fromString / serdes                common/scala/.../core/entity/Size.scala:64-66, 119-138, 166-172
 *   ActivationId.parse / serdes                 common/scala/.../core/entity/ActivationId.scala:50-95
 *   TransactionId.serdes, invokerHealth         common/scala/.../common/TransactionId.scala:216-253
 * and the JSON grammar of spray-json 1.3.5 (common/scala/build.gradle:37; an un-vendored dependency: its parser is
 * restated here as RFC 8259 -- whitespace " \t\n\r", strict numbers, escapes \" \\ \/ \b \f \n \r \t \uXXXX, no raw
 * control characters in strings, the last duplicate member wins as in spray's JsObject Map).
 *
 * Written as recursive descent (one function per grammar rule), independently of the GPU kernel's iterative scanner.
 *
 * Outcome of one message (owa_parse):
 *   OWA_FAIL        Failure branch of processAcknowledgement (CLB:226-228): not JSON, not an object, or a required
 *                   member missing / of the wrong type
 *   OWA_JVM         the message has a "response" member (ResultMessage / CombinedCompletionAndResultMessage): the
 *                   WhiskActivation inside is deserialised by the JVM, which then completes the slot itself
 *   OWA_UNSUPPORTED outside the device parser's contract (documented limits, see owgs.h): the JVM parses it
 *   OWA_COMPLETION  a CompletionMessage: activation id, invoker instance, isSystemError, transid == invokerHealth
 * Precedence: U+FFFF anywhere -> UNSUPPORTED; then the first grammar event left to right (error -> FAIL, container
 * depth > 64 or an exponent of more than 9 digits -> UNSUPPORTED); then member conversion, where any definite
 * failure -> FAIL, else any unsupported member -> UNSUPPORTED.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OWA_FAIL 0
#define OWA_JVM 1
#define OWA_UNSUPPORTED 2
#define OWA_COMPLETION 3

#define MAXDEPTH 64

typedef struct {
    const uint8_t* s;
    int64_t n, i;
    int ev;  /* 0 none, 1 error, 2 unsupported */
    /* last occurrence of each top-level member: value start (or -1) */
    int64_t v_aid, v_inv, v_sys, v_resp, v_tid;
} P;

static int cur(P* p) { return p->i < p->n ? p->s[p->i] : -1; }
static void ws(P* p) {
    while (p->i < p->n && (p->s[p->i] == ' ' || p->s[p->i] == '\t' || p->s[p->i] == '\n' || p->s[p->i] == '\r')) p->i++;
}
static int hexv(int c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

static int value(P* p, int depth);

/* string: validates, leaves p->i after the closing quote */
static int string(P* p) {
    if (cur(p) != '"') return p->ev = 1, 0;
    p->i++;
    for (;;) {
        int c = cur(p);
        if (c < 0) return p->ev = 1, 0;
        if (c == '"') {
            p->i++;
            return 1;
        }
        if (c < 0x20) return p->ev = 1, 0;
        if (c == '\\') {
            p->i++;
            c = cur(p);
            if (c == 'u') {
                for (int k = 1; k <= 4; ++k)
                    if (p->i + k >= p->n || hexv(p->s[p->i + k]) < 0) return p->ev = 1, 0;
                p->i += 5;
                continue;
            }
            if (c == '"' || c == '\\' || c == '/' || c == 'b' || c == 'f' || c == 'n' || c == 'r' || c == 't') {
                p->i++;
                continue;
            }
            return p->ev = 1, 0;
        }
        p->i++;
    }
}

static int digits(P* p) {
    int64_t b = p->i;
    while (cur(p) >= '0' && cur(p) <= '9') p->i++;
    return (int)(p->i > b);
}

static int number(P* p) {
    if (cur(p) == '-') p->i++;
    if (cur(p) == '0') p->i++;
    else if (cur(p) >= '1' && cur(p) <= '9') digits(p);
    else return p->ev = 1, 0;
    if (cur(p) == '.') {
        p->i++;
        if (!digits(p)) return p->ev = 1, 0;
    }
    if (cur(p) == 'e' || cur(p) == 'E') {
        p->i++;
        if (cur(p) == '+' || cur(p) == '-') p->i++;
        int64_t b = p->i;
        if (!digits(p)) return p->ev = 1, 0;
        if (p->i - b > 9) return p->ev = 2, 0;
    }
    return 1;
}

static int literal(P* p, const char* w) {
    size_t L = strlen(w);
    if (p->i + (int64_t)L > p->n || memcmp(p->s + p->i, w, L) != 0) return p->ev = 1, 0;
    p->i += (int64_t)L;
    return 1;
}

/* decoded UTF-16 code units of the JSON string at position a (validated) compared with an ASCII literal */
static int str_eq(const uint8_t* s, int64_t a, const char* lit) {
    int64_t i = a + 1;
    size_t k = 0, L = strlen(lit);
    for (;;) {
        int c = s[i];
        int unit;
        if (c == '"') return k == L;
        if (c == '\\') {
            int e = s[i + 1];
            if (e == 'u') {
                unit = (hexv(s[i + 2]) << 12) | (hexv(s[i + 3]) << 8) | (hexv(s[i + 4]) << 4) | hexv(s[i + 5]);
                i += 6;
            } else {
                unit = e == 'b' ? 8 : e == 'f' ? 12 : e == 'n' ? 10 : e == 'r' ? 13 : e == 't' ? 9 : e;
                i += 2;
            }
        } else {
            unit = c >= 0x80 ? 0x10000 : c;  /* any non-ASCII byte decodes to a non-ASCII unit */
            i += 1;
        }
        if (k >= L || unit != (unsigned char)lit[k]) return 0;
        k++;
    }
}

static int object(P* p, int depth) {
    p->i++; /* '{' */
    ws(p);
    if (cur(p) == '}') {
        p->i++;
        return 1;
    }
    for (;;) {
        ws(p);
        int64_t k = p->i;
        if (!string(p)) return 0;
        ws(p);
        if (cur(p) != ':') return p->ev = 1, 0;
        p->i++;
        ws(p);
        int64_t v = p->i;
        if (!value(p, depth)) return 0;
        if (depth == 1) {
            if (str_eq(p->s, k, "activationId")) p->v_aid = v;
            else if (str_eq(p->s, k, "invoker")) p->v_inv = v;
            else if (str_eq(p->s, k, "isSystemError")) p->v_sys = v;
            else if (str_eq(p->s, k, "response")) p->v_resp = v;
            else if (str_eq(p->s, k, "transid")) p->v_tid = v;
        }
        ws(p);
        if (cur(p) == ',') {
            p->i++;
            continue;
        }
        if (cur(p) == '}') {
            p->i++;
            return 1;
        }
        return p->ev = 1, 0;
    }
}

static int array(P* p, int depth) {
    p->i++; /* '[' */
    ws(p);
    if (cur(p) == ']') {
        p->i++;
        return 1;
    }
    for (;;) {
        ws(p);
        if (!value(p, depth)) return 0;
        ws(p);
        if (cur(p) == ',') {
            p->i++;
            continue;
        }
        if (cur(p) == ']') {
            p->i++;
            return 1;
        }
        return p->ev = 1, 0;
    }
}

static int value(P* p, int depth) {
    int c = cur(p);
    if (c == '{' || c == '[') {
        if (depth + 1 > MAXDEPTH) return p->ev = 2, 0;
        return c == '{' ? object(p, depth + 1) : array(p, depth + 1);
    }
    if (c == '"') return string(p);
    if (c == '-' || (c >= '0' && c <= '9')) return number(p);
    if (c == 't') return literal(p, "true");
    if (c == 'f') return literal(p, "false");
    if (c == 'n') return literal(p, "null");
    return p->ev = 1, 0;
}

/* ---- member conversion (phase 2) ---- */

/* low 64 bits of BigDecimal(literal).toBigInteger (Java longValue / intValue semantics); *sig = significant digits */
static uint64_t num_low_bits(const uint8_t* s, int64_t a, int* sig) {
    int64_t i = a;
    int neg = 0;
    if (s[i] == '-') neg = 1, i++;
    int64_t ib = i;
    while (s[i] >= '0' && s[i] <= '9') i++;
    int64_t ie = i, fb = i, fe = i;
    if (s[i] == '.') {
        fb = i + 1;
        i = fb;
        while (s[i] >= '0' && s[i] <= '9') i++;
        fe = i;
    }
    int64_t e = 0;
    if (s[i] == 'e' || s[i] == 'E') {
        i++;
        int en = 0;
        if (s[i] == '+') i++;
        else if (s[i] == '-') en = 1, i++;
        while (s[i] >= '0' && s[i] <= '9') e = e * 10 + (s[i++] - '0');
        if (en) e = -e;
    }
    /* digit sequence D = int digits ++ frac digits; value = D * 10^(e - fracLen) */
    const int64_t nd = (ie - ib) + (fe - fb);
    int started = 0;
    *sig = 0;
    for (int64_t k = 0; k < nd; ++k) {
        int d = k < ie - ib ? s[ib + k] - '0' : s[fb + k - (ie - ib)] - '0';
        if (d) started = 1;
        if (started) (*sig)++;
    }
    const int64_t shift = e - (fe - fb);
    int64_t keep = shift >= 0 ? nd : nd + shift; /* digits that stay in the integer part */
    uint64_t v = 0;
    for (int64_t k = 0; k < keep; ++k) {
        int d = k < ie - ib ? s[ib + k] - '0' : s[fb + k - (ie - ib)] - '0';
        v = v * 10u + (uint64_t)d;
    }
    if (shift > 0 && keep > 0) {
        for (int64_t k = 0; k < shift && k < 64; ++k) v *= 10u;
    }
    return neg ? (uint64_t)0 - v : v;
}

/* skip a validated value starting at a; returns the index after it */
static int64_t skip_value(const uint8_t* s, int64_t n, int64_t a) {
    P q;
    memset(&q, 0, sizeof(q));
    q.s = s;
    q.n = n;
    q.i = a;
    value(&q, 2); /* depth limit was already checked in phase 1; members below depth 1 are not recorded */
    return q.i;
}

/* ByteSize.fromString regex (?i)\s?(\d+)\s?(GB|MB|KB|B|G|M|K)\s? over the decoded string; size.toLong must fit */
static int bytesize_ok(const uint8_t* s, int64_t a) {
    /* decode into code units on the fly */
    int64_t i = a + 1;
    int st = 0; /* 0 start, 1 after lead ws, 2 digits, 3 after mid ws, 4 unit G/M/K, 5 unit done, 6 trail ws */
    uint64_t val = 0;
    int ovf = 0;
    for (;;) {
        int c = s[i], u;
        if (c == '"') break;
        if (c == '\\') {
            int e = s[i + 1];
            if (e == 'u') {
                u = (hexv(s[i + 2]) << 12) | (hexv(s[i + 3]) << 8) | (hexv(s[i + 4]) << 4) | hexv(s[i + 5]);
                i += 6;
            } else {
                u = e == 'b' ? 8 : e == 'f' ? 12 : e == 'n' ? 10 : e == 'r' ? 13 : e == 't' ? 9 : e;
                i += 2;
            }
        } else {
            u = c >= 0x80 ? 0x10000 : c;
            i++;
        }
        const int isws = u == ' ' || u == '\t' || u == '\n' || u == 0x0B || u == '\f' || u == '\r';
        const int isd = u >= '0' && u <= '9';
        const int U = (u >= 'a' && u <= 'z') ? u - 32 : u;
        switch (st) {
            case 0:
                if (isws) st = 1;
                else if (isd) st = 2, val = (uint64_t)(u - '0');
                else return 0;
                break;
            case 1:
                if (isd) st = 2, val = (uint64_t)(u - '0');
                else return 0;
                break;
            case 2:
                if (isd) {
                    if (val > (uint64_t)(INT64_MAX - (u - '0')) / 10u) ovf = 1;
                    else val = val * 10u + (uint64_t)(u - '0');
                } else if (isws) st = 3;
                else if (U == 'G' || U == 'M' || U == 'K') st = 4;
                else if (U == 'B') st = 5;
                else return 0;
                break;
            case 3:
                if (U == 'G' || U == 'M' || U == 'K') st = 4;
                else if (U == 'B') st = 5;
                else return 0;
                break;
            case 4:
                if (U == 'B') st = 5;
                else if (isws) st = 6;
                else return 0;
                break;
            case 5:
                if (isws) st = 6;
                else return 0;
                break;
            default:
                return 0;
        }
    }
    if (!(st == 4 || st == 5 || st == 6)) return 0;
    return !ovf;
}

typedef struct {
    int32_t kind;
    int32_t instance;
    int32_t syserr;
    int32_t health;
    uint64_t aid_hi, aid_lo;
} owa_ack;

int owa_parse(const char* msg, int64_t n, int64_t health_start_ms, owa_ack* out) {
    const uint8_t* s = (const uint8_t*)msg;
    memset(out, 0, sizeof(*out));
    out->instance = -1;
    for (int64_t i = 0; i + 2 < n; ++i)
        if (s[i] == 0xEF && s[i + 1] == 0xBF && s[i + 2] == 0xBF) return out->kind = OWA_UNSUPPORTED;
    P p;
    memset(&p, 0, sizeof(p));
    p.s = s;
    p.n = n;
    p.v_aid = p.v_inv = p.v_sys = p.v_resp = p.v_tid = -1;
    ws(&p);
    if (!value(&p, 0)) return out->kind = (p.ev == 2 ? OWA_UNSUPPORTED : OWA_FAIL);
    ws(&p);
    if (p.i != n) return out->kind = OWA_FAIL;
    {  /* val JsObject(fields) = json (Message.scala:246): a MatchError for any other top-level value */
        int64_t f = 0;
        while (s[f] == ' ' || s[f] == '\t' || s[f] == '\n' || s[f] == '\r') f++;
        if (s[f] != '{') return out->kind = OWA_FAIL;
    }
    if (p.v_resp >= 0) return out->kind = OWA_JVM;
    if (p.v_inv < 0) return out->kind = OWA_FAIL; /* ResultMessage without "response" */
    /* CompletionMessage: transid, activationId, isSystemError, invoker */
    int fail = 0, unsup = 0;
    if (p.v_tid < 0) fail = 1;
    /* activationId */
    if (p.v_aid < 0) fail = 1;
    else {
        int64_t a = p.v_aid;
        if (s[a] == '"') {
            int64_t i = a + 1;
            int len = 0, nonascii = 0, bad = 0;
            uint64_t hi = 0, lo = 0;
            for (;;) {
                int c = s[i], u;
                if (c == '"') break;
                if (c == '\\') {
                    int e = s[i + 1];
                    if (e == 'u') {
                        u = (hexv(s[i + 2]) << 12) | (hexv(s[i + 3]) << 8) | (hexv(s[i + 4]) << 4) | hexv(s[i + 5]);
                        i += 6;
                    } else {
                        u = e == 'b' ? 8 : e == 'f' ? 12 : e == 'n' ? 10 : e == 'r' ? 13 : e == 't' ? 9 : e;
                        i += 2;
                    }
                } else {
                    u = c;
                    i++;
                }
                if (u >= 0x80) nonascii = 1;
                int h = (u >= '0' && u <= '9') ? u - '0' : (u >= 'a' && u <= 'f') ? u - 'a' + 10 : -1;
                if (h < 0) bad = 1;
                else if (len < 32) {
                    if (len < 16) hi = (hi << 4) | (uint64_t)h;
                    else lo = (lo << 4) | (uint64_t)h;
                }
                len++;
            }
            /* ActivationId.parse: length 32 (UTF-16 units), every char isDigit or a-f (ActivationId.scala:50-68);
             * Character.isDigit accepts non-ASCII digits too: those ids are left to the JVM */
            if (nonascii) unsup = 1;
            else if (len != 32 || bad) fail = 1;
            out->aid_hi = hi;
            out->aid_lo = lo;
        } else if (s[a] == '-' || (s[a] >= '0' && s[a] <= '9')) {
            unsup = 1; /* JsNumber(n) => parse(n.toString): BigDecimal rendering, left to the JVM */
        } else {
            fail = 1;
        }
    }
    /* isSystemError: Option[Boolean] */
    if (p.v_sys >= 0) {
        int c = s[p.v_sys];
        if (c == 't') out->syserr = 1;
        else if (c == 'f' || c == 'n') out->syserr = 0;
        else fail = 1;
    }
    /* invoker: InvokerInstanceId(instance: Int, uniqueName: Option[String], displayedName: Option[String],
     * userMemory: ByteSize) */
    {
        int64_t a = p.v_inv;
        if (s[a] != '{') fail = 1;
        else {
            int64_t v_in = -1, v_un = -1, v_dn = -1, v_um = -1;
            int64_t i = a + 1;
            P q;
            memset(&q, 0, sizeof(q));
            q.s = s;
            q.n = n;
            q.i = i;
            ws(&q);
            if (cur(&q) != '}') {
                for (;;) {
                    ws(&q);
                    int64_t k = q.i;
                    string(&q);
                    ws(&q);
                    q.i++; /* ':' */
                    ws(&q);
                    int64_t v = q.i;
                    q.i = skip_value(s, n, v);
                    if (str_eq(s, k, "instance")) v_in = v;
                    else if (str_eq(s, k, "uniqueName")) v_un = v;
                    else if (str_eq(s, k, "displayedName")) v_dn = v;
                    else if (str_eq(s, k, "userMemory")) v_um = v;
                    ws(&q);
                    if (cur(&q) == ',') {
                        q.i++;
                        continue;
                    }
                    break;
                }
            }
            if (v_in < 0) fail = 1;
            else if (s[v_in] == '-' || (s[v_in] >= '0' && s[v_in] <= '9')) {
                int sig;
                uint64_t lb = num_low_bits(s, v_in, &sig);
                if (sig > 34) unsup = 1;
                out->instance = (int32_t)(uint32_t)lb;
            } else fail = 1;
            if (v_un >= 0 && !(s[v_un] == '"' || s[v_un] == 'n')) fail = 1;
            if (v_dn >= 0 && !(s[v_dn] == '"' || s[v_dn] == 'n')) fail = 1;
            if (v_um < 0 || s[v_um] != '"' || !bytesize_ok(s, v_um)) fail = 1;
        }
    }
    /* transid == TransactionId.invokerHealth: JsArray(JsString("sid_invokerHealth"), JsNumber(start)[, false]) */
    if (p.v_tid >= 0 && s[p.v_tid] == '[') {
        int64_t el[4];
        int ne = 0;
        P q;
        memset(&q, 0, sizeof(q));
        q.s = s;
        q.n = n;
        q.i = p.v_tid + 1;
        ws(&q);
        if (cur(&q) != ']') {
            for (;;) {
                ws(&q);
                if (ne < 4) el[ne] = q.i;
                ne++;
                q.i = skip_value(s, n, q.i);
                ws(&q);
                if (cur(&q) == ',') {
                    q.i++;
                    continue;
                }
                break;
            }
        }
        if ((ne == 2 || ne == 3) && s[el[0]] == '"' && (s[el[1]] == '-' || (s[el[1]] >= '0' && s[el[1]] <= '9')) &&
            (ne == 2 || s[el[2]] == 't' || s[el[2]] == 'f') && str_eq(s, el[0], "sid_invokerHealth")) {
            int sig;
            uint64_t st = num_low_bits(s, el[1], &sig);
            if (sig > 34) unsup = 1;
            out->health = (int64_t)st == health_start_ms && (ne == 2 || s[el[2]] == 'f');
        }
    }
    if (fail) return out->kind = OWA_FAIL;
    if (unsup) return out->kind = OWA_UNSUPPORTED;
    return out->kind = OWA_COMPLETION;
}

int owa_parse_batch(int32_t n, const char* bytes, const int64_t* off, int64_t health_start_ms, int32_t* kind,
                    int32_t* instance, int32_t* syserr, int32_t* health, uint64_t* aid /* 2n */) {
    for (int32_t i = 0; i < n; ++i) {
        owa_ack a;
        owa_parse(bytes + off[i], off[i + 1] - off[i], health_start_ms, &a);
        kind[i] = a.kind;
        instance[i] = a.instance;
        syserr[i] = a.syserr;
        health[i] = a.health;
        aid[2 * i] = a.aid_hi;
        aid[2 * i + 1] = a.aid_lo;
    }
    return 0;
}

/* ---- activationSlots: a map aid -> (action, ticket), CLB:60 TrieMap restated as a linear-probing table ---- */
typedef struct {
    int64_t cap, live;
    uint64_t* k;  /* 2 per slot; hi = ~0 & lo = ~0 marks empty */
    int32_t* act;
    int32_t* ticket;
    uint8_t* used; /* 0 empty, 1 live, 2 deleted */
} owa_table;

owa_table* owa_table_new(int64_t cap_pow2) {
    owa_table* t = (owa_table*)calloc(1, sizeof(owa_table));
    t->cap = cap_pow2;
    t->k = (uint64_t*)calloc((size_t)(2 * cap_pow2), 8);
    t->act = (int32_t*)calloc((size_t)cap_pow2, 4);
    t->ticket = (int32_t*)calloc((size_t)cap_pow2, 4);
    t->used = (uint8_t*)calloc((size_t)cap_pow2, 1);
    return t;
}

void owa_table_free(owa_table* t) {
    if (!t) return;
    free(t->k);
    free(t->act);
    free(t->ticket);
    free(t->used);
    free(t);
}

static uint64_t mix(uint64_t hi, uint64_t lo) {
    uint64_t x = hi * 0x9E3779B97F4A7C15ull ^ lo;
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    return x;
}

static int64_t find(const owa_table* t, uint64_t hi, uint64_t lo) {
    for (int64_t s = (int64_t)(mix(hi, lo) & (uint64_t)(t->cap - 1)), k = 0; k < t->cap; ++k, s = (s + 1) & (t->cap - 1)) {
        if (t->used[s] == 0) return -1;
        if (t->used[s] == 1 && t->k[2 * s] == hi && t->k[2 * s + 1] == lo) return s;
    }
    return -1;
}

/* setupActivation: activationSlots.getOrElseUpdate(aid, entry) (CLB:148-166). returns 1 if it already existed */
int owa_track(owa_table* t, uint64_t hi, uint64_t lo, int32_t action, int32_t ticket, int32_t* out_ticket) {
    int64_t s = find(t, hi, lo);
    if (s >= 0) {
        *out_ticket = t->ticket[s];
        return 1;
    }
    for (s = (int64_t)(mix(hi, lo) & (uint64_t)(t->cap - 1));; s = (s + 1) & (t->cap - 1))
        if (t->used[s] != 1) break;
    t->used[s] = 1;
    t->k[2 * s] = hi;
    t->k[2 * s + 1] = lo;
    t->act[s] = action;
    t->ticket[s] = ticket;
    t->live++;
    *out_ticket = ticket;
    return 0;
}

/* activationSlots.remove(aid): returns 1 and the entry if present */
int owa_remove(owa_table* t, uint64_t hi, uint64_t lo, int32_t* action, int32_t* ticket) {
    int64_t s = find(t, hi, lo);
    if (s < 0) return 0;
    *action = t->act[s];
    *ticket = t->ticket[s];
    t->used[s] = 2;
    t->live--;
    return 1;
}

int64_t owa_live(const owa_table* t) { return t->live; }

/* processAcknowledgement for a batch, in order (CLB:205-232 -> 260-346), over an oracle BalancerState:
 * kind[i] = OWA_FAIL / OWA_JVM / OWA_UNSUPPORTED or the processCompletion outcome 3 released, 4 health ack,
 * 5 no entry (regular after forced); flags = isSystemError | release flags << 1 (NoSuchElement 1, overflow 2). */
extern int owo_release(void* st, int32_t invoker, int32_t action);
int owa_process_acks(owa_table* t, void* st, int32_t n, const char* bytes, const int64_t* off, int64_t health_ms,
                     int32_t* kind, int32_t* instance, int32_t* ticket, uint8_t* flags) {
    for (int32_t i = 0; i < n; ++i) {
        owa_ack a;
        owa_parse(bytes + off[i], off[i + 1] - off[i], health_ms, &a);
        kind[i] = a.kind;
        instance[i] = a.instance;
        ticket[i] = -1;
        flags[i] = 0;
        if (a.kind != OWA_COMPLETION) continue;
        flags[i] = (uint8_t)(a.syserr & 1);
        int32_t act, tk;
        if (owa_remove(t, a.aid_hi, a.aid_lo, &act, &tk)) {
            kind[i] = 3;
            ticket[i] = tk;
            const int rc = owo_release(st, a.instance, act); /* invokerSlots.lift: out-of-range ids return 0 */
            flags[i] |= (uint8_t)((rc == -4 ? 1 : rc == -5 ? 2 : 0) << 1);
        } else {
            kind[i] = a.health ? 4 : 5;
        }
    }
    return 0;
}
