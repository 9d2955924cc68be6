/*
 * owmsg_oracle.c -- TEST INFRASTRUCTURE (CPU oracle): restatement of ActivationMessage serialisation and the
 * per-invoker topic fan-out.  Only tests/ load it; the product path never does.
 *
 * Follows, in the reference repository:
 *   ActivationMessage (11 fields) + serialize = serdes.write(this).compactPrint   common/scala/.../core/connector/
 *                                                                                 Message.scala:51-70, 170-175
 *   jsonFormat11 field order: transid, action, revision, user, activationId, rootControllerIndex, blocking, content,
 *   initArgs, cause, traceContext; Option fields that are None are omitted (DefaultJsonProtocol without NullOptions)
 *   TransactionId.serdes.write: ["id", start] or ["id", start, true]        common/.../TransactionId.scala:235-241
 *   ActivationId serdes: the 32-char lowercase hex string                    core/entity/ActivationId.scala:50-95
 *   sendActivationToInvoker: topic s"invoker${invoker.toInt}", one send per activation in publish order
 *                                                                             core/controller/.../CommonLoadBalancer.scala:175-198
 * and spray-json 1.3.5's CompactPrinter (an un-vendored dependency, restated): strings are printed with `"` -> \",
 * `\` -> \\, \b \f \n \r \t, every other UTF-16 unit below 0x20, DEL (0x7F) and every non-ASCII unit as \u + lowercase
 * hex (Integer.toHexString, left-padded to 4 digits); JsNumber(Long) prints its decimal digits.
 *
 * The invariant members of a message are the caller's templates, printed once per (action, identity): part A =
 * `"action":...,"revision":...,"user":...` and part B = the initArgs array; the controller's rootControllerIndex is
 * one JSON value per context; content (the JsObject of parameters) and traceContext arrive printed.  The
 * per-activation members (transid, activationId, blocking, cause) are formatted here.
 *
 * Output: the messages of every activation with invoker >= 0, grouped by invoker id ascending (one topic each), in
 * stream order within a topic (Kafka's per-topic send order).
 */
#include <stdint.h>
#include <string.h>

#define OWM_BLOCKING 1
#define OWM_EXTRA_LOGGING 2
#define OWM_HAS_CONTENT 4
#define OWM_HAS_CAUSE 8
#define OWM_HAS_TRACE 16

typedef struct {
    char* p;
    int64_t n, cap;
    int overflow;
} sbuf;

static void put(sbuf* b, const char* s, int64_t n) {
    if (b->n + n > b->cap) {
        b->overflow = 1;
    } else if (n > 0) {
        memcpy(b->p + b->n, s, (size_t)n);
    }
    b->n += n;
}
static void puts_(sbuf* b, const char* s) { put(b, s, (int64_t)strlen(s)); }

static const char HEX[] = "0123456789abcdef";

/* one UTF-16 unit as spray prints it inside a string */
static void put_unit(sbuf* b, unsigned u) {
    char t[8];
    switch (u) {
        case '"': puts_(b, "\\\""); return;
        case '\\': puts_(b, "\\\\"); return;
        case '\b': puts_(b, "\\b"); return;
        case '\f': puts_(b, "\\f"); return;
        case '\n': puts_(b, "\\n"); return;
        case '\r': puts_(b, "\\r"); return;
        case '\t': puts_(b, "\\t"); return;
        default: break;
    }
    if (u >= 0x20 && u < 0x7F) {
        t[0] = (char)u;
        put(b, t, 1);
        return;
    }
    t[0] = '\\';
    t[1] = 'u';
    t[2] = HEX[(u >> 12) & 15];
    t[3] = HEX[(u >> 8) & 15];
    t[4] = HEX[(u >> 4) & 15];
    t[5] = HEX[u & 15];
    put(b, t, 6);
}

/* a UTF-8 byte string printed as a JSON string (decoded to UTF-16 units); -1 on malformed UTF-8 */
static int put_string(sbuf* b, const uint8_t* s, int64_t n) {
    puts_(b, "\"");
    for (int64_t i = 0; i < n;) {
        unsigned c = s[i], cp, need;
        if (c < 0x80) {
            put_unit(b, c);
            ++i;
            continue;
        }
        if ((c & 0xE0) == 0xC0) { cp = c & 0x1F; need = 1; }
        else if ((c & 0xF0) == 0xE0) { cp = c & 0x0F; need = 2; }
        else if ((c & 0xF8) == 0xF0) { cp = c & 0x07; need = 3; }
        else return -1;
        for (unsigned k = 1; k <= need; ++k) {
            if (i + k >= n || (s[i + k] & 0xC0) != 0x80) return -1;
            cp = cp << 6 | (s[i + k] & 0x3F);
        }
        /* shortest form, no surrogates, <= U+10FFFF */
        if ((need == 1 && cp < 0x80) || (need == 2 && cp < 0x800) || (need == 3 && cp < 0x10000) || cp > 0x10FFFF ||
            (cp >= 0xD800 && cp <= 0xDFFF))
            return -1;
        if (cp >= 0x10000) {
            put_unit(b, 0xD800 + ((cp - 0x10000) >> 10));
            put_unit(b, 0xDC00 + ((cp - 0x10000) & 0x3FF));
        } else {
            put_unit(b, cp);
        }
        i += need + 1;
    }
    puts_(b, "\"");
    return 0;
}

static void put_i64(sbuf* b, int64_t v) {
    char t[24];
    int k = 24;
    uint64_t u = v < 0 ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
    do {
        t[--k] = (char)('0' + u % 10);
        u /= 10;
    } while (u);
    if (v < 0) t[--k] = '-';
    put(b, t + k, 24 - k);
}

static void put_aid(sbuf* b, uint64_t hi, uint64_t lo) {
    char t[34];
    t[0] = '"';
    for (int k = 0; k < 16; ++k) t[1 + k] = HEX[(hi >> (60 - 4 * k)) & 15];
    for (int k = 0; k < 16; ++k) t[17 + k] = HEX[(lo >> (60 - 4 * k)) & 15];
    t[33] = '"';
    put(b, t, 34);
}

typedef struct {
    int32_t n;
    const int32_t* invoker;   /* chosen invoker id, < 0: no message (publish failed) */
    const int32_t* tmpl;      /* template of each activation */
    const char* ta;           /* template part A bytes, offsets ta_off[t..t+1] */
    const int64_t* ta_off;
    const char* tb;           /* template part B (initArgs value) */
    const int64_t* tb_off;
    int32_t n_templates;
    const char* rci;          /* rootControllerIndex JSON value */
    int32_t rci_len;
    const uint64_t* aid;      /* 2 per activation: hi, lo */
    const char* tid;          /* transaction id strings (UTF-8), offsets tid_off */
    const int64_t* tid_off;
    const int64_t* tid_start; /* epoch ms */
    const uint8_t* flags;     /* OWM_* */
    const char* content;      /* printed JsObject, offsets content_off */
    const int64_t* content_off;
    const uint64_t* cause;    /* 2 per activation (when OWM_HAS_CAUSE) */
    const char* trace;        /* printed traceContext map, offsets trace_off */
    const int64_t* trace_off;
    int32_t n_topics;         /* invoker ids must be < n_topics */
} owm_batch;

/* one message into b; -1 on malformed UTF-8 in the transaction id */
static int message(sbuf* b, const owm_batch* B, int32_t i) {
    const int32_t t = B->tmpl[i];
    const uint8_t f = B->flags[i];
    puts_(b, "{\"transid\":[");
    if (put_string(b, (const uint8_t*)B->tid + B->tid_off[i], B->tid_off[i + 1] - B->tid_off[i])) return -1;
    puts_(b, ",");
    put_i64(b, B->tid_start[i]);
    if (f & OWM_EXTRA_LOGGING) puts_(b, ",true");
    puts_(b, "],");
    put(b, B->ta + B->ta_off[t], B->ta_off[t + 1] - B->ta_off[t]);
    puts_(b, ",\"activationId\":");
    put_aid(b, B->aid[2 * i], B->aid[2 * i + 1]);
    puts_(b, ",\"rootControllerIndex\":");
    put(b, B->rci, B->rci_len);
    puts_(b, (f & OWM_BLOCKING) ? ",\"blocking\":true" : ",\"blocking\":false");
    if (f & OWM_HAS_CONTENT) {
        puts_(b, ",\"content\":");
        put(b, B->content + B->content_off[i], B->content_off[i + 1] - B->content_off[i]);
    }
    puts_(b, ",\"initArgs\":");
    put(b, B->tb + B->tb_off[t], B->tb_off[t + 1] - B->tb_off[t]);
    if (f & OWM_HAS_CAUSE) {
        puts_(b, ",\"cause\":");
        put_aid(b, B->cause[2 * i], B->cause[2 * i + 1]);
    }
    if (f & OWM_HAS_TRACE) {
        puts_(b, ",\"traceContext\":");
        put(b, B->trace + B->trace_off[i], B->trace_off[i + 1] - B->trace_off[i]);
    }
    puts_(b, "}");
    return 0;
}

/* Serialise and fan out.  out_off[m+1] byte offsets of the m messages in output order, out_order[m] their
 * activation index, topic_start[n_topics+1] the message range of each invoker topic.  Returns m, -1 on a bad
 * argument (template or invoker out of range, malformed transaction id), -2 when cap is too small (*total = bytes
 * needed). */
int64_t owm_serialize(const owm_batch* B, char* out, int64_t cap, int64_t* out_off, int32_t* out_order,
                      int32_t* topic_start, int64_t* total) {
    for (int32_t i = 0; i < B->n; ++i)
        if (B->invoker[i] >= B->n_topics || (B->invoker[i] >= 0 && (B->tmpl[i] < 0 || B->tmpl[i] >= B->n_templates)))
            return -1;
    /* counting sort by topic, stable */
    for (int32_t k = 0; k <= B->n_topics; ++k) topic_start[k] = 0;
    for (int32_t i = 0; i < B->n; ++i)
        if (B->invoker[i] >= 0) topic_start[B->invoker[i] + 1]++;
    for (int32_t k = 0; k < B->n_topics; ++k) topic_start[k + 1] += topic_start[k];
    const int32_t m = topic_start[B->n_topics];
    for (int32_t k = B->n_topics; k > 0; --k) topic_start[k] = topic_start[k - 1];
    topic_start[0] = 0;
    for (int32_t i = 0; i < B->n; ++i)
        if (B->invoker[i] >= 0) out_order[topic_start[B->invoker[i] + 1]++] = i;
    /* topic_start[k + 1] is now the end of topic k = the start of topic k + 1 */
    sbuf b = {out, 0, cap, 0};
    out_off[0] = 0;
    for (int32_t j = 0; j < m; ++j) {
        if (message(&b, B, out_order[j])) return -1;
        out_off[j + 1] = b.n;
    }
    *total = b.n;
    return b.overflow ? -2 : m;
}
