/*
 * owsched_oracle.c -- CPU ORACLE (test infrastructure; see owsched_oracle.h for scope and citations).
 *
 * Literal sequential restatement of the reference path.  Every function names the reference lines it follows.
 * Integer arithmetic reproduces Java int semantics (32-bit two's complement wrap, truncating '/' and '%').
 */
#include "owsched_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------------ */
/* Java int helpers                                                                                  */
/* ------------------------------------------------------------------------------------------------ */
static inline int32_t jadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static inline int32_t jsub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
static inline int32_t jmul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }

/* Scala Double.toInt: NaN -> 0, saturating at Int bounds */
static int32_t d2i(double d) {
    if (d != d) return 0;
    if (d >= 2147483647.0) return 2147483647;
    if (d <= -2147483648.0) return (-2147483647 - 1);
    return (int32_t)d;
}

/* java.lang.String.hashCode (JLS): h = 31*h + c over UTF-16 code units.  EntityName's regex
 * (common/.../core/entity/EntityPath.scala:199-208) restricts names to ASCII, so bytes == code units. */
int32_t owo_java_hash(const char* s, int32_t len) {
    int32_t h = 0;
    for (int32_t i = 0; i < len; ++i) h = jadd(jmul(31, h), (int32_t)(uint8_t)s[i]);
    return h;
}

/* SCPB:370-372  (namespace.asString.hashCode() ^ action.asString.hashCode()).abs ; Int.MinValue.abs == MinValue */
int32_t owo_generate_hash(const char* ns, int32_t ns_len, const char* path, int32_t path_len) {
    int32_t x = owo_java_hash(ns, ns_len) ^ owo_java_hash(path, path_len);
    return x < 0 ? jsub(0, x) : x;
}

/* SCPB:375-376 */
int32_t owo_gcd(int32_t a, int32_t b) {
    while (b != 0) {
        int32_t t = (b == -1) ? 0 : a % b; /* Java: MIN_VALUE % -1 == 0 */
        a = b;
        b = t;
    }
    return a;
}

/* SCPB:379-384  (1 to x).foldLeft: keep cur iff gcd(cur,x)==1 && coprime to every kept number */
int32_t owo_pairwise_coprime(int32_t x, int32_t* out, int32_t cap) {
    int32_t n = 0;
    for (int32_t cur = 1; cur <= x && cur > 0; ++cur) {
        if (owo_gcd(cur, x) != 1) continue;
        int ok = 1;
        for (int32_t i = 0; i < n && ok; ++i)
            if (owo_gcd(out ? out[i] : 0, cur) != 1) ok = 0;
        if (ok) {
            if (n >= cap) return -1;
            out[n++] = cur;
        }
    }
    return n;
}

/* Bench-defined counter RNG replacing ThreadLocalRandom.current().nextInt(|H|) (SCPB:421); SURVEY A.7. */
static inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
uint32_t owo_rng_index(uint64_t seed, uint64_t seq, uint32_t n) {
    uint64_t u = splitmix64(seed ^ (seq * 0x9E3779B97F4A7C15ULL)) >> 32;
    return (uint32_t)((u * (uint64_t)n) >> 32);
}

/* ------------------------------------------------------------------------------------------------ */
/* ResizableSemaphore  RS:33-115                                                                     */
/* ------------------------------------------------------------------------------------------------ */
void owo_rs_init(owo_rs* s, int32_t max_allowed, int32_t reduction_size) {
    s->c = max_allowed;
    s->ops = 0;
    s->R = reduction_size;
}

/* RS:82-90 -> nonFairTryAcquireShared RS:62-70 */
int owo_rs_try_acquire(owo_rs* s, int32_t acquires) {
    if (acquires <= 0) return OWO_THROW_ARG; /* require RS:83 */
    int32_t remaining = jsub(s->c, acquires);
    if (remaining < 0) return 0;
    s->c = remaining;
    s->ops = jadd(s->ops, 1);
    return 1;
}

/* RS:99-108 -> tryReleaseSharedWithResult RS:42-56.  returns bit0 = memory release, bit1 = action release */
int owo_rs_release(owo_rs* s, int32_t acquires, int op_complete) {
    if (acquires <= 0) return OWO_THROW_ARG; /* require RS:100 */
    int action_rel;
    if (op_complete) {
        s->ops = jsub(s->ops, 1);
        action_rel = (s->ops == 0);
    } else {
        s->ops = jadd(s->ops, 1);
        action_rel = (s->ops == 0);
    }
    int32_t next2 = jadd(s->c, acquires);
    int mem_rel = 0;
    if (s->R == 0) return OWO_THROW_ARG; /* ArithmeticException (/ by zero); unreachable for maxConcurrent >= 2 */
    if (next2 % s->R == 0) {
        s->c = jsub(next2, s->R);
        mem_rel = 1;
    } else {
        s->c = next2;
    }
    return mem_rel | (action_rel << 1);
}

/* ------------------------------------------------------------------------------------------------ */
/* NestedSemaphore  NS:29-116  (ForcibleSemaphore FS:37-124 for the memory permits)                  */
/* ------------------------------------------------------------------------------------------------ */
typedef struct {
    uint32_t key;
    uint8_t used; /* 0 empty, 1 live, 2 tombstone */
    owo_rs rs;
} owo_cslot;

struct owo_ns {
    int32_t permits;   /* FS Sync state */
    int zombies;       /* 1: getOrElseUpdate creates entries on failed tries too (literal NS:61-62) */
    int32_t cap, live, filled;
    owo_cslot* tab;    /* TrieMap[T, ResizableSemaphore] */
};

owo_ns* owo_ns_new(int32_t memory_permits, int zombies) {
    owo_ns* s = (owo_ns*)calloc(1, sizeof(owo_ns));
    s->permits = memory_permits;
    s->zombies = zombies;
    return s;
}
void owo_ns_free(owo_ns* s) {
    if (!s) return;
    free(s->tab);
    free(s);
}

static inline uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

static owo_cslot* cmap_find(const owo_ns* s, uint32_t key) {
    if (!s->tab) return NULL;
    uint32_t m = (uint32_t)s->cap - 1, i = mix32(key) & m;
    for (;;) {
        owo_cslot* e = &s->tab[i];
        if (e->used == 0) return NULL;
        if (e->used == 1 && e->key == key) return e;
        i = (i + 1) & m;
    }
}

static void cmap_grow(owo_ns* s) {
    int32_t ncap = s->cap ? s->cap * 2 : 8;
    while (s->live * 2 >= ncap) ncap *= 2;
    owo_cslot* old = s->tab;
    int32_t ocap = s->cap;
    s->tab = (owo_cslot*)calloc((size_t)ncap, sizeof(owo_cslot));
    s->cap = ncap;
    s->filled = 0;
    for (int32_t j = 0; j < ocap; ++j) {
        if (old[j].used != 1) continue;
        uint32_t m = (uint32_t)ncap - 1, i = mix32(old[j].key) & m;
        while (s->tab[i].used) i = (i + 1) & m;
        s->tab[i] = old[j];
        s->filled++;
    }
    free(old);
}

static owo_cslot* cmap_insert(owo_ns* s, uint32_t key, int32_t R) {
    if ((s->filled + 1) * 2 > s->cap) cmap_grow(s);
    uint32_t m = (uint32_t)s->cap - 1, i = mix32(key) & m;
    while (s->tab[i].used == 1) i = (i + 1) & m;
    if (s->tab[i].used == 0) s->filled++;
    owo_cslot* e = &s->tab[i];
    e->used = 1;
    e->key = key;
    owo_rs_init(&e->rs, 0, R); /* new ResizableSemaphore(0, maxConcurrent)  NS:62 */
    s->live++;
    return e;
}

static void cmap_remove(owo_ns* s, owo_cslot* e) {
    e->used = 2;
    s->live--;
}

/* FS:95-98 / FS:63-71 */
int owo_ns_try_acquire(owo_ns* s, int32_t acquires) {
    if (acquires <= 0) return OWO_THROW_ARG;
    int32_t remaining = jsub(s->permits, acquires);
    if (remaining < 0) return 0;
    s->permits = remaining;
    return 1;
}
/* FS:107-110 / FS:78-84 */
int owo_ns_force_acquire(owo_ns* s, int32_t acquires) {
    if (acquires <= 0) return OWO_THROW_ARG;
    s->permits = jsub(s->permits, acquires);
    return 0;
}
/* FS:117-120 / FS:45-56 (overflow -> Error, state unchanged) */
int owo_ns_release(owo_ns* s, int32_t acquires) {
    if (acquires <= 0) return OWO_THROW_ARG;
    int32_t next = jadd(s->permits, acquires);
    if (next < s->permits) return OWO_THROW_OVERFLOW;
    s->permits = next;
    return 0;
}
int32_t owo_ns_available(const owo_ns* s) { return s->permits; }

/* NS:57-82 tryOrForceAcquireConcurrent (sequential: the synchronized re-check is a no-op) */
static int ns_try_or_force(owo_ns* s, uint32_t key, int32_t max_conc, int32_t mem, int force) {
    owo_cslot* e = cmap_find(s, key);
    owo_rs tmp;
    owo_rs* rs;
    if (e) {
        rs = &e->rs;
    } else if (s->zombies) {
        e = cmap_insert(s, key, max_conc); /* getOrElseUpdate NS:61-62 */
        rs = &e->rs;
    } else {
        owo_rs_init(&tmp, 0, max_conc);
        rs = &tmp;
    }
    int r = owo_rs_try_acquire(rs, 1); /* NS:63 */
    if (r < 0) return r;
    int ok = r;
    if (!ok) {
        if (force) { /* NS:70-73 */
            owo_ns_force_acquire(s, mem);
            int rr = owo_rs_release(rs, max_conc - 1, 0);
            if (rr < 0) return rr;
            ok = 1;
        } else { /* NS:74-79 */
            int t = owo_ns_try_acquire(s, mem);
            if (t < 0) return t;
            if (t) {
                int rr = owo_rs_release(rs, max_conc - 1, 0);
                if (rr < 0) return rr;
                ok = 1;
            }
        }
    }
    if (ok && rs == &tmp) { /* materialise the entry only once it holds state (non-zombie mode) */
        owo_cslot* ne = cmap_insert(s, key, max_conc);
        ne->rs = tmp;
    }
    return ok;
}

/* NS:32-39 */
int owo_ns_try_acquire_concurrent(owo_ns* s, uint32_t key, int32_t max_conc, int32_t mem) {
    if (max_conc == 1) return owo_ns_try_acquire(s, mem);
    return ns_try_or_force(s, key, max_conc, mem, 0);
}
/* NS:84-91 */
int owo_ns_force_acquire_concurrent(owo_ns* s, uint32_t key, int32_t max_conc, int32_t mem) {
    if (mem <= 0) return OWO_THROW_ARG;
    if (max_conc == 1) return owo_ns_force_acquire(s, mem);
    int r = ns_try_or_force(s, key, max_conc, mem, 1);
    return r < 0 ? r : 0;
}
/* NS:98-113 */
int owo_ns_release_concurrent(owo_ns* s, uint32_t key, int32_t max_conc, int32_t mem) {
    if (mem <= 0) return OWO_THROW_ARG;
    if (max_conc == 1) return owo_ns_release(s, mem);
    owo_cslot* e = cmap_find(s, key);
    if (!e) return OWO_THROW_NOSUCHELEMENT; /* actionConcurrentSlotsMap(actionid) NS:103 */
    int r = owo_rs_release(&e->rs, 1, 1);
    if (r < 0) return r;
    if (r & 1) {
        int f = owo_ns_release(s, mem);
        if (f < 0) return f; /* Error thrown after the RS update; map removal skipped (literal) */
    }
    if (r & 2) cmap_remove(s, e);
    return 0;
}

int owo_ns_concurrent_state(const owo_ns* s, uint32_t key, int32_t* c, int32_t* ops) {
    owo_cslot* e = cmap_find(s, key);
    if (!e) return 0;
    if (c) *c = e->rs.c;
    if (ops) *ops = e->rs.ops;
    return 1;
}
int32_t owo_ns_concurrent_size(const owo_ns* s) { return s->live; }

/* ------------------------------------------------------------------------------------------------ */
/* IndexedSeq[NestedSemaphore]                                                                      */
/* ------------------------------------------------------------------------------------------------ */
struct owo_slots {
    int32_t n, cap;
    owo_ns** v;
};

owo_slots* owo_slots_new(int32_t count, int32_t permits, int zombies) {
    owo_slots* v = (owo_slots*)calloc(1, sizeof(owo_slots));
    v->cap = count > 4 ? count : 4;
    v->v = (owo_ns**)calloc((size_t)v->cap, sizeof(owo_ns*));
    for (int32_t i = 0; i < count; ++i) v->v[i] = owo_ns_new(permits, zombies);
    v->n = count;
    return v;
}
static void slots_clear(owo_slots* v) {
    for (int32_t i = 0; i < v->n; ++i) owo_ns_free(v->v[i]);
    v->n = 0;
}
static void slots_push(owo_slots* v, owo_ns* s) {
    if (v->n == v->cap) {
        v->cap *= 2;
        v->v = (owo_ns**)realloc(v->v, (size_t)v->cap * sizeof(owo_ns*));
    }
    v->v[v->n++] = s;
}
void owo_slots_free(owo_slots* v) {
    if (!v) return;
    slots_clear(v);
    free(v->v);
    free(v);
}
int32_t owo_slots_count(const owo_slots* v) { return v->n; }
owo_ns* owo_slots_get(owo_slots* v, int32_t i) { return (i >= 0 && i < v->n) ? v->v[i] : NULL; }

/* ------------------------------------------------------------------------------------------------ */
/* SCPB.schedule  SCPB:398-436 (tail recursion unrolled into a loop; n+2 probes before the fallback)  */
/* ------------------------------------------------------------------------------------------------ */
int owo_schedule(owo_slots* dispatched, int32_t max_conc, uint32_t key, int32_t n, const int32_t* ids,
                 const uint8_t* status, int32_t slots, int32_t index, int32_t step, uint64_t rng_seed, uint64_t seq,
                 int32_t* out_id, uint8_t* out_flags) {
    *out_flags = 0;
    if (n <= 0) { /* SCPB:433-435 */
        *out_id = OWO_NONE;
        return 0;
    }
    for (int32_t steps_done = 0;; ++steps_done) {
        if (index < 0 || index >= n) { /* invokers(index): IndexOutOfBoundsException */
            *out_id = OWO_THROW_INDEX;
            return OWO_THROW_INDEX;
        }
        int32_t id = ids[index];
        if (status[index] == OWO_HEALTHY) { /* short-circuit && SCPB:413 */
            if (id < 0 || id >= dispatched->n) {
                *out_id = OWO_THROW_INDEX;
                return OWO_THROW_INDEX;
            }
            int r = owo_ns_try_acquire_concurrent(dispatched->v[id], key, max_conc, slots);
            if (r < 0) {
                *out_id = r;
                return r;
            }
            if (r) {
                *out_id = id; /* Some(invoker.id, false) SCPB:414 */
                return 1;
            }
        }
        if (steps_done == n + 1) { /* SCPB:417-427 */
            int32_t healthy = 0;
            for (int32_t i = 0; i < n; ++i) healthy += (status[i] == OWO_HEALTHY);
            if (healthy == 0) {
                *out_id = OWO_NONE;
                return 0;
            }
            uint32_t k = owo_rng_index(rng_seed, seq, (uint32_t)healthy);
            int32_t rid = -1;
            for (int32_t i = 0; i < n; ++i)
                if (status[i] == OWO_HEALTHY && k-- == 0) {
                    rid = ids[i];
                    break;
                }
            if (rid < 0 || rid >= dispatched->n) {
                *out_id = OWO_THROW_INDEX;
                return OWO_THROW_INDEX;
            }
            int r = owo_ns_force_acquire_concurrent(dispatched->v[rid], key, max_conc, slots);
            if (r < 0) {
                *out_id = r;
                return r;
            }
            *out_id = rid;
            *out_flags = 1;
            return 1;
        }
        index = jadd(index, step) % n; /* SCPB:429 */
    }
}

/* ------------------------------------------------------------------------------------------------ */
/* ShardingContainerPoolBalancerState  SCPB:449-585                                                  */
/* ------------------------------------------------------------------------------------------------ */
typedef struct {
    int32_t hash;
    uint32_t key;
    int32_t mem_mb;
    int32_t max_conc;
    int32_t blackbox;
} owo_action;

struct owo_state {
    double managed_fraction, blackbox_fraction;
    int64_t min_memory_bytes;
    uint64_t rng_seed;
    int zombies;
    int32_t n_inv;
    int32_t* ids;
    int64_t* mem;
    uint8_t* status;
    int32_t managed, blackboxes; /* configured counts (SCPB:518-519) */
    int32_t n_msteps, n_bsteps;
    int32_t *msteps, *bsteps;
    owo_slots* slots;
    int32_t cluster_size;
    int32_t n_actions, cap_actions;
    owo_action* actions;
};

owo_state* owo_state_new(double mf, double bf, int64_t min_memory_bytes, uint64_t rng_seed, int zombies) {
    owo_state* st = (owo_state*)calloc(1, sizeof(owo_state));
    /* SCPB:467-468 */
    st->managed_fraction = fmax(0.0, fmin(1.0, mf));
    st->blackbox_fraction = fmax(1.0 - st->managed_fraction, fmin(1.0, bf));
    st->min_memory_bytes = min_memory_bytes;
    st->rng_seed = rng_seed;
    st->zombies = zombies;
    st->slots = owo_slots_new(0, 0, zombies);
    st->cluster_size = 1;
    return st;
}

void owo_state_free(owo_state* st) {
    if (!st) return;
    free(st->ids);
    free(st->mem);
    free(st->status);
    free(st->msteps);
    free(st->bsteps);
    owo_slots_free(st->slots);
    free(st->actions);
    free(st);
}

/* SCPB:485-499 getInvokerSlot(memory).toMB.toInt */
static int32_t invoker_slot_mb(const owo_state* st, int64_t mem_bytes) {
    int64_t shard = mem_bytes / st->cluster_size;
    if (shard < st->min_memory_bytes) shard = st->min_memory_bytes;
    return (int32_t)(shard / 1024 / 1024);
}

static int32_t* coprime_list(int32_t x, int32_t* count) {
    int32_t cap = x > 0 ? x : 1;
    int32_t* out = (int32_t*)malloc((size_t)cap * sizeof(int32_t));
    *count = owo_pairwise_coprime(x, out, cap);
    return out;
}

/* SCPB:512-551 */
int owo_update_invokers(owo_state* st, int32_t n, const int32_t* ids, const int64_t* mem, const uint8_t* status) {
    int32_t old_size = st->n_inv;
    int32_t new_size = n;
    int32_t managed = d2i(ceil((double)new_size * st->managed_fraction));
    if (managed < 1) managed = 1;
    int32_t blackboxes = d2i(floor((double)new_size * st->blackbox_fraction));
    if (blackboxes < 1) blackboxes = 1;

    free(st->ids);
    free(st->mem);
    free(st->status);
    st->ids = (int32_t*)malloc((size_t)(n > 0 ? n : 1) * sizeof(int32_t));
    st->mem = (int64_t*)malloc((size_t)(n > 0 ? n : 1) * sizeof(int64_t));
    st->status = (uint8_t*)malloc((size_t)(n > 0 ? n : 1));
    if (n > 0) {
        memcpy(st->ids, ids, (size_t)n * sizeof(int32_t));
        memcpy(st->mem, mem, (size_t)n * sizeof(int64_t));
        memcpy(st->status, status, (size_t)n);
    }
    st->n_inv = n;
    st->managed = managed;
    st->blackboxes = blackboxes;

    if (old_size != new_size) {
        free(st->msteps);
        free(st->bsteps);
        st->msteps = coprime_list(managed, &st->n_msteps);
        st->bsteps = coprime_list(blackboxes, &st->n_bsteps);
        if (old_size < new_size) { /* keep existing state; append only new invokers SCPB:529-534 */
            for (int32_t i = st->slots->n; i < n; ++i)
                slots_push(st->slots, owo_ns_new(invoker_slot_mb(st, st->mem[i]), st->zombies));
        }
    }
    return 0;
}

/* SCPB:561-584 */
int owo_update_cluster(owo_state* st, int32_t new_size) {
    int32_t actual = new_size > 1 ? new_size : 1;
    if (st->cluster_size != actual) {
        st->cluster_size = actual;
        slots_clear(st->slots);
        for (int32_t i = 0; i < st->n_inv; ++i)
            slots_push(st->slots, owo_ns_new(invoker_slot_mb(st, st->mem[i]), st->zombies));
    }
    return 0;
}

int32_t owo_cluster_size(const owo_state* st) { return st->cluster_size; }
int32_t owo_n_invokers(const owo_state* st) { return st->n_inv; }
int32_t owo_managed_size(const owo_state* st) { return st->managed < st->n_inv ? st->managed : st->n_inv; }
int32_t owo_blackbox_size(const owo_state* st) { return st->blackboxes < st->n_inv ? st->blackboxes : st->n_inv; }
static int32_t copy_out(const int32_t* src, int32_t n, int32_t* out, int32_t cap) {
    for (int32_t i = 0; i < n && i < cap; ++i) out[i] = src[i];
    return n;
}
int32_t owo_managed_steps(const owo_state* st, int32_t* out, int32_t cap) {
    return copy_out(st->msteps, st->n_msteps, out, cap);
}
int32_t owo_blackbox_steps(const owo_state* st, int32_t* out, int32_t cap) {
    return copy_out(st->bsteps, st->n_bsteps, out, cap);
}
owo_slots* owo_state_slots(owo_state* st) { return st->slots; }
int32_t owo_read_permits(const owo_state* st, int32_t* out, int32_t cap) {
    for (int32_t i = 0; i < st->slots->n && i < cap; ++i) out[i] = st->slots->v[i]->permits;
    return st->slots->n;
}

int32_t owo_register_action(owo_state* st, const char* ns, int32_t ns_len, const char* path, int32_t path_len,
                            uint32_t key, int32_t mem_mb, int32_t max_conc, int32_t blackbox) {
    if (st->n_actions == st->cap_actions) {
        st->cap_actions = st->cap_actions ? st->cap_actions * 2 : 64;
        st->actions = (owo_action*)realloc(st->actions, (size_t)st->cap_actions * sizeof(owo_action));
    }
    owo_action* a = &st->actions[st->n_actions];
    a->hash = owo_generate_hash(ns, ns_len, path, path_len);
    a->key = key;
    a->mem_mb = mem_mb;
    a->max_conc = max_conc;
    a->blackbox = blackbox;
    return st->n_actions++;
}

int32_t owo_action_hash(const owo_state* st, int32_t action) { return st->actions[action].hash; }

/* SCPB:260-290: pool selection, generateHash, home = hash % n, step = stepSizes(hash % k), schedule */
int owo_publish(owo_state* st, int32_t action, uint64_t seq, int32_t* out_invoker, uint8_t* out_flags) {
    const owo_action* a = &st->actions[action];
    *out_flags = 0;
    int32_t base, n, nsteps;
    const int32_t* steps;
    if (!a->blackbox) {
        n = owo_managed_size(st);
        base = 0;
        steps = st->msteps;
        nsteps = st->n_msteps;
    } else {
        n = owo_blackbox_size(st);
        base = st->n_inv - n;
        steps = st->bsteps;
        nsteps = st->n_bsteps;
    }
    if (n <= 0) { /* invokersToUse.nonEmpty false SCPB:265, 288-290 */
        *out_invoker = OWO_NONE;
        return 0;
    }
    int32_t home = a->hash % n;
    int32_t sidx = a->hash % nsteps;
    if (sidx < 0) { /* stepSizes(negative) */
        *out_invoker = OWO_THROW_INDEX;
        return OWO_THROW_INDEX;
    }
    return owo_schedule(st->slots, a->max_conc, a->key, n, st->ids + base, st->status + base, a->mem_mb, home,
                        steps[sidx], st->rng_seed, seq, out_invoker, out_flags);
}

/* SCPB:327-331 releaseInvoker: invokerSlots.lift(invoker).foreach(_.releaseConcurrent(...)) */
int owo_release(owo_state* st, int32_t invoker, int32_t action) {
    if (invoker < 0 || invoker >= st->slots->n) return 0;
    const owo_action* a = &st->actions[action];
    return owo_ns_release_concurrent(st->slots->v[invoker], a->key, a->max_conc, a->mem_mb);
}

int owo_replay(owo_state* st, int32_t n_batches, const int64_t* acq_off, const int32_t* act, const int64_t* rel_off,
               const int64_t* rel_aid, uint64_t seq_base, int32_t* out_invoker, uint8_t* out_flags,
               uint8_t* rel_flags) {
    for (int32_t b = 0; b < n_batches; ++b) {
        for (int64_t r = rel_off[b]; r < rel_off[b + 1]; ++r) {
            int64_t aid = rel_aid[r];
            int32_t inv = out_invoker[aid];
            uint8_t f = 0;
            if (inv < 0) {
                f = 4; /* CLB:278-279: no ActivationEntry -> nothing to release */
            } else {
                int rc = owo_release(st, inv, act[aid]);
                if (rc == OWO_THROW_NOSUCHELEMENT) f = 1;
                else if (rc == OWO_THROW_OVERFLOW) f = 2;
                else if (rc < 0) f = 8;
            }
            if (rel_flags) rel_flags[r] = f;
        }
        for (int64_t i = acq_off[b]; i < acq_off[b + 1]; ++i)
            owo_publish(st, act[i], seq_base + (uint64_t)i, &out_invoker[i], &out_flags[i]);
    }
    return 0;
}

typedef struct {
    owo_state* st;
    int32_t n_batches;
    const int64_t *acq_off, *rel_off, *rel_aid;
    const int32_t* act;
    uint64_t seq_base;
    int32_t* out_invoker;
    uint8_t *out_flags, *rel_flags;
} replay_job;

static void* replay_thread(void* p) {
    replay_job* j = (replay_job*)p;
    owo_replay(j->st, j->n_batches, j->acq_off, j->act, j->rel_off, j->rel_aid, j->seq_base, j->out_invoker,
               j->out_flags, j->rel_flags);
    return NULL;
}

int owo_replay_parallel(owo_state** states, int32_t nthreads, int32_t n_batches, const int64_t* acq_off,
                        const int32_t* const* acts, const int64_t* rel_off, const int64_t* rel_aid, uint64_t seq_base,
                        int32_t* const* out_invoker, uint8_t* const* out_flags, uint8_t* const* rel_flags) {
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    replay_job* jobs = (replay_job*)calloc((size_t)nthreads, sizeof(replay_job));
    for (int32_t t = 0; t < nthreads; ++t) {
        replay_job j = {states[t], n_batches, acq_off, rel_off, rel_aid, acts[t], seq_base,
                        out_invoker[t], out_flags[t], rel_flags ? rel_flags[t] : NULL};
        jobs[t] = j;
        pthread_create(&th[t], NULL, replay_thread, &jobs[t]);
    }
    for (int32_t t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
    return 0;
}
