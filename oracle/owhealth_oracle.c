/*
 * owhealth_oracle.c -- TEST INFRASTRUCTURE (CPU oracle): restatement of the invoker health supervision for the parity
 * tests.  Only tests/ and __graft_entry__.smoke() load it; the product path never does.
 *
 * Follows, in the reference repository (ISUP = core/controller/src/main/scala/org/apache/openwhisk/core/loadBalancer/
 * InvokerSupervision.scala):
 *   InvokerPool.receive (PingMessage, InvocationFinishedMessage, CurrentState, Transition)   ISUP:119-150
 *   InvokerPool.registerInvoker / padToIndexed                                               ISUP:180-199
 *   InvokerActor states, stateTimeout = 10 s, Tick                                           ISUP:285-331
 *   whenUnhandled -> handleCompletionMessage (ring buffer of 10, tolerance 3)                ISUP:334-336, 383-410
 *   onTransition handlers (test action + 1-minute repeating Tick while Unhealthy/Unresponsive,
 *   registered in the order: log, Unhealthy handler, Unresponsive handler)                   ISUP:339-365
 *   RingBuffer = commons CircularFifoBuffer(10)                                              common/.../RingBuffer.scala
 * and the akka 2.5 FSM timer rules (an un-vendored dependency, restated): every message the FSM processes -- timer
 * messages (Tick) included, StateTimeout excluded -- cancels the pending state timeout, and the state reached
 * (stay() included) re-arms it from that moment when that state has one (Unhealthy, Unresponsive, Healthy: 10 s;
 * Offline: none); initialize() runs the transition handlers for the start state (Unhealthy) once.
 *
 * Written event by event over the global mailbox order with a per-invoker record (the GPU groups events by invoker).
 *
 * Time model (the bench's and the tests' contract, shared with the GPU path): every event carries a time in ms, the
 * sequence is non-decreasing, and the batch ends at `now_ms`.  Before an event at time t (and at the end, t = now),
 * each invoker's due timers fire in deadline order: the state timeout at last + 10000 and the Tick at its period
 * boundary; a timer is due when its deadline <= t; equal deadlines fire the state timeout first.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OWH_HEALTHY 0
#define OWH_UNHEALTHY 1
#define OWH_UNRESPONSIVE 2
#define OWH_OFFLINE 3
#define OWH_PADDED 254 /* a status entry without an actor (padToIndexed, ISUP:188-191): Offline */
#define OWH_ABSENT 255

#define OWH_EV_PING 0
#define OWH_EV_SUCCESS 1
#define OWH_EV_SYSTEM_ERROR 2
#define OWH_EV_TIMEOUT 3
#define OWH_EV_STATE_TIMEOUT 4

#define OWH_STATE_TIMEOUT_MS 10000 /* healthyTimeout, ISUP:298 */
#define OWH_TICK_MS 60000          /* setTimer(..., 1.minute, repeat = true), ISUP:360 */
#define OWH_BUFFER 10              /* InvokerActor.bufferSize, ISUP:437 */
#define OWH_TOLERANCE 3            /* bufferErrorTolerance, ISUP:438 */
#define OWH_NEVER INT64_MAX

typedef struct {
    uint8_t st;
    uint8_t nbuf;        /* entries in the ring buffer (<= 10) */
    uint8_t buf[OWH_BUFFER]; /* results, oldest first (CircularFifoBuffer.toArray order) */
    int64_t last;        /* when the state timeout was last armed (OWH_NEVER: none pending) */
    int64_t tick;        /* next Tick, OWH_NEVER when the timer is cancelled */
    int64_t mem;         /* userMemory (bytes) of the instance in the status vector */
    int32_t tests;       /* invokeTestAction calls during the current batch */
} owh_inv;

typedef struct {
    int32_t size, cap;   /* status.size (ISUP:117) */
    int64_t now;         /* end of the previous batch: event times never go back before it */
    owh_inv* v;
} owh_pool;

owh_pool* owh_new(int64_t start_ms) {
    owh_pool* p = (owh_pool*)calloc(1, sizeof(owh_pool));
    if (p) p->now = start_ms;
    return p;
}
void owh_free(owh_pool* p) {
    if (p) free(p->v);
    free(p);
}

static int has_timeout(int st) { return st == OWH_HEALTHY || st == OWH_UNHEALTHY || st == OWH_UNRESPONSIVE; }

static void arm(owh_inv* a, int64_t t) { a->last = has_timeout(a->st) ? t : OWH_NEVER; }

/* goto(to) from a->st at time t: onTransition handlers in registration order (ISUP:339-365), then the new state's
 * timeout is armed by the caller. */
static void transition(owh_inv* a, int to, int64_t t) {
    const int from = a->st;
    /* healthPingingTransitionHandler(Unhealthy): case _ -> Unhealthy => test + setTimer; case Unhealthy -> _ => cancel */
    if (to == OWH_UNHEALTHY) {
        a->tests++;
        a->tick = t + OWH_TICK_MS;
    } else if (from == OWH_UNHEALTHY) {
        a->tick = OWH_NEVER;
    }
    /* healthPingingTransitionHandler(Unresponsive) */
    if (to == OWH_UNRESPONSIVE) {
        a->tests++;
        a->tick = t + OWH_TICK_MS;
    } else if (from == OWH_UNRESPONSIVE) {
        a->tick = OWH_NEVER;
    }
    a->st = (uint8_t)to;
}

static void go(owh_inv* a, int to, int64_t t) {
    if (to != a->st) transition(a, to, t);
    arm(a, t);
}

/* fire every timer of a due at or before t */
static void fire_due(owh_inv* a, int64_t t) {
    for (;;) {
        const int64_t ds = (a->last == OWH_NEVER) ? OWH_NEVER : a->last + OWH_STATE_TIMEOUT_MS;
        const int64_t dt = a->tick;
        if (ds <= t && ds <= dt) {          /* StateTimeout: goto(Offline) from every state that has one */
            a->last = OWH_NEVER;
            go(a, OWH_OFFLINE, ds);
        } else if (dt <= t) {               /* Tick (pinging states only): invokeTestAction(); stay */
            a->tests++;
            a->tick = dt + OWH_TICK_MS;
            arm(a, dt);
        } else {
            return;
        }
    }
}

static int grow(owh_pool* p, int32_t n) {
    if (n <= p->cap) return 0;
    int32_t c = p->cap ? p->cap : 64;
    while (c < n) c *= 2;
    owh_inv* v = (owh_inv*)realloc(p->v, (size_t)c * sizeof(owh_inv));
    if (!v) return -1;
    for (int32_t i = p->cap; i < c; ++i) {
        memset(&v[i], 0, sizeof(owh_inv));
        v[i].st = OWH_ABSENT;
        v[i].last = OWH_NEVER;
        v[i].tick = OWH_NEVER;
    }
    p->v = v;
    p->cap = c;
    return 0;
}

static void completion(owh_inv* a, int result, int64_t t) {
    /* buffer.add(result) -- CircularFifoBuffer drops the oldest when full */
    if (a->nbuf == OWH_BUFFER) {
        memmove(a->buf, a->buf + 1, OWH_BUFFER - 1);
        a->nbuf--;
    }
    a->buf[a->nbuf++] = (uint8_t)result;
    if (result == OWH_EV_SUCCESS && a->st == OWH_UNHEALTHY) a->tests++;
    if ((a->st == OWH_HEALTHY && result == OWH_EV_SUCCESS) || a->st == OWH_OFFLINE) {
        arm(a, t); /* stay */
        return;
    }
    int se = 0, to = 0;
    for (int k = 0; k < a->nbuf; ++k) {
        se += a->buf[k] == OWH_EV_SYSTEM_ERROR;
        to += a->buf[k] == OWH_EV_TIMEOUT;
    }
    go(a, se > OWH_TOLERANCE ? OWH_UNHEALTHY : to > OWH_TOLERANCE ? OWH_UNRESPONSIVE : OWH_HEALTHY, t);
}

/* One batch of supervision events in mailbox order, then timers up to now_ms.  Returns 0, or -1 on a bad argument
 * (kind > 4, negative invoker, decreasing time), -2 out of memory.  mem[i] = the pinging instance's userMemory. */
int owh_events(owh_pool* p, int32_t n, const int32_t* inv, const uint8_t* kind, const int64_t* t_ms,
               const int64_t* mem, int64_t now_ms) {
    int64_t prev = p->now;
    for (int32_t e = 0; e < n; ++e) {
        if (kind[e] > OWH_EV_STATE_TIMEOUT || inv[e] < 0 || t_ms[e] < prev) return -1;
        prev = t_ms[e];
    }
    if (now_ms < prev) return -1;
    p->now = now_ms;
    for (int32_t i = 0; i < p->size; ++i) p->v[i].tests = 0;
    for (int32_t e = 0; e < n; ++e) {
        const int32_t id = inv[e];
        const int64_t t = t_ms[e];
        /* an invoker's timers only act on its own actor, so they are fired when its next event arrives (and for
         * every actor at the end of the batch) */
        if (id < p->size && p->v[id].st < OWH_PADDED) fire_due(&p->v[id], t);
        if (kind[e] == OWH_EV_PING) {
            if (id >= p->size || p->v[id].st >= OWH_PADDED) { /* registerInvoker (ISUP:180-199) */
                if (grow(p, id + 1)) return -2;
                for (int32_t i = p->size; i < id; ++i) {  /* padToIndexed: Offline, userMemory of this instance */
                    p->v[i].st = OWH_PADDED;
                    p->v[i].mem = mem[e];
                }
                if (id + 1 > p->size) p->size = id + 1;
                owh_inv* a = &p->v[id];
                a->nbuf = 0;
                a->tick = OWH_NEVER;
                a->st = OWH_UNHEALTHY; /* startWith(Unhealthy) + initialize(): handlers of _ -> Unhealthy */
                a->tests++;
                a->tick = t + OWH_TICK_MS;
            }
            owh_inv* a = &p->v[id];
            a->mem = mem[e]; /* status.updated(..., new InvokerHealth(p.instance, oldHealth.status)) */
            if (a->st == OWH_OFFLINE) go(a, OWH_UNHEALTHY, t);
            else arm(a, t); /* stay */
        } else if (id < p->size && p->v[id].st < OWH_PADDED) {
            owh_inv* a = &p->v[id];
            if (kind[e] == OWH_EV_STATE_TIMEOUT) {
                /* an FSM.StateTimeout message: handled in the states that have a timeout, unhandled (stay) in Offline */
                if (has_timeout(a->st)) go(a, OWH_OFFLINE, t);
                else arm(a, t);
            } else {
                completion(a, kind[e], t);
            }
        } /* else: instanceToRef.get(...) is None -- dropped (ISUP:134-136) */
    }
    for (int32_t i = 0; i < p->size; ++i)
        if (p->v[i].st < OWH_PADDED) fire_due(&p->v[i], now_ms);
    return 0;
}

int32_t owh_size(const owh_pool* p) { return p->size; }

/* status vector (InvokerState, padded entries Offline), userMemory, test actions of the last batch, ring buffers
 * packed 2 bits per result oldest first | count << 20, next Tick (-1 = none) */
void owh_read(const owh_pool* p, uint8_t* status, int64_t* mem, int32_t* tests, uint32_t* ring, int64_t* tick) {
    for (int32_t i = 0; i < p->size; ++i) {
        const owh_inv* a = &p->v[i];
        if (status) status[i] = a->st >= OWH_PADDED ? OWH_OFFLINE : a->st;
        if (mem) mem[i] = a->mem;
        if (tests) tests[i] = a->tests;
        if (ring) {
            uint32_t r = (uint32_t)a->nbuf << 20;
            for (int k = 0; k < a->nbuf; ++k) r |= (uint32_t)(a->buf[k] & 3) << (2 * k);
            ring[i] = r;
        }
        if (tick) tick[i] = a->tick == OWH_NEVER ? -1 : a->tick;
    }
}
