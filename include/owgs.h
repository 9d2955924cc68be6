/*
 * owgs.h -- C ABI of the MI355X-native batched invoker scheduler ("GPU sharding" balancer).
 *
 * This is the drop-in boundary for OpenWhisk's controller-side invoker assignment hot path.  A JVM shim
 * (GpuShardingContainerPoolBalancer) binds these symbols over JNI and keeps everything
 * else of CommonLoadBalancer (activation bookkeeping, Kafka send, ack feed) on the JVM side.
 * Paths below are relative to the reference repository root; abbreviations:
 *   SCPB = core/controller/src/main/scala/org/apache/openwhisk/core/loadBalancer/ShardingContainerPoolBalancer.scala
 *   CLB  = core/controller/src/main/scala/org/apache/openwhisk/core/loadBalancer/CommonLoadBalancer.scala
 *   LB   = core/controller/src/main/scala/org/apache/openwhisk/core/loadBalancer/LoadBalancer.scala
 *   NS   = common/scala/src/main/scala/org/apache/openwhisk/common/NestedSemaphore.scala
 *
 * Conventions
 *   - Every entry point returns 0 on success or a negative OWGS_E* code; nothing throws or aborts across the ABI.
 *     owgs_last_error() describes the last failure of a context.
 *   - Buffers are owned by the caller.  Functions without a _device suffix take HOST pointers; *_device functions
 *     take HIP device pointers (HBM-resident) and an optional hipStream_t passed as void*.
 *   - Per-activation outcome: out_invoker >= 0 is the chosen invoker id; OWGS_NONE (-1) is the reference's None
 *     ("No invokers available", SCPB:305-316); OWGS_THROW_INDEX (-2) marks an input for which the reference's
 *     schedule() throws IndexOutOfBoundsException (Int.MinValue hash, SCPB:266-268/411, or an invoker id outside
 *     invokerSlots, SCPB:413/422).  out_flags bit0 (OWGS_FLAG_OVERLOAD) = overload random fallback + forceAcquire
 *     (SCPB:417-424); the JVM shim turns it into the MANAGED/BLACKBOX_SYSTEM_OVERLOAD counter (SCPB:277-286).
 *   - Release flags: bit0 NoSuchElementException (NS:103), bit1 permit overflow Error (ForcibleSemaphore.scala:48-50),
 *     bit2 activation has no entry (it was never scheduled: CLB:278-279 finds no ActivationEntry).
 *   - Sequential semantics: a batch is equivalent to the reference executing, in array order, one schedule()
 *     (or releaseInvoker()) per element against the single-writer context.  The random overload fallback draws
 *     its index with the counter RNG keyed by (rng_seed, seq) documented in DESIGN.md (replaces ThreadLocalRandom,
 *     SCPB:421).
 *   - One context = one controller shard (SCPB horizontal sharding, SCPB:126-133); contexts are single-writer.
 *   - Calls on one context take effect in the order they are issued, whatever stream each names: an asynchronous call
 *     (the *_device functions, owgs_restore, owgs_update_health_device) leaves its work as the context's tail, and
 *     the next call -- on any stream, or a synchronous one -- is ordered after it on the device.  Device buffers the
 *     caller passes to an asynchronous call are read when `stream` reaches the call's work: keep them valid (and
 *     unmodified) until then.
 */
#ifndef OWGS_H
#define OWGS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OWGS_ABI_VERSION 1

#define OWGS_OK 0
#define OWGS_EINVAL (-22)  /* bad argument */
#define OWGS_ENOMEM (-12)  /* allocation failed (host or device) */
#define OWGS_EDEVICE (-5)  /* HIP runtime error */
#define OWGS_ERANGE (-34)  /* state too large for the engine (see owgs_limits) */
#define OWGS_ENOENT (-2)   /* unknown action / invoker */

#define OWGS_NONE (-1)
#define OWGS_THROW_INDEX (-2)
#define OWGS_FLAG_OVERLOAD 1u

#define OWGS_REL_NOSUCHELEMENT 1u
#define OWGS_REL_OVERFLOW 2u
#define OWGS_REL_NOENTRY 4u

/* InvokerState (core/controller/.../loadBalancer/InvokerSupervision.scala:47-66): only HEALTHY is usable. */
#define OWGS_HEALTHY 0
#define OWGS_UNHEALTHY 1
#define OWGS_UNRESPONSIVE 2
#define OWGS_OFFLINE 3

typedef struct owgs_ctx owgs_ctx;

typedef struct owgs_config {
    double managed_fraction;  /* whisk.loadbalancer.managed-fraction  (core/controller/src/main/resources/reference.conf:22-32) */
    double blackbox_fraction; /* whisk.loadbalancer.blackbox-fraction */
    int64_t min_memory_bytes; /* MemoryLimit.MIN_MEMORY (common/scala/src/main/resources/application.conf:377) */
    int32_t cluster_size;     /* initial cluster size (SCPB:457 default 1) */
    int32_t device;           /* HIP device ordinal */
    uint64_t rng_seed;        /* overload-fallback RNG seed (DESIGN.md "Counter RNG") */
} owgs_config;

/* Replaces: object ShardingContainerPoolBalancer.instance(...) building the balancer (SCPB:336-365) and
 * ShardingContainerPoolBalancerState() (SCPB:449-470). */
int owgs_create(const owgs_config* cfg, owgs_ctx** out);
void owgs_destroy(owgs_ctx* ctx);
const char* owgs_last_error(const owgs_ctx* ctx);
int owgs_abi_version(void);
/* Diagnostics (runs without a GPU): each engine object (wide / narrow geometry) refuses a launch prepared for the other
 * geometry before anything runs -- the launch wrappers compare the host's geometry tag with their own, and the kernels
 * check it again before their first barrier (a mismatch fails the call with OWGS_EDEVICE, "engine geometry").
 * OWGS_OK when every wrapper refused. */
int owgs_geometry_selfcheck(void);
/* max invokers / slots the engine holds on chip (LDS); larger pools return OWGS_ERANGE from update_invokers */
int owgs_limits(int32_t* max_invokers, int32_t* max_slots);

/* Replaces: ShardingContainerPoolBalancerState.updateInvokers(newInvokers: IndexedSeq[InvokerHealth]) (SCPB:512-551),
 * driven by the monitor actor on CurrentInvokerPoolState (SCPB:226-227).  status: OWGS_HEALTHY..OWGS_OFFLINE. */
int owgs_update_invokers(owgs_ctx* ctx, int32_t n, const int32_t* ids, const int64_t* user_memory_bytes,
                         const uint8_t* status);

/* Replaces: ShardingContainerPoolBalancerState.updateCluster(newSize) (SCPB:561-584), driven by the Akka cluster
 * membership events in the monitor actor (SCPB:230-248). */
int owgs_update_cluster(owgs_ctx* ctx, int32_t new_size);

/* Registers actions (the per-activation inputs of publish, SCPB:260-276).  For action i:
 *   namespace  = msg.user.namespace.name.asString   (SCPB:266, hashed)
 *   path       = action.fullyQualifiedName(false).asString, e.g. "ns/pkg/name" (SCPB:266, hashed)
 *   key        = action.fullyQualifiedName(true).asString ("ns/pkg/name@0.0.1"): the NestedSemaphore map key (SCPB:271)
 *   mem_mb     = action.limits.memory.megabytes (SCPB:274);  max_conc = action.limits.concurrency.maxConcurrent (SCPB:270)
 *   blackbox   = action.exec.pull (SCPB:260)
 * Strings are concatenated in *_bytes with offsets *_off[0..n] (n+1 entries).  generateHash (SCPB:370-372) runs on the
 * GPU; out_hash (optional) receives it, out_action receives the action handle used by the batch calls. */
int owgs_register_actions(owgs_ctx* ctx, int32_t n, const char* ns_bytes, const int32_t* ns_off,
                          const char* path_bytes, const int32_t* path_off, const char* key_bytes,
                          const int32_t* key_off, const int32_t* mem_mb, const int32_t* max_conc,
                          const uint8_t* blackbox, int32_t* out_action, int32_t* out_hash);

/* Replaces the reference's NestedSemaphore map lifetime (NestedSemaphore.scala:109-111: an entry exists only while
 * activations of its fqn@version are in flight; nothing else is keyed by it).  The caller drops action handles it will
 * not name again (a cold action, a superseded fqn@version): none of their activations may still be in flight and no
 * later call may name them.  Handle ids are reused by later owgs_register_actions calls; an fqn@version key that no
 * live handle names is recycled when registrations run out of key ids, once no map entry and no watched pair holds it
 * (a device scan; keys still held stay pending).  A restore of a snapshot taken before a key was recycled returns
 * OWGS_EINVAL.  With this a long-running controller never runs out of the 131,070 key / 131,070 handle ids. */
int owgs_release_actions(owgs_ctx* ctx, int32_t n, const int32_t* actions);

/* Replaces: the scheduling half of ShardingContainerPoolBalancer.publish (SCPB:257-290) -- pool selection, hash,
 * home invoker, step size and ShardingContainerPoolBalancer.schedule (SCPB:398-436) with NestedSemaphore
 * tryAcquireConcurrent / forceAcquireConcurrent (NS:32-91) -- for n activations in array order.
 * seq[i] keys the overload RNG (may be NULL: seq = seq_base + i). */
int owgs_publish_batch(owgs_ctx* ctx, int32_t n, const int32_t* action, const uint64_t* seq, uint64_t seq_base,
                       int32_t* out_invoker, uint8_t* out_flags);

/* Replaces: ShardingContainerPoolBalancer.releaseInvoker (SCPB:327-331) reached from CommonLoadBalancer
 * .processCompletion (CLB:260-346): invokerSlots.lift(invoker).foreach(_.releaseConcurrent(fqn, maxConcurrent, mem)).
 * invoker < 0 means "no ActivationEntry" (flag OWGS_REL_NOENTRY, no state change). out_flags may be NULL. */
int owgs_release_batch(owgs_ctx* ctx, int32_t n, const int32_t* invoker, const int32_t* action, uint8_t* out_flags);

/* Replaces: one drained batch of the JVM shim's batching thread -- for each run r in order, releaseInvoker for the
 * completions [rel_off[r], rel_off[r+1]) (SCPB:327-331 via CommonLoadBalancer.processCompletion, CLB:260-346; invoker
 * and action handle of the ActivationEntry, invoker < 0 = no entry) and then the scheduling half of publish
 * (SCPB:257-290) for the activations [pub_off[r], pub_off[r+1]).  Same results as alternating owgs_release_batch and
 * owgs_publish_batch calls.  Small calls on identity pools without watched pairs (at most OWGS_RES_MAX = 1024
 * releases + publishes by default) are served by a resident engine that keeps the slot state on chip between calls:
 * inputs and outputs through pinned host memory, a doorbell, no launch or synchronisation per call; it writes the
 * state back and exits when any other entry point of the context is called, or after 20 ms without a call
 * (OWGS_RES_IDLE_US; OWGS_RESIDENT=0 disables it).  Other calls: one pinned copy in, one launch chain, one pinned copy
 * out, one synchronisation.  rel_off / pub_off have n_runs + 1 entries starting at 0; seq may be NULL (seq = seq_base
 * + publish index); rel_flags may be NULL. */
int owgs_process_batch(owgs_ctx* ctx, int32_t n_runs, const int32_t* rel_off, const int32_t* rel_invoker,
                       const int32_t* rel_action, uint8_t* rel_flags, const int32_t* pub_off,
                       const int32_t* pub_action, const uint64_t* seq, uint64_t seq_base, int32_t* out_invoker,
                       uint8_t* out_flags);

/* Replaces: ShardingContainerPoolBalancer.schedule(maxConcurrent, fqn, invokers, dispatched, slots, index, step)
 * (SCPB:398-436) called directly with an explicit walk, as the reference unit tests do (ShardingContainerPoolBalancer
 * Tests.scala:244-412).  pool = 0 managed / 1 blackbox pool of the context; key = slot-key id (see owgs_key_id). */
int owgs_schedule_walks(owgs_ctx* ctx, int32_t n, const uint8_t* pool, const int32_t* index, const int32_t* step,
                        const int32_t* mem_mb, const int32_t* max_conc, const int32_t* key, const uint64_t* seq,
                        int32_t* out_invoker, uint8_t* out_flags);

/* Test seam mirroring `protected[loadBalancer] var _invokerSlots` (SCPB:455): replace the slot vector with n fresh
 * NestedSemaphores of the given memory permits (concurrency maps emptied). */
int owgs_set_slots(owgs_ctx* ctx, int32_t n, const int32_t* permits);
/* Replaces the pool vectors for the explicit-walk tests: managed pool = (ids, status) as given. */
int owgs_set_pool(owgs_ctx* ctx, int32_t pool, int32_t n, const int32_t* ids, const uint8_t* status);

/* Introspection (ForcibleSemaphore.availablePermits / NestedSemaphore.concurrentState / state getters). */
int owgs_read_permits(owgs_ctx* ctx, int32_t* out, int32_t cap, int32_t* n_slots);
int owgs_read_concurrent(owgs_ctx* ctx, int32_t invoker, int32_t key, int32_t* permits, int32_t* op_count);
int owgs_key_id(owgs_ctx* ctx, int32_t action);
/* Diagnostics (synchronises): the NestedSemaphore map's fill -- live and deleted entries of the on-chip primary table,
 * entries (live + deleted) and capacity of the HBM overflow. */
int owgs_map_fill(owgs_ctx* ctx, int32_t* primary_live, int32_t* primary_deleted, int32_t* overflow_entries,
                  int32_t* overflow_cap);
int owgs_state_info(owgs_ctx* ctx, int32_t* n_invokers, int32_t* managed, int32_t* blackbox, int32_t* cluster_size);
int owgs_step_sizes(owgs_ctx* ctx, int32_t pool, int32_t* out, int32_t cap, int32_t* n);

/* Replaces: ShardingContainerPoolBalancer.pairwiseCoprimeNumbersUntil(x) (SCPB:379-384), the step-size table that
 * updateInvokers (SCPB:525-527) rebuilds on the device; exposed for the reference's unit test
 * (ShardingContainerPoolBalancerTests.scala:371-384).  Writes min(cap, n) values to out (may be NULL), n = list length.
 * x > owgs_limits' pool range returns OWGS_ERANGE. */
int owgs_pairwise_coprime(owgs_ctx* ctx, int32_t x, int32_t* out, int32_t cap, int32_t* n);

/* Stream replay with HBM-resident buffers (bench / batching thread).  Batch b first releases the activations
 * rel_aid[rel_off[b]..rel_off[b+1]) (ids into this stream; their invoker is this stream's own earlier output),
 * then publishes activations [acq_off[b], acq_off[b+1]) with action act[i] and seq = seq_base + i.
 * n_activations = acq_off[n_batches], n_releases = rel_off[n_batches] (given so no device read is needed).
 * All pointers are device pointers; stream is a hipStream_t (NULL = the context's stream).  Asynchronous, with one
 * exception: when the call's activations could fill the HBM overflow of the NestedSemaphore map past half its capacity
 * (its upper bound: the entries it holds plus one per activation), the call first synchronises `stream`, reads the
 * exact entry count back and, if still needed, grows and rehashes the table before launching. */
int owgs_replay_device(owgs_ctx* ctx, int32_t n_batches, const int64_t* acq_off, const int32_t* act,
                       int64_t n_activations, const int64_t* rel_off, const int64_t* rel_aid, int64_t n_releases,
                       uint64_t seq_base, int32_t* out_invoker, uint8_t* out_flags, uint8_t* rel_flags, void* stream);
/* One batch of a stream replayed batch by batch, so that state updates can come in between (configs[4]: the health
 * all-gather between batches feeding owgs_update_health_device, i.e. updateInvokers, SCPB:512-551): releases
 * rel_aid[r_beg, r_end) -- activations of this stream decided by EARLIER calls, their invoker read from out_invoker --
 * then publishes act[a_beg, a_end) with seq = seq_base + i; every index is into the whole stream's arrays (device
 * pointers).  Same results as the batch inside one owgs_replay_device call of the whole stream with the same state
 * updates between batches.  Asynchronous on `stream` (same exception as owgs_replay_device). */
int owgs_replay_device_span(owgs_ctx* ctx, int64_t a_beg, int64_t a_end, int64_t r_beg, int64_t r_end,
                            const int32_t* act, const int64_t* rel_aid, uint64_t seq_base, int32_t* out_invoker,
                            uint8_t* out_flags, uint8_t* rel_flags, void* stream);
/* Consecutive batches of a stream replayed batch by batch in ONE engine launch, with a health vector applied before
 * each batch (configs[4]'s cadence: the health all-gathered between batches, applied as updateInvokers with a new
 * status vector, SCPB:512-551, before the batch's releases).  acq_off / rel_off are HOST arrays [n_batches + 1] of
 * indices into the whole stream's device arrays (as owgs_replay_device_span's a_beg..r_end, per batch); releases may
 * name activations decided by earlier calls or by earlier batches of this group.  status_dev (device, nullable):
 * row b = status_dev + b * status_stride holds n_status InvokerState codes (n_status = the context's invokers);
 * after the call the context's health is the last row's.  Same results as owgs_update_health_device(row b) +
 * owgs_replay_device_span(batch b) for every b.  Identity pools without watched pairs run one launch; otherwise the
 * call takes exactly that batch-by-batch sequence.  Asynchronous on `stream` (same exception as owgs_replay_device). */
int owgs_replay_device_group(owgs_ctx* ctx, int32_t n_batches, const int64_t* acq_off, const int64_t* rel_off,
                             const int32_t* act, const int64_t* rel_aid, uint64_t seq_base, int32_t* out_invoker,
                             uint8_t* out_flags, uint8_t* rel_flags, const uint8_t* status_dev, int64_t status_stride,
                             int32_t n_status, void* stream);
/* Several controller shards (clusterSize > 1, one context each, same device) replayed by ONE engine launch, one
 * workgroup per shard: the reference runs one ShardingContainerPoolBalancer per controller (SCPB:126-133,
 * 485-499); this hosts up to 64 of them on one GPU (up to 8 argument blocks travel in the kernarg segment, more
 * through a pinned host buffer and HBM owned by ctxs[0]).  io[i] holds owgs_replay_device's arguments for ctxs[i];
 * every shard needs n_batches > 0.  Same results as k separate owgs_replay_device calls.  Asynchronous on `stream`
 * (same exception as owgs_replay_device, per shard). */
typedef struct owgs_replay_io {
    int32_t n_batches;
    const int64_t* acq_off;
    const int32_t* act;
    int64_t n_activations;
    const int64_t* rel_off;
    const int64_t* rel_aid;
    int64_t n_releases;
    uint64_t seq_base;
    int32_t* out_invoker;
    uint8_t* out_flags;
    uint8_t* rel_flags;
} owgs_replay_io;
int owgs_replay_device_multi(owgs_ctx** ctxs, int32_t k, const owgs_replay_io* io, void* stream);
/* Same with host buffers (copies in and out, synchronous). */
int owgs_replay(owgs_ctx* ctx, int32_t n_batches, const int64_t* acq_off, const int32_t* act, const int64_t* rel_off,
                const int64_t* rel_aid, uint64_t seq_base, int32_t* out_invoker, uint8_t* out_flags,
                uint8_t* rel_flags);

/* ---- completion path (CommonLoadBalancer.processAcknowledgement / processCompletion, CLB:205-346) ----------------
 * activationSlots (CLB:60) lives on the device: an activation is tracked when it is published and removed by its
 * completion ack.  Per-message outcome codes (out_kind): */
#define OWGS_ACK_FAIL 0           /* AcknowledegmentMessage.parse fails (CLB:226-228): the shim logs the raw message */
#define OWGS_ACK_JVM 1            /* the message has a "response" member (ResultMessage / Combined...): its
                                     WhiskActivation is deserialised by the JVM, which completes the slot with
                                     owgs_complete_activations */
#define OWGS_ACK_UNSUPPORTED 2    /* outside the device parser's limits (container depth > 64, an exponent of more
                                     than 9 digits, a non-ASCII or numeric activation id, U+FFFF, a number of more
                                     than 34 significant digits in instance / transid): the JVM parses it */
#define OWGS_ACK_RELEASED 3       /* processCompletion found the entry: releaseInvoker ran (CLB:286-319) */
#define OWGS_ACK_HEALTH 4         /* no entry, transid == TransactionId.invokerHealth (CLB:320-328) */
#define OWGS_ACK_NOENTRY 5        /* no entry, regular ack after a forced one (CLB:329-337) */
#define OWGS_ACK_FORCED_NOENTRY 6 /* no entry, forced (timeout) after a regular ack (CLB:338-345) */

/* TransactionId.invokerHealth's start (TransactionId.scala:225) of this controller: health acks echo it. */
int owgs_set_health_tid(owgs_ctx* ctx, int64_t start_ms);

/* Replaces: activationSlots.getOrElseUpdate(msg.activationId, ActivationEntry(...)) in setupActivation (CLB:148-166),
 * in array order.  aid32 = n activation ids of 32 chars [0-9a-f] (ActivationId.asString, no terminator); action =
 * the action handle (its limits and fqn@version are the entry's); ticket = the caller's handle for its own per-
 * activation state (promise, timeout handler).  out_ticket = the ticket of the entry now in the map (the existing
 * one when out_existed = 1). */
int owgs_track_activations(owgs_ctx* ctx, int32_t n, const char* aid32, const int32_t* action, const int32_t* ticket,
                           int32_t* out_ticket, uint8_t* out_existed);

/* Replaces: processAcknowledgement (CLB:205-232) for n raw ack messages (UTF-8 bytes, offsets off[0..n]) processed
 * in array order: AcknowledegmentMessage.parse (Message.scala:237-256) on the device, then for every
 * CompletionMessage processCompletion(aid, tid, forced = false, isSystemError, invoker) (CLB:260-346): the entry is
 * removed and releaseInvoker(invoker, entry) (SCPB:327-331) applied.  out_invoker = the message's invoker instance,
 * out_ticket = the removed entry's ticket (-1 otherwise), out_flags bit0 = isSystemError, bits1-2 = the release
 * flags (OWGS_REL_NOSUCHELEMENT, OWGS_REL_OVERFLOW) of releaseInvoker.  The shim sends InvocationFinishedMessage
 * for RELEASED / HEALTH outcomes and completes promises for OWGS_ACK_JVM messages. */
int owgs_process_acks(owgs_ctx* ctx, int32_t n, const char* bytes, const int64_t* off, uint8_t* out_kind,
                      int32_t* out_invoker, int32_t* out_ticket, uint8_t* out_flags);
/* Same with device buffers (bytes padded by 16 readable bytes past off[n]); stream as in owgs_replay_device. */
int owgs_process_acks_device(owgs_ctx* ctx, int32_t n, const uint8_t* bytes, const int64_t* off, uint8_t* out_kind,
                             int32_t* out_invoker, int32_t* out_ticket, uint8_t* out_flags, void* stream);

/* Replaces: processCompletion (CLB:260-346) called directly -- the completion-ack timeout (forced, CLB:150-152) and
 * the completion half of messages the JVM parsed itself (OWGS_ACK_JVM).  flags bit0 forced, bit1 isSystemError,
 * bit2 transid == invokerHealth.  Outcomes and out_flags as in owgs_process_acks. */
int owgs_complete_activations(owgs_ctx* ctx, int32_t n, const char* aid32, const int32_t* invoker,
                              const uint8_t* flags, uint8_t* out_kind, int32_t* out_ticket, uint8_t* out_flags);
/* activationSlots.size */
int owgs_activations_live(owgs_ctx* ctx, int64_t* live);

/* ---- invoker health supervision ----
 * Replaces: InvokerPool (InvokerSupervision.scala:95-210: registerInvoker on the first ping, padToIndexed with Offline
 * entries, InvocationFinishedMessage forwarding) and one InvokerActor FSM per invoker (InvokerSupervision.scala:
 * 285-440: Offline / Unhealthy / Unresponsive / Healthy, 10 s state timeout, 1-minute Tick sending test actions
 * while Unhealthy or Unresponsive, a ring buffer of the last 10 results with tolerance 3).
 * Events are in mailbox order with non-decreasing times (ms, in [0, 2^60)) that never go back before the previous
 * batch's now_ms;
 * timers due at or before an event's time fire before it, and all timers due at or before now_ms fire at the end.
 * user_memory_bytes = the pinging InvokerInstanceId's userMemory (ignored for other kinds).  apply != 0 hands the
 * resulting status vector to owgs_update_invokers (the monitor's CurrentInvokerPoolState -> updateInvokers,
 * SCPB:226-227).  Bad kinds, negative ids or times out of order: OWGS_EINVAL with no state change. */
#define OWGS_HEALTH_MAX_ID (1 << 24) /* invoker ids accepted by owgs_health_events (the status vector is dense) */
#define OWGS_EV_PING 0          /* PingMessage (InvokerSupervision.scala:120-131) */
#define OWGS_EV_SUCCESS 1       /* InvocationFinishedMessage(InvocationFinishedResult.Success) */
#define OWGS_EV_SYSTEM_ERROR 2  /* ... SystemError */
#define OWGS_EV_TIMEOUT 3       /* ... Timeout */
#define OWGS_EV_STATE_TIMEOUT 4 /* an FSM.StateTimeout message to the invoker's actor */
int owgs_health_events(owgs_ctx* ctx, int32_t n, const int32_t* invoker, const uint8_t* kind, const int64_t* t_ms,
                       const int64_t* user_memory_bytes, int64_t now_ms, int32_t apply);
/* Replaces: InvokerPool's GetStatus (status vector, InvokerSupervision.scala:132) plus per-invoker detail: userMemory
 * of the instance in the status vector, test actions sent during the last batch (invokeTestAction,
 * InvokerSupervision.scala:416-434), the ring buffer (2 bits per result oldest first: 1 Success, 2 SystemError,
 * 3 Timeout; count << 20) and the next Tick (-1: none).  *n = the status vector's length; any output may be NULL. */
int owgs_health_read(owgs_ctx* ctx, int32_t cap, int32_t* n, uint8_t* status, int64_t* user_memory_bytes,
                     int32_t* test_actions, uint32_t* ring, int64_t* next_tick);

/* ---- ActivationMessage serialisation + per-invoker topic fan-out ----
 * Replaces: ActivationMessage.serialize (jsonFormat11 + spray-json compactPrint, Message.scala:51-70, 170-175) and
 * the per-activation producer.send to topic "invoker<N>" (sendActivationToInvoker, CommonLoadBalancer.scala:175-198)
 * for a batch of publishes.  The invariant members are templates printed once per (action, identity) by the caller:
 * part A = the three members `"action":<fqn>,"revision":<rev>,"user":<identity>` (no surrounding commas), part B =
 * the initArgs array value; rootControllerIndex is one JSON value per context.  Templates append; returns the id
 * of the first new one. */
int owgs_register_templates(owgs_ctx* ctx, int32_t n, const char* a_bytes, const int64_t* a_off, const char* b_bytes,
                            const int64_t* b_off, int32_t* out_first_id);
int owgs_set_root_controller(owgs_ctx* ctx, const char* json, int32_t len);

#define OWGS_MSG_BLOCKING 1       /* ActivationMessage.blocking */
#define OWGS_MSG_EXTRA_LOGGING 2  /* transid.meta.extraLogging: ["id", start, true] */
#define OWGS_MSG_HAS_CONTENT 4    /* content = Some(JsObject) (printed, in content/content_off) */
#define OWGS_MSG_HAS_CAUSE 8      /* cause = Some(ActivationId) */
#define OWGS_MSG_HAS_TRACE 16     /* traceContext = Some(Map) (printed, in trace/trace_off) */
typedef struct owgs_msg_batch {
    int32_t n;
    const int32_t* invoker;      /* the publish decisions (owgs_publish_batch out_invoker); < 0: no message */
    const int32_t* tmpl;         /* template id per activation */
    const uint64_t* aid;         /* 2 per activation: the 32 hex digits of ActivationId as (hi, lo) */
    const char* tid;             /* TransactionId.meta.id strings, UTF-8, offsets tid_off[0..n] */
    const int64_t* tid_off;
    const int64_t* tid_start;    /* TransactionId.meta.start, epoch ms */
    const uint8_t* flags;        /* OWGS_MSG_* */
    const char* content;         /* may be NULL when no flag asks for it */
    const int64_t* content_off;
    const uint64_t* cause;       /* 2 per activation */
    const char* trace;
    const int64_t* trace_off;
} owgs_msg_batch;
/* Host buffers.  Output: the m messages (activations with invoker >= 0) grouped by invoker id ascending, publish order
 * within a topic: bytes out[out_off[j] .. out_off[j+1]), out_order[j] = activation index, topic_start[k] ..
 * topic_start[k+1] = the messages of topic "invoker<k>" for k < n_topics.  out_off has n + 1 entries, out_order n,
 * topic_start n_topics + 1.  *total = bytes needed; OWGS_ERANGE (nothing written) when it exceeds cap; OWGS_EINVAL
 * for an invoker >= n_topics, an unknown template or a malformed UTF-8 transaction id. */
int owgs_serialize_activations(owgs_ctx* ctx, const owgs_msg_batch* batch, int32_t n_topics, char* out, int64_t cap,
                               int64_t* out_off, int32_t* out_order, int32_t* topic_start, int64_t* total,
                               int32_t* m);
/* Same with every pointer of batch and the outputs in device memory (e.g. invoker = owgs_replay_device's out_invoker),
 * on `stream`; content_off and trace_off are required (n + 1 zeros when unused); no host-side argument check beyond
 * NULLs (the device flags bad templates / invokers / UTF-8 as above); *total and *m are host values (the call
 * synchronises once). */
int owgs_serialize_activations_device(owgs_ctx* ctx, const owgs_msg_batch* batch, int32_t n_topics, char* out,
                                      int64_t cap, int64_t* out_off, int32_t* out_order, int32_t* topic_start,
                                      int64_t* total, int32_t* m, void* stream);

/* Duration of the last owgs_engine_kernel launch (HIP events recorded on its stream right before and after it);
 * waits for it to finish.  Measurement hook for bench.py's roofline. */
int owgs_engine_ms(owgs_ctx* ctx, float* ms);

/* Counters of owgs_process_batch's two paths: out[0] calls the resident engine served, [1] its launches, [2] calls it
 * refused untouched (a release that could leave the on-chip permit range; the chain took them), [3] calls the launch
 * chain took, [4] 1 while a resident engine is live; then, summed over the served calls: [5] walk rounds, [6]
 * decisions, [7] staging cycles, [8] release cycles, [9] publish cycles, [10] overflow lookups, [11] walks that
 * started at a cursor, [12] walks skipped by the pool permit bound, [13] decisions committed from speculative walks,
 * [14] validation passes, [15] decisions decided alone, [16] their cycles, [17] speculation cycles, [18] validation
 * cycles (the decisions decided alone included), [19..23] cycles of the speculation's rank matching, plain walks and
 * concurrent walks, of the validation's map inserts and of the releases' concurrent part; [24] chunks whose
 * concurrent decisions the helper wave speculated while wave 0 finished the chunk before, [25] the helper wave's
 * cycles in its concurrent walks; [26] the duration in ns of the last owgs_publish_batch / owgs_release_batch /
 * owgs_process_batch call, entry to return, timed inside the library; [27] 1 when the last owgs_replay /
 * owgs_replay_device(_span) ran through the resident engine's stream mode (OWGS_SPEC_REPLAY), [28..48] that replay's
 * counters [5..25] summed over its launch (waits for the context's stream, not for a live resident engine); [49],
 * [50] the largest primary-table fill (live + deleted entries) and deleted entries after a served call; [51], [52]
 * host nanoseconds over the served calls: building the call (records, chunk ranks), bell to answer; [53] launches
 * that ended at the engine's lifetime bound (OWGS_RES_LIFE_US, default 100 ms: it exits between calls so that
 * launches of other streams sharing its hardware queue are not held back); [54] served calls while watched pairs
 * existed (after owgs_update_cluster with activations in flight).  Returns the number of counters (55). */
int owgs_resident_stats(owgs_ctx* ctx, int64_t* out, int32_t cap);

/* Restore the slot state captured by owgs_snapshot (bench: every timed step starts from the same state). */
int owgs_snapshot(owgs_ctx* ctx);
int owgs_restore(owgs_ctx* ctx, void* stream);

/* Health all-gather hook (RCCL over xGMI, done by the caller): overwrite the status vector from a device buffer of
 * n bytes (InvokerState codes), e.g. the rank-0 row of an all_gather of CurrentInvokerPoolState.  Asynchronous on
 * `stream` for identity pools (the status bytes are copied and the usable bitmap rebuilt there; status_dev must stay
 * valid until `stream` reaches the copy); later calls on any stream see the new health (see Conventions). */
int owgs_update_health_device(owgs_ctx* ctx, int32_t n, const uint8_t* status_dev, void* stream);

/* Device self-test of the engine's wave primitives (DPP scans/reductions vs a serial computation); 0 = pass. */
int owgs_selftest(owgs_ctx* ctx);

/* Engine counters of the last engine launch (diagnostics): [0] resolution passes, [1] walk probes, [2] overload
 * fallbacks, [3] wave-cooperative long walks, [4] chunks, [5] passes that stopped before the chunk end,
 * [31] lanes re-decided inside their pass; [8..15] per-phase shader cycles in the diagnostic build
 * (libowgs_prof.so). */
int owgs_read_stats(owgs_ctx* ctx, uint64_t* out, int32_t cap);

#ifdef __cplusplus
}
#endif
#endif
