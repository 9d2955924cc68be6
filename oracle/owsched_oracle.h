/*
 * owsched_oracle.h -- CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the reference's controller-side invoker assignment path:
 *   ShardingContainerPoolBalancer.{generateHash, gcd, pairwiseCoprimeNumbersUntil, schedule}
 *     core/controller/src/main/scala/org/apache/openwhisk/core/loadBalancer/ShardingContainerPoolBalancer.scala:370-436
 *   ShardingContainerPoolBalancerState.{getInvokerSlot, updateInvokers, updateCluster}   (same file :449-585)
 *   ShardingContainerPoolBalancer.publish (pool/hash/home/step selection) / releaseInvoker  (same file :257-331)
 *   NestedSemaphore      common/scala/src/main/scala/org/apache/openwhisk/common/NestedSemaphore.scala:29-116
 *   ForcibleSemaphore    common/scala/src/main/scala/org/apache/openwhisk/common/ForcibleSemaphore.scala:37-124
 *   ResizableSemaphore   common/scala/src/main/scala/org/apache/openwhisk/common/ResizableSemaphore.scala:33-115
 *   java.lang.String.hashCode (JLS definition; JDK 11.0.3 per common/scala/Dockerfile:1, un-vendored)
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.  It is the
 * CHECKER for the HIP path (openwhisk_amd/csrc) and the CPU baseline ("kind": "port"), never the product.
 *
 * Pinning: every golden vector held by the reference's own unit tests for this path
 * (tests/src/test/scala/org/apache/openwhisk/core/loadBalancer/test/ShardingContainerPoolBalancerTests.scala,
 *  tests/src/test/scala/org/apache/openwhisk/common/{Nested,Forcible,Resizable}SemaphoreTests.scala) is
 * re-expressed in tests/golden/reference_unit_vectors.json and checked in tests/test_oracle_golden.py.
 * ThreadLocalRandom (SCPB:421) is replaced on both sides by the counter RNG below (bench-defined).
 *
 * Conventions (shared with include/owgs.h):
 *   schedule outcome: invoker id >= 0, OWO_NONE (-1) = None, OWO_THROW_INDEX (-2) = the reference would throw
 *   IndexOutOfBoundsException, OWO_THROW_ARG (-3) = IllegalArgumentException (require(...) failed).
 *   flags bit0 = overload (random fallback + forceAcquire).
 */
#ifndef OWSCHED_ORACLE_H
#define OWSCHED_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OWO_NONE (-1)
#define OWO_THROW_INDEX (-2)
#define OWO_THROW_ARG (-3)
#define OWO_THROW_NOSUCHELEMENT (-4)
#define OWO_THROW_OVERFLOW (-5)

/* invoker states (InvokerSupervision.scala:47-66); only Healthy isUsable */
#define OWO_HEALTHY 0
#define OWO_UNHEALTHY 1
#define OWO_UNRESPONSIVE 2
#define OWO_OFFLINE 3

/* ---- JDK / Scala primitives ---- */
int32_t owo_java_hash(const char* s, int32_t len);
int32_t owo_generate_hash(const char* ns, int32_t ns_len, const char* path, int32_t path_len);
int32_t owo_gcd(int32_t a, int32_t b);
int32_t owo_pairwise_coprime(int32_t x, int32_t* out, int32_t cap);
uint32_t owo_rng_index(uint64_t seed, uint64_t seq, uint32_t n);

/* ---- ResizableSemaphore (standalone, for T-RS vectors) ---- */
typedef struct owo_rs {
    int32_t c;   /* sync state (permits) */
    int32_t ops; /* operationCount */
    int32_t R;   /* reductionSize */
} owo_rs;
void owo_rs_init(owo_rs* s, int32_t max_allowed, int32_t reduction_size);
int owo_rs_try_acquire(owo_rs* s, int32_t acquires);                 /* 1/0, OWO_THROW_ARG */
int owo_rs_release(owo_rs* s, int32_t acquires, int op_complete);    /* bit0 memRel, bit1 actionRel; <0 throw */

/* ---- NestedSemaphore (ForcibleSemaphore + per-key ResizableSemaphore map) ---- */
typedef struct owo_ns owo_ns;
owo_ns* owo_ns_new(int32_t memory_permits, int zombies);
void owo_ns_free(owo_ns* s);
int owo_ns_try_acquire(owo_ns* s, int32_t acquires);
int owo_ns_force_acquire(owo_ns* s, int32_t acquires);
int owo_ns_release(owo_ns* s, int32_t acquires);
int32_t owo_ns_available(const owo_ns* s);
int owo_ns_try_acquire_concurrent(owo_ns* s, uint32_t key, int32_t max_conc, int32_t mem);
int owo_ns_force_acquire_concurrent(owo_ns* s, uint32_t key, int32_t max_conc, int32_t mem);
int owo_ns_release_concurrent(owo_ns* s, uint32_t key, int32_t max_conc, int32_t mem);
/* 1 if key present (c, ops written), 0 if absent */
int owo_ns_concurrent_state(const owo_ns* s, uint32_t key, int32_t* c, int32_t* ops);
int32_t owo_ns_concurrent_size(const owo_ns* s);

/* ---- vector of NestedSemaphores (the `dispatched` argument of schedule) ---- */
typedef struct owo_slots owo_slots;
owo_slots* owo_slots_new(int32_t count, int32_t permits, int zombies);
void owo_slots_free(owo_slots* v);
int32_t owo_slots_count(const owo_slots* v);
owo_ns* owo_slots_get(owo_slots* v, int32_t i);

/* ---- SCPB.schedule, literal (SCPB:398-436) ---- */
int owo_schedule(owo_slots* dispatched, int32_t max_conc, uint32_t key, int32_t n_invokers, const int32_t* inv_ids,
                 const uint8_t* inv_status, int32_t slots, int32_t index, int32_t step, uint64_t rng_seed,
                 uint64_t seq, int32_t* out_id, uint8_t* out_flags);

/* ---- ShardingContainerPoolBalancerState + publish/releaseInvoker ---- */
typedef struct owo_state owo_state;
owo_state* owo_state_new(double managed_fraction, double blackbox_fraction, int64_t min_memory_bytes,
                         uint64_t rng_seed, int zombies);
void owo_state_free(owo_state* st);
int owo_update_invokers(owo_state* st, int32_t n, const int32_t* ids, const int64_t* user_memory_bytes,
                        const uint8_t* status);
int owo_update_cluster(owo_state* st, int32_t new_size);
int32_t owo_cluster_size(const owo_state* st);
int32_t owo_n_invokers(const owo_state* st);
int32_t owo_managed_size(const owo_state* st);
int32_t owo_blackbox_size(const owo_state* st);
int32_t owo_managed_steps(const owo_state* st, int32_t* out, int32_t cap);
int32_t owo_blackbox_steps(const owo_state* st, int32_t* out, int32_t cap);
owo_slots* owo_state_slots(owo_state* st);
int32_t owo_read_permits(const owo_state* st, int32_t* out, int32_t cap);

/* actions: (invoking namespace, action path w/o version) -> hash; key = slot key (fqn@version id) */
int32_t owo_register_action(owo_state* st, const char* ns, int32_t ns_len, const char* path, int32_t path_len,
                            uint32_t key, int32_t mem_mb, int32_t max_conc, int32_t blackbox);
int32_t owo_action_hash(const owo_state* st, int32_t action);
int owo_publish(owo_state* st, int32_t action, uint64_t seq, int32_t* out_invoker, uint8_t* out_flags);
int owo_release(owo_state* st, int32_t invoker, int32_t action);

/* stream replay: batch b = releases rel_aid[rel_off[b]..rel_off[b+1]) then acquires [acq_off[b], acq_off[b+1]).
 * activation i has action act[i] and sequence number seq_base + i.  rel_flags: bit0 NoSuchElement,
 * bit1 overflow Error, bit2 activation had no entry (not scheduled). */
int owo_replay(owo_state* st, int32_t n_batches, const int64_t* acq_off, const int32_t* act, const int64_t* rel_off,
               const int64_t* rel_aid, uint64_t seq_base, int32_t* out_invoker, uint8_t* out_flags,
               uint8_t* rel_flags);

/* CPU baseline helper: replay nthreads independent shard streams concurrently (pthreads); returns 0 */
int owo_replay_parallel(owo_state** states, int32_t nthreads, int32_t n_batches, const int64_t* acq_off,
                        const int32_t* const* acts, const int64_t* rel_off, const int64_t* rel_aid, uint64_t seq_base,
                        int32_t* const* out_invoker, uint8_t* const* out_flags, uint8_t* const* rel_flags);

#ifdef __cplusplus
}
#endif
#endif
