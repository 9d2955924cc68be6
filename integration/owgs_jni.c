/*
 * owgs_jni.c -- JNI binding of include/owgs.h for integration/GpuShardingContainerPoolBalancer.scala
 * (this image has no JDK: tests/test_jni_syntax.py compiles it against a minimal stand-in of jni.h; build on a
 * controller host with
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I<repo>/include owgs_jni.c \
 *       -L<repo>/openwhisk_amd -lowgs -o libowgs_jni.so ).
 *
 * No JVM array is pinned across a GPU round trip: the hot call (processBatch, one drained batch of the shim) reads
 * and writes direct ByteBuffers (GetDirectBufferAddress: native memory the GC never moves), and every other entry
 * point copies its arrays in with Get<Type>ArrayRegion before the native call and out with Set<Type>ArrayRegion after
 * it.  Every length is checked in 64-bit arithmetic before any copy; a failed check or allocation returns OWGS_EINVAL /
 * OWGS_ENOMEM without calling the engine.  The native context is single-writer (the shim's batching thread).
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "owgs.h"

#define CTX(h) ((owgs_ctx*)(intptr_t)(h))

/* n must not exceed any of the given arrays (NULL = not given): a short array would be read / written past its end */
static int n_fits(JNIEnv* env, jlong n, jarray a, jarray b, jarray c, jarray d) {
    jarray xs[4] = {a, b, c, d};
    if (n < 0) return 0;
    for (int i = 0; i < 4; ++i)
        if (xs[i] && (jlong)(*env)->GetArrayLength(env, xs[i]) < n) return 0;
    return 1;
}

/* copies of Java arrays (n elements; NULL array or n == 0 -> a 1-element zeroed buffer so callers never see NULL) */
static void* jcopy_in(JNIEnv* env, jarray a, jlong n, size_t elem, char type) {
    void* p = calloc((size_t)(n > 0 ? n : 1), elem);
    if (!p || !a || n <= 0) return p;
    switch (type) {
        case 'I': (*env)->GetIntArrayRegion(env, (jintArray)a, 0, (jsize)n, (jint*)p); break;
        case 'J': (*env)->GetLongArrayRegion(env, (jlongArray)a, 0, (jsize)n, (jlong*)p); break;
        default: (*env)->GetByteArrayRegion(env, (jbyteArray)a, 0, (jsize)n, (jbyte*)p); break;
    }
    return p;
}
static void jcopy_out(JNIEnv* env, jarray a, jlong n, const void* p, char type) {
    if (!a || !p || n <= 0) return;
    switch (type) {
        case 'I': (*env)->SetIntArrayRegion(env, (jintArray)a, 0, (jsize)n, (const jint*)p); break;
        case 'J': (*env)->SetLongArrayRegion(env, (jlongArray)a, 0, (jsize)n, (const jlong*)p); break;
        default: (*env)->SetByteArrayRegion(env, (jbyteArray)a, 0, (jsize)n, (const jbyte*)p); break;
    }
}
#define FREE_ALL(...)                                  \
    do {                                               \
        void* fs_[] = {__VA_ARGS__};                   \
        for (size_t k_ = 0; k_ < sizeof fs_ / sizeof fs_[0]; ++k_) free(fs_[k_]); \
    } while (0)

JNIEXPORT jlong JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_create(
    JNIEnv* env, jobject self, jdouble mf, jdouble bf, jlong min_mem, jint cluster, jint device, jlong seed) {
    owgs_config cfg = {mf, bf, (int64_t)min_mem, (int32_t)cluster, (int32_t)device, (uint64_t)seed};
    owgs_ctx* c = NULL;
    return owgs_create(&cfg, &c) == OWGS_OK ? (jlong)(intptr_t)c : 0;
}

JNIEXPORT void JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_destroy(JNIEnv* env, jobject self,
                                                                                          jlong h) {
    owgs_destroy(CTX(h));
}

JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_updateInvokers(
    JNIEnv* env, jobject self, jlong h, jintArray ids, jlongArray mem, jbyteArray status) {
    if (!ids || !mem || !status) return OWGS_EINVAL;
    const jlong n = (*env)->GetArrayLength(env, ids);
    if (!n_fits(env, n, mem, status, NULL, NULL)) return OWGS_EINVAL;
    int32_t* pi = jcopy_in(env, ids, n, 4, 'I');
    int64_t* pm = jcopy_in(env, mem, n, 8, 'J');
    uint8_t* ps = jcopy_in(env, status, n, 1, 'B');
    int rc = OWGS_ENOMEM;
    if (pi && pm && ps) rc = owgs_update_invokers(CTX(h), (int32_t)n, pi, pm, ps);
    FREE_ALL(pi, pm, ps);
    return rc;
}

JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_updateCluster(JNIEnv* env,
                                                                                                jobject self, jlong h,
                                                                                                jint size) {
    return owgs_update_cluster(CTX(h), size);
}

JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_registerAction(
    JNIEnv* env, jobject self, jlong h, jstring ns, jstring path, jstring key, jint mem, jint maxc, jboolean bb) {
    if (!ns || !path || !key) return OWGS_EINVAL;
    const char* s0 = (*env)->GetStringUTFChars(env, ns, NULL);
    const char* s1 = (*env)->GetStringUTFChars(env, path, NULL);
    const char* s2 = (*env)->GetStringUTFChars(env, key, NULL);
    int rc = OWGS_ENOMEM;
    int32_t action = -1;
    if (s0 && s1 && s2) {
        const int32_t o0[2] = {0, (int32_t)strlen(s0)}, o1[2] = {0, (int32_t)strlen(s1)}, o2[2] = {0, (int32_t)strlen(s2)};
        const int32_t m = mem, c = maxc;
        const uint8_t b = bb ? 1 : 0;
        rc = owgs_register_actions(CTX(h), 1, s0, o0, s1, o1, s2, o2, &m, &c, &b, &action, NULL);
    }
    if (s2) (*env)->ReleaseStringUTFChars(env, key, s2);
    if (s1) (*env)->ReleaseStringUTFChars(env, path, s1);
    if (s0) (*env)->ReleaseStringUTFChars(env, ns, s0);
    return rc == OWGS_OK ? action : rc;
}

/* One drained batch (owgs_process_batch) over direct buffers, layout as BatchBuffers in the Scala shim:
 * in  = rel_off[n_runs + 1], pub_off[n_runs + 1], rel_invoker[n_rel], rel_action[n_rel], pub_action[n_pub] (int32);
 * out = out_invoker[n_pub] (int32), out_flags[n_pub], rel_flags[n_rel].  The publishes' overload-RNG sequence numbers
 * are seq_base, seq_base + 1, ... (the shim numbers them in queue order). */
JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_processBatch(
    JNIEnv* env, jobject self, jlong h, jobject in, jobject out, jint n_runs, jint n_rel, jint n_pub, jlong seq_base) {
    if (!in || !out || n_runs < 0 || n_rel < 0 || n_pub < 0) return OWGS_EINVAL;
    char* pi = (char*)(*env)->GetDirectBufferAddress(env, in);
    char* po = (char*)(*env)->GetDirectBufferAddress(env, out);
    if (!pi || !po) return OWGS_EINVAL;  /* not direct buffers */
    const jlong ints = 2 * ((jlong)n_runs + 1) + 2 * (jlong)n_rel + (jlong)n_pub;
    if ((*env)->GetDirectBufferCapacity(env, in) < 4 * ints ||
        (*env)->GetDirectBufferCapacity(env, out) < 5 * (jlong)n_pub + (jlong)n_rel)
        return OWGS_EINVAL;
    const int32_t* rel_off = (const int32_t*)pi;
    const int32_t* pub_off = rel_off + n_runs + 1;
    const int32_t* rel_inv = pub_off + n_runs + 1;
    const int32_t* rel_act = rel_inv + n_rel;
    const int32_t* pub_act = rel_act + n_rel;
    if (n_runs > 0 && (rel_off[n_runs] != n_rel || pub_off[n_runs] != n_pub)) return OWGS_EINVAL;
    return owgs_process_batch(CTX(h), n_runs, rel_off, rel_inv, rel_act, (uint8_t*)(po + 5 * (jlong)n_pub), pub_off,
                              pub_act, NULL, (uint64_t)seq_base, (int32_t*)po, (uint8_t*)(po + 4 * (jlong)n_pub));
}

/* handles of cold fqn@version keys (owgs_release_actions) */
JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_releaseActions(
    JNIEnv* env, jobject self, jlong h, jintArray handles, jint n) {
    if (!handles || !n_fits(env, n, handles, NULL, NULL, NULL)) return OWGS_EINVAL;
    int32_t* ph = jcopy_in(env, handles, n, 4, 'I');
    const int rc = ph ? owgs_release_actions(CTX(h), n, ph) : OWGS_ENOMEM;
    free(ph);
    return rc;
}

JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_publishBatch(
    JNIEnv* env, jobject self, jlong h, jintArray actions, jlongArray seq, jint n, jintArray out, jbyteArray flags) {
    if (!actions || !out || !flags || !n_fits(env, n, actions, seq, out, flags)) return OWGS_EINVAL;
    int32_t* pa = jcopy_in(env, actions, n, 4, 'I');
    uint64_t* ps = seq ? jcopy_in(env, seq, n, 8, 'J') : NULL;
    int32_t* po = calloc((size_t)(n > 0 ? n : 1), 4);
    uint8_t* pf = calloc((size_t)(n > 0 ? n : 1), 1);
    int rc = OWGS_ENOMEM;
    if (pa && po && pf && (ps || !seq)) rc = owgs_publish_batch(CTX(h), n, pa, ps, 0, po, pf);
    if (rc == OWGS_OK) {
        jcopy_out(env, out, n, po, 'I');
        jcopy_out(env, flags, n, pf, 'B');
    }
    FREE_ALL(pa, ps, po, pf);
    return rc;
}

JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_releaseBatch(
    JNIEnv* env, jobject self, jlong h, jintArray invokers, jintArray actions, jint n, jbyteArray flags) {
    if (!invokers || !actions || !n_fits(env, n, invokers, actions, flags, NULL)) return OWGS_EINVAL;
    int32_t* pi = jcopy_in(env, invokers, n, 4, 'I');
    int32_t* pa = jcopy_in(env, actions, n, 4, 'I');
    uint8_t* pf = calloc((size_t)(n > 0 ? n : 1), 1);
    int rc = OWGS_ENOMEM;
    if (pi && pa && pf) rc = owgs_release_batch(CTX(h), n, pi, pa, pf);
    if (rc == OWGS_OK) jcopy_out(env, flags, n, pf, 'B');
    FREE_ALL(pi, pa, pf);
    return rc;
}

/* ---- completion path (CommonLoadBalancer.setupActivation / processAcknowledgement / processCompletion) ---- */
JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_trackActivations(
    JNIEnv* env, jobject self, jlong h, jbyteArray aid32, jintArray actions, jintArray tickets, jint n,
    jintArray outTicket, jbyteArray outExisted) {
    if (!aid32 || !actions || !tickets || !outTicket || !outExisted ||
        !n_fits(env, n, actions, tickets, outTicket, outExisted) || !n_fits(env, 32LL * n, aid32, NULL, NULL, NULL))
        return OWGS_EINVAL;
    char* pa = jcopy_in(env, aid32, 32LL * n, 1, 'B');
    int32_t* pc = jcopy_in(env, actions, n, 4, 'I');
    int32_t* pt = jcopy_in(env, tickets, n, 4, 'I');
    int32_t* po = calloc((size_t)(n > 0 ? n : 1), 4);
    uint8_t* pe = calloc((size_t)(n > 0 ? n : 1), 1);
    int rc = OWGS_ENOMEM;
    if (pa && pc && pt && po && pe) rc = owgs_track_activations(CTX(h), n, pa, pc, pt, po, pe);
    if (rc == OWGS_OK) {
        jcopy_out(env, outTicket, n, po, 'I');
        jcopy_out(env, outExisted, n, pe, 'B');
    }
    FREE_ALL(pa, pc, pt, po, pe);
    return rc;
}

/* raw ack bytes of one feed batch (MessageFeed hands the consumer's records over as Array[Byte], LB:94-108) */
JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_processAcks(
    JNIEnv* env, jobject self, jlong h, jbyteArray bytes, jlongArray off, jint n, jbyteArray outKind,
    jintArray outInvoker, jintArray outTicket, jbyteArray outFlags) {
    if (!bytes || !off || !outKind || !outInvoker || !outTicket || !outFlags ||
        !n_fits(env, n, outKind, outInvoker, outTicket, outFlags) || !n_fits(env, (jlong)n + 1, off, NULL, NULL, NULL))
        return OWGS_EINVAL;
    int64_t* po = jcopy_in(env, off, (jlong)n + 1, 8, 'J');
    if (!po) return OWGS_ENOMEM;
    const jlong nb = (*env)->GetArrayLength(env, bytes);
    for (jint i = 0; i < n; ++i)
        if (po[i] < 0 || po[i + 1] < po[i] || po[i + 1] > nb) {
            free(po);
            return OWGS_EINVAL;
        }
    char* pb = jcopy_in(env, bytes, nb, 1, 'B');
    uint8_t* pk = calloc((size_t)(n > 0 ? n : 1), 1);
    int32_t* pi = calloc((size_t)(n > 0 ? n : 1), 4);
    int32_t* pt = calloc((size_t)(n > 0 ? n : 1), 4);
    uint8_t* pf = calloc((size_t)(n > 0 ? n : 1), 1);
    int rc = OWGS_ENOMEM;
    if (pb && pk && pi && pt && pf) rc = owgs_process_acks(CTX(h), n, pb, po, pk, pi, pt, pf);
    if (rc == OWGS_OK) {
        jcopy_out(env, outKind, n, pk, 'B');
        jcopy_out(env, outInvoker, n, pi, 'I');
        jcopy_out(env, outTicket, n, pt, 'I');
        jcopy_out(env, outFlags, n, pf, 'B');
    }
    FREE_ALL(po, pb, pk, pi, pt, pf);
    return rc;
}

JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_completeActivations(
    JNIEnv* env, jobject self, jlong h, jbyteArray aid32, jintArray invokers, jbyteArray flags, jint n,
    jbyteArray outKind, jintArray outTicket, jbyteArray outFlags) {
    if (!aid32 || !invokers || !flags || !outKind || !outTicket || !outFlags ||
        !n_fits(env, n, invokers, flags, outKind, outTicket) || !n_fits(env, n, outFlags, NULL, NULL, NULL) ||
        !n_fits(env, 32LL * n, aid32, NULL, NULL, NULL))
        return OWGS_EINVAL;
    char* pa = jcopy_in(env, aid32, 32LL * n, 1, 'B');
    int32_t* pi = jcopy_in(env, invokers, n, 4, 'I');
    uint8_t* pc = jcopy_in(env, flags, n, 1, 'B');
    uint8_t* pk = calloc((size_t)(n > 0 ? n : 1), 1);
    int32_t* pt = calloc((size_t)(n > 0 ? n : 1), 4);
    uint8_t* pf = calloc((size_t)(n > 0 ? n : 1), 1);
    int rc = OWGS_ENOMEM;
    if (pa && pi && pc && pk && pt && pf) rc = owgs_complete_activations(CTX(h), n, pa, pi, pc, pk, pt, pf);
    if (rc == OWGS_OK) {
        jcopy_out(env, outKind, n, pk, 'B');
        jcopy_out(env, outTicket, n, pt, 'I');
        jcopy_out(env, outFlags, n, pf, 'B');
    }
    FREE_ALL(pa, pi, pc, pk, pt, pf);
    return rc;
}

/* ---- invoker health supervision (InvokerPool + InvokerActor) ---- */
JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_healthEvents(
    JNIEnv* env, jobject self, jlong h, jintArray invokers, jbyteArray kinds, jlongArray tMs, jlongArray userMemory,
    jint n, jlong nowMs, jboolean apply) {
    if (!invokers || !kinds || !tMs || !userMemory || !n_fits(env, n, invokers, kinds, tMs, userMemory))
        return OWGS_EINVAL;
    int32_t* pi = jcopy_in(env, invokers, n, 4, 'I');
    uint8_t* pk = jcopy_in(env, kinds, n, 1, 'B');
    int64_t* pt = jcopy_in(env, tMs, n, 8, 'J');
    int64_t* pm = jcopy_in(env, userMemory, n, 8, 'J');
    int rc = OWGS_ENOMEM;
    if (pi && pk && pt && pm) rc = owgs_health_events(CTX(h), n, pi, pk, pt, pm, nowMs, apply ? 1 : 0);
    FREE_ALL(pi, pk, pt, pm);
    return rc;
}

/* status vector + test actions to send (the shim sends one health test action per count, InvokerPool.ActivationRequest) */
JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_healthRead(
    JNIEnv* env, jobject self, jlong h, jint cap, jbyteArray status, jlongArray userMemory, jintArray tests) {
    if (!status || !userMemory || !tests || !n_fits(env, cap, status, userMemory, tests, NULL)) return OWGS_EINVAL;
    int32_t n = 0;
    uint8_t* ps = calloc((size_t)(cap > 0 ? cap : 1), 1);
    int64_t* pm = calloc((size_t)(cap > 0 ? cap : 1), 8);
    int32_t* pt = calloc((size_t)(cap > 0 ? cap : 1), 4);
    int rc = OWGS_ENOMEM;
    if (ps && pm && pt) rc = owgs_health_read(CTX(h), cap, &n, ps, pm, pt, NULL, NULL);
    if (rc == OWGS_OK) {
        const jlong m = n < cap ? n : cap;
        jcopy_out(env, status, m, ps, 'B');
        jcopy_out(env, userMemory, m, pm, 'J');
        jcopy_out(env, tests, m, pt, 'I');
    }
    FREE_ALL(ps, pm, pt);
    return rc == OWGS_OK ? n : rc;
}

/* ---- ActivationMessage serialisation + topic fan-out ---- */
JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_registerTemplates(
    JNIEnv* env, jobject self, jlong h, jbyteArray a, jlongArray aOff, jbyteArray b, jlongArray bOff, jint n) {
    if (!a || !aOff || !b || !bOff || !n_fits(env, (jlong)n + 1, aOff, bOff, NULL, NULL)) return OWGS_EINVAL;
    int64_t* pao = jcopy_in(env, aOff, (jlong)n + 1, 8, 'J');
    int64_t* pbo = jcopy_in(env, bOff, (jlong)n + 1, 8, 'J');
    if (!pao || !pbo) {
        FREE_ALL(pao, pbo);
        return OWGS_ENOMEM;
    }
    if (pao[n] > (*env)->GetArrayLength(env, a) || pbo[n] > (*env)->GetArrayLength(env, b)) {
        FREE_ALL(pao, pbo);
        return OWGS_EINVAL;
    }
    char* pa = jcopy_in(env, a, (*env)->GetArrayLength(env, a), 1, 'B');
    char* pb = jcopy_in(env, b, (*env)->GetArrayLength(env, b), 1, 'B');
    int32_t first = 0;
    int rc = OWGS_ENOMEM;
    if (pa && pb) rc = owgs_register_templates(CTX(h), n, pa, pao, pb, pbo, &first);
    FREE_ALL(pao, pbo, pa, pb);
    return rc == OWGS_OK ? first : rc;
}

/* returns the number of messages (>= 0) or an OWGS_E* code; out must hold the batch's bytes (size query: out = null) */
JNIEXPORT jlong JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_serializeActivations(
    JNIEnv* env, jobject self, jlong h, jintArray invoker, jintArray tmpl, jlongArray aid, jbyteArray tid,
    jlongArray tidOff, jlongArray tidStart, jbyteArray flags, jbyteArray content, jlongArray contentOff, jint n,
    jint nTopics, jbyteArray out, jlongArray outOff, jintArray outOrder, jintArray topicStart) {
    if (!invoker || !tmpl || !aid || !tid || !tidOff || !tidStart || !flags || !outOff || !outOrder || !topicStart ||
        nTopics < 0 || !n_fits(env, n, invoker, tmpl, tidStart, flags) || !n_fits(env, 2LL * n, aid, NULL, NULL, NULL) ||
        !n_fits(env, (jlong)n + 1, tidOff, outOff, NULL, NULL) || !n_fits(env, n, outOrder, NULL, NULL, NULL) ||
        !n_fits(env, (jlong)nTopics + 1, topicStart, NULL, NULL, NULL) ||
        (contentOff && !n_fits(env, (jlong)n + 1, contentOff, NULL, NULL, NULL)))
        return OWGS_EINVAL;
    owgs_msg_batch b;
    memset(&b, 0, sizeof b);
    b.n = n;
    int32_t* pinv = jcopy_in(env, invoker, n, 4, 'I');
    int32_t* ptm = jcopy_in(env, tmpl, n, 4, 'I');
    uint64_t* paid = jcopy_in(env, aid, 2LL * n, 8, 'J');
    char* ptid = jcopy_in(env, tid, (*env)->GetArrayLength(env, tid), 1, 'B');
    int64_t* ptoff = jcopy_in(env, tidOff, (jlong)n + 1, 8, 'J');
    int64_t* ptst = jcopy_in(env, tidStart, n, 8, 'J');
    uint8_t* pfl = jcopy_in(env, flags, n, 1, 'B');
    char* pct = content ? jcopy_in(env, content, (*env)->GetArrayLength(env, content), 1, 'B') : NULL;
    int64_t* pco = contentOff ? jcopy_in(env, contentOff, (jlong)n + 1, 8, 'J') : NULL;
    const jlong cap = out ? (*env)->GetArrayLength(env, out) : 0;
    char* po = cap > 0 ? malloc((size_t)cap) : NULL;
    int64_t* poff = calloc((size_t)n + 1, 8);
    int32_t* pord = calloc((size_t)(n > 0 ? n : 1), 4);
    int32_t* pts = calloc((size_t)nTopics + 1, 4);
    int rc = OWGS_ENOMEM;
    int64_t total = 0;
    int32_t m = 0;
    if (pinv && ptm && paid && ptid && ptoff && ptst && pfl && (pct || !content) && (pco || !contentOff) &&
        (po || cap <= 0) && poff && pord && pts) {
        if (ptoff[n] > (*env)->GetArrayLength(env, tid) ||
            (pco && (!content || pco[n] > (*env)->GetArrayLength(env, content)))) {
            rc = OWGS_EINVAL;
        } else {
            b.invoker = pinv;
            b.tmpl = ptm;
            b.aid = paid;
            b.tid = ptid;
            b.tid_off = ptoff;
            b.tid_start = ptst;
            b.flags = pfl;
            b.content = pct;
            b.content_off = pco;
            rc = owgs_serialize_activations(CTX(h), &b, nTopics, po, cap, poff, pord, pts, &total, &m);
        }
    }
    if (rc == OWGS_OK) {
        jcopy_out(env, out, total, po, 'B');
        jcopy_out(env, outOff, (jlong)n + 1, poff, 'J');
        jcopy_out(env, outOrder, n, pord, 'I');
        jcopy_out(env, topicStart, (jlong)nTopics + 1, pts, 'I');
    }
    FREE_ALL(pinv, ptm, paid, ptid, ptoff, ptst, pfl, pct, pco, po, poff, pord, pts);
    return rc == OWGS_OK ? (jlong)m : (jlong)rc;
}

JNIEXPORT jstring JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_lastError(JNIEnv* env,
                                                                                               jobject self, jlong h) {
    return (*env)->NewStringUTF(env, owgs_last_error(CTX(h)));
}
