/*
 * owgs_jni.c -- JNI binding of include/owgs.h for integration/GpuShardingContainerPoolBalancer.scala
 * (SOURCE ONLY: this image has no JDK, so no jni.h; build on a controller host with
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I<repo>/include owgs_jni.c \
 *       -L<repo>/openwhisk_amd -lowgs -o libowgs_jni.so ).
 * Arrays are pinned with Get/ReleasePrimitiveArrayCritical for the duration of one batch call; the native context is
 * single-writer (the shim's batching thread), as owgs.h requires.
 */
#include <jni.h>
#include <stdlib.h>
#include <string.h>

#include "owgs.h"

#define CTX(h) ((owgs_ctx*)(intptr_t)(h))

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
    const jsize n = (*env)->GetArrayLength(env, ids);
    if (!n_fits(env, n, mem, status, NULL, NULL)) return OWGS_EINVAL;
    jint* pi = (*env)->GetPrimitiveArrayCritical(env, ids, NULL);
    jlong* pm = (*env)->GetPrimitiveArrayCritical(env, mem, NULL);
    jbyte* ps = (*env)->GetPrimitiveArrayCritical(env, status, NULL);
    const int rc = owgs_update_invokers(CTX(h), n, (const int32_t*)pi, (const int64_t*)pm, (const uint8_t*)ps);
    (*env)->ReleasePrimitiveArrayCritical(env, status, ps, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, mem, pm, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, ids, pi, JNI_ABORT);
    return rc;
}

JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_updateCluster(JNIEnv* env,
                                                                                                jobject self, jlong h,
                                                                                                jint size) {
    return owgs_update_cluster(CTX(h), size);
}

JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_registerAction(
    JNIEnv* env, jobject self, jlong h, jstring ns, jstring path, jstring key, jint mem, jint maxc, jboolean bb) {
    const char* s0 = (*env)->GetStringUTFChars(env, ns, NULL);
    const char* s1 = (*env)->GetStringUTFChars(env, path, NULL);
    const char* s2 = (*env)->GetStringUTFChars(env, key, NULL);
    const int32_t o0[2] = {0, (int32_t)strlen(s0)}, o1[2] = {0, (int32_t)strlen(s1)}, o2[2] = {0, (int32_t)strlen(s2)};
    const int32_t m = mem, c = maxc;
    const uint8_t b = bb ? 1 : 0;
    int32_t action = -1;
    const int rc = owgs_register_actions(CTX(h), 1, s0, o0, s1, o1, s2, o2, &m, &c, &b, &action, NULL);
    (*env)->ReleaseStringUTFChars(env, key, s2);
    (*env)->ReleaseStringUTFChars(env, path, s1);
    (*env)->ReleaseStringUTFChars(env, ns, s0);
    return rc == OWGS_OK ? action : rc;
}

/* n must not exceed any array: bound it by every length (a short array would be read / written past its end) */
static int n_fits(JNIEnv* env, jint n, jarray a, jarray b, jarray c, jarray d) {
    jarray xs[4] = {a, b, c, d};
    if (n < 0) return 0;
    for (int i = 0; i < 4; ++i)
        if (xs[i] && (*env)->GetArrayLength(env, xs[i]) < n) return 0;
    return 1;
}

JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_publishBatch(
    JNIEnv* env, jobject self, jlong h, jintArray actions, jlongArray seq, jint n, jintArray out, jbyteArray flags) {
    if (!n_fits(env, n, actions, seq, out, flags)) return OWGS_EINVAL;
    jint* pa = (*env)->GetPrimitiveArrayCritical(env, actions, NULL);
    jlong* ps = (*env)->GetPrimitiveArrayCritical(env, seq, NULL);
    jint* po = (*env)->GetPrimitiveArrayCritical(env, out, NULL);
    jbyte* pf = (*env)->GetPrimitiveArrayCritical(env, flags, NULL);
    const int rc = owgs_publish_batch(CTX(h), n, (const int32_t*)pa, (const uint64_t*)ps, 0, (int32_t*)po, (uint8_t*)pf);
    (*env)->ReleasePrimitiveArrayCritical(env, flags, pf, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, out, po, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, seq, ps, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, actions, pa, JNI_ABORT);
    return rc;
}

JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_releaseBatch(
    JNIEnv* env, jobject self, jlong h, jintArray invokers, jintArray actions, jint n, jbyteArray flags) {
    if (!n_fits(env, n, invokers, actions, flags, NULL)) return OWGS_EINVAL;
    jint* pi = (*env)->GetPrimitiveArrayCritical(env, invokers, NULL);
    jint* pa = (*env)->GetPrimitiveArrayCritical(env, actions, NULL);
    jbyte* pf = (*env)->GetPrimitiveArrayCritical(env, flags, NULL);
    const int rc = owgs_release_batch(CTX(h), n, (const int32_t*)pi, (const int32_t*)pa, (uint8_t*)pf);
    (*env)->ReleasePrimitiveArrayCritical(env, flags, pf, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, actions, pa, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, invokers, pi, JNI_ABORT);
    return rc;
}

/* ---- completion path (CommonLoadBalancer.setupActivation / processAcknowledgement / processCompletion) ---- */
JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_trackActivations(
    JNIEnv* env, jobject self, jlong h, jbyteArray aid32, jintArray actions, jintArray tickets, jint n,
    jintArray outTicket, jbyteArray outExisted) {
    if (!n_fits(env, n, actions, tickets, outTicket, outExisted) || (*env)->GetArrayLength(env, aid32) < 32LL * n)
        return OWGS_EINVAL;
    jbyte* pa = (*env)->GetPrimitiveArrayCritical(env, aid32, NULL);
    jint* pc = (*env)->GetPrimitiveArrayCritical(env, actions, NULL);
    jint* pt = (*env)->GetPrimitiveArrayCritical(env, tickets, NULL);
    jint* po = (*env)->GetPrimitiveArrayCritical(env, outTicket, NULL);
    jbyte* pe = (*env)->GetPrimitiveArrayCritical(env, outExisted, NULL);
    const int rc = owgs_track_activations(CTX(h), n, (const char*)pa, (const int32_t*)pc, (const int32_t*)pt,
                                          (int32_t*)po, (uint8_t*)pe);
    (*env)->ReleasePrimitiveArrayCritical(env, outExisted, pe, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, outTicket, po, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, tickets, pt, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, actions, pc, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, aid32, pa, JNI_ABORT);
    return rc;
}

/* raw ack bytes of one feed batch (MessageFeed hands the consumer's records over as Array[Byte], LB:94-108) */
JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_processAcks(
    JNIEnv* env, jobject self, jlong h, jbyteArray bytes, jlongArray off, jint n, jbyteArray outKind,
    jintArray outInvoker, jintArray outTicket, jbyteArray outFlags) {
    if (!n_fits(env, n, outKind, outInvoker, outTicket, outFlags) || (*env)->GetArrayLength(env, off) < n + 1)
        return OWGS_EINVAL;
    jbyte* pb = (*env)->GetPrimitiveArrayCritical(env, bytes, NULL);
    jlong* po = (*env)->GetPrimitiveArrayCritical(env, off, NULL);
    jbyte* pk = (*env)->GetPrimitiveArrayCritical(env, outKind, NULL);
    jint* pi = (*env)->GetPrimitiveArrayCritical(env, outInvoker, NULL);
    jint* pt = (*env)->GetPrimitiveArrayCritical(env, outTicket, NULL);
    jbyte* pf = (*env)->GetPrimitiveArrayCritical(env, outFlags, NULL);
    const int rc = owgs_process_acks(CTX(h), n, (const char*)pb, (const int64_t*)po, (uint8_t*)pk, (int32_t*)pi,
                                     (int32_t*)pt, (uint8_t*)pf);
    (*env)->ReleasePrimitiveArrayCritical(env, outFlags, pf, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, outTicket, pt, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, outInvoker, pi, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, outKind, pk, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, off, po, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, bytes, pb, JNI_ABORT);
    return rc;
}

JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_completeActivations(
    JNIEnv* env, jobject self, jlong h, jbyteArray aid32, jintArray invokers, jbyteArray flags, jint n,
    jbyteArray outKind, jintArray outTicket, jbyteArray outFlags) {
    if (!n_fits(env, n, invokers, flags, outKind, outTicket) || !n_fits(env, n, outFlags, NULL, NULL, NULL) ||
        (*env)->GetArrayLength(env, aid32) < 32LL * n)
        return OWGS_EINVAL;
    jbyte* pa = (*env)->GetPrimitiveArrayCritical(env, aid32, NULL);
    jint* pi = (*env)->GetPrimitiveArrayCritical(env, invokers, NULL);
    jbyte* pc = (*env)->GetPrimitiveArrayCritical(env, flags, NULL);
    jbyte* pk = (*env)->GetPrimitiveArrayCritical(env, outKind, NULL);
    jint* pt = (*env)->GetPrimitiveArrayCritical(env, outTicket, NULL);
    jbyte* pf = (*env)->GetPrimitiveArrayCritical(env, outFlags, NULL);
    const int rc = owgs_complete_activations(CTX(h), n, (const char*)pa, (const int32_t*)pi, (const uint8_t*)pc,
                                             (uint8_t*)pk, (int32_t*)pt, (uint8_t*)pf);
    (*env)->ReleasePrimitiveArrayCritical(env, outFlags, pf, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, outTicket, pt, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, outKind, pk, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, flags, pc, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, invokers, pi, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, aid32, pa, JNI_ABORT);
    return rc;
}

/* ---- invoker health supervision (InvokerPool + InvokerActor) ---- */
JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_healthEvents(
    JNIEnv* env, jobject self, jlong h, jintArray invokers, jbyteArray kinds, jlongArray tMs, jlongArray userMemory,
    jint n, jlong nowMs, jboolean apply) {
    if (!n_fits(env, n, invokers, kinds, tMs, userMemory)) return OWGS_EINVAL;
    jint* pi = (*env)->GetPrimitiveArrayCritical(env, invokers, NULL);
    jbyte* pk = (*env)->GetPrimitiveArrayCritical(env, kinds, NULL);
    jlong* pt = (*env)->GetPrimitiveArrayCritical(env, tMs, NULL);
    jlong* pm = (*env)->GetPrimitiveArrayCritical(env, userMemory, NULL);
    const int rc = owgs_health_events(CTX(h), n, (const int32_t*)pi, (const uint8_t*)pk, (const int64_t*)pt,
                                      (const int64_t*)pm, nowMs, apply ? 1 : 0);
    (*env)->ReleasePrimitiveArrayCritical(env, userMemory, pm, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, tMs, pt, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, kinds, pk, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, invokers, pi, JNI_ABORT);
    return rc;
}

/* status vector + test actions to send (the shim sends one health test action per count, InvokerPool.ActivationRequest) */
JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_healthRead(
    JNIEnv* env, jobject self, jlong h, jint cap, jbyteArray status, jlongArray userMemory, jintArray tests) {
    int32_t n = 0;
    jbyte* ps = (*env)->GetPrimitiveArrayCritical(env, status, NULL);
    jlong* pm = (*env)->GetPrimitiveArrayCritical(env, userMemory, NULL);
    jint* pt = (*env)->GetPrimitiveArrayCritical(env, tests, NULL);
    const int rc = owgs_health_read(CTX(h), cap, &n, (uint8_t*)ps, (int64_t*)pm, (int32_t*)pt, NULL, NULL);
    (*env)->ReleasePrimitiveArrayCritical(env, tests, pt, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, userMemory, pm, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, status, ps, 0);
    return rc == OWGS_OK ? n : rc;
}

/* ---- ActivationMessage serialisation + topic fan-out ---- */
JNIEXPORT jint JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_registerTemplates(
    JNIEnv* env, jobject self, jlong h, jbyteArray a, jlongArray aOff, jbyteArray b, jlongArray bOff, jint n) {
    int32_t first = 0;
    jbyte* pa = (*env)->GetPrimitiveArrayCritical(env, a, NULL);
    jlong* pao = (*env)->GetPrimitiveArrayCritical(env, aOff, NULL);
    jbyte* pb = (*env)->GetPrimitiveArrayCritical(env, b, NULL);
    jlong* pbo = (*env)->GetPrimitiveArrayCritical(env, bOff, NULL);
    const int rc = owgs_register_templates(CTX(h), n, (const char*)pa, (const int64_t*)pao, (const char*)pb,
                                           (const int64_t*)pbo, &first);
    (*env)->ReleasePrimitiveArrayCritical(env, bOff, pbo, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, b, pb, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, aOff, pao, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, a, pa, JNI_ABORT);
    return rc == OWGS_OK ? first : rc;
}

/* returns the number of messages (>= 0) or an OWGS_E* code; out must hold the batch's bytes (size query: out = null) */
JNIEXPORT jlong JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_serializeActivations(
    JNIEnv* env, jobject self, jlong h, jintArray invoker, jintArray tmpl, jlongArray aid, jbyteArray tid,
    jlongArray tidOff, jlongArray tidStart, jbyteArray flags, jbyteArray content, jlongArray contentOff, jint n,
    jint nTopics, jbyteArray out, jlongArray outOff, jintArray outOrder, jintArray topicStart) {
    owgs_msg_batch b;
    memset(&b, 0, sizeof b);
    b.n = n;
    b.invoker = (*env)->GetPrimitiveArrayCritical(env, invoker, NULL);
    b.tmpl = (*env)->GetPrimitiveArrayCritical(env, tmpl, NULL);
    b.aid = (*env)->GetPrimitiveArrayCritical(env, aid, NULL);
    b.tid = (*env)->GetPrimitiveArrayCritical(env, tid, NULL);
    b.tid_off = (*env)->GetPrimitiveArrayCritical(env, tidOff, NULL);
    b.tid_start = (*env)->GetPrimitiveArrayCritical(env, tidStart, NULL);
    b.flags = (*env)->GetPrimitiveArrayCritical(env, flags, NULL);
    b.content = content ? (*env)->GetPrimitiveArrayCritical(env, content, NULL) : NULL;
    b.content_off = contentOff ? (*env)->GetPrimitiveArrayCritical(env, contentOff, NULL) : NULL;
    const jsize cap = out ? (*env)->GetArrayLength(env, out) : 0;
    jbyte* po = out ? (*env)->GetPrimitiveArrayCritical(env, out, NULL) : NULL;
    jlong* poff = (*env)->GetPrimitiveArrayCritical(env, outOff, NULL);
    jint* pord = (*env)->GetPrimitiveArrayCritical(env, outOrder, NULL);
    jint* pts = (*env)->GetPrimitiveArrayCritical(env, topicStart, NULL);
    int64_t total = 0;
    int32_t m = 0;
    const int rc = owgs_serialize_activations(CTX(h), &b, nTopics, (char*)po, cap, (int64_t*)poff, (int32_t*)pord,
                                              (int32_t*)pts, &total, &m);
    (*env)->ReleasePrimitiveArrayCritical(env, topicStart, pts, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, outOrder, pord, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, outOff, poff, 0);
    if (po) (*env)->ReleasePrimitiveArrayCritical(env, out, po, 0);
    if (b.content_off) (*env)->ReleasePrimitiveArrayCritical(env, contentOff, (void*)b.content_off, JNI_ABORT);
    if (b.content) (*env)->ReleasePrimitiveArrayCritical(env, content, (void*)b.content, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, flags, (void*)b.flags, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, tidStart, (void*)b.tid_start, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, tidOff, (void*)b.tid_off, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, tid, (void*)b.tid, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, aid, (void*)b.aid, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, tmpl, (void*)b.tmpl, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, invoker, (void*)b.invoker, JNI_ABORT);
    return rc == OWGS_OK ? (jlong)m : (jlong)rc;
}

JNIEXPORT jstring JNICALL Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_lastError(JNIEnv* env,
                                                                                               jobject self, jlong h) {
    return (*env)->NewStringUTF(env, owgs_last_error(CTX(h)));
}
