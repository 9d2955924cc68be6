/*
 * jni_harness.c -- executes integration/owgs_jni.c without a JVM (this image has no JDK).
 *
 * A JNIEnv whose function table implements exactly the JNI functions owgs_jni.c calls, over stand-in Java objects:
 * int[] / long[] / byte[] arrays, Strings (modified UTF-8 bytes) and direct ByteBuffers (an address and a capacity;
 * GetDirectBufferAddress returns NULL and GetDirectBufferCapacity -1 for anything else, as the JNI specification says).
 * Region accesses outside an array are counted (a JVM would raise ArrayIndexOutOfBoundsException) instead of performed.
 * The h_* functions below are what tests/test_gpu_jni.py calls through ctypes: they wrap host buffers (numpy arrays,
 * no copy) as Java objects and call the Java_..._OwgsNative_00024_* entry points with this environment, so the test
 * drives the binding exactly as the Scala shim's native methods would -- including the direct-buffer layout of
 * BatchBuffers (integration/GpuShardingContainerPoolBalancer.scala) that processBatch reads.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { K_INTS = 1, K_LONGS, K_BYTES, K_STRING, K_DIRECT };
typedef struct {
    int kind;
    jsize len;  /* elements (arrays) or bytes (strings) */
    void* data;
    jlong cap;  /* direct buffers */
} fake_obj;

static long g_oob = 0;        /* region accesses outside an array */
static long g_strings = 0;    /* GetStringUTFChars without ReleaseStringUTFChars */

static fake_obj* O(jobject o) { return (fake_obj*)o; }
static int in_range(jarray a, jsize start, jsize len) {
    if (!a || start < 0 || len < 0 || (jlong)start + len > O(a)->len) {
        ++g_oob;
        return 0;
    }
    return 1;
}

static jsize GetArrayLength(JNIEnv* e, jarray a) {
    (void)e;
    return a ? O(a)->len : 0;
}
#define REGION(NAME, T, KIND, DIR)                                                          \
    static void NAME(JNIEnv* e, jarray a, jsize start, jsize len, DIR T* buf) {             \
        (void)e;                                                                            \
        if (!in_range(a, start, len) || O(a)->kind != KIND) return;                         \
        GETSET(T)                                                                           \
    }
#define GETSET(T) memcpy(buf, (T*)O(a)->data + start, (size_t)len * sizeof(T));
REGION(GetIntArrayRegion, jint, K_INTS, )
REGION(GetLongArrayRegion, jlong, K_LONGS, )
REGION(GetByteArrayRegion, jbyte, K_BYTES, )
#undef GETSET
#define GETSET(T) memcpy((T*)O(a)->data + start, buf, (size_t)len * sizeof(T));
REGION(SetIntArrayRegion, jint, K_INTS, const)
REGION(SetLongArrayRegion, jlong, K_LONGS, const)
REGION(SetByteArrayRegion, jbyte, K_BYTES, const)
#undef GETSET

static const char* GetStringUTFChars(JNIEnv* e, jstring s, jboolean* is_copy) {
    (void)e;
    if (!s || O(s)->kind != K_STRING) return NULL;
    char* p = malloc((size_t)O(s)->len + 1);
    if (!p) return NULL;
    memcpy(p, O(s)->data, (size_t)O(s)->len);
    p[O(s)->len] = 0;
    if (is_copy) *is_copy = 1;
    ++g_strings;
    return p;
}
static void ReleaseStringUTFChars(JNIEnv* e, jstring s, const char* p) {
    (void)e;
    (void)s;
    free((void*)p);
    --g_strings;
}
static fake_obj g_last_string;  /* NewStringUTF: one result at a time (lastError) */
static char g_last_text[1024];
static jstring NewStringUTF(JNIEnv* e, const char* t) {
    (void)e;
    strncpy(g_last_text, t ? t : "", sizeof g_last_text - 1);
    g_last_string.kind = K_STRING;
    g_last_string.len = (jsize)strlen(g_last_text);
    g_last_string.data = g_last_text;
    return (jstring)&g_last_string;
}
static void* GetDirectBufferAddress(JNIEnv* e, jobject b) {
    (void)e;
    return (b && O(b)->kind == K_DIRECT) ? O(b)->data : NULL;
}
static jlong GetDirectBufferCapacity(JNIEnv* e, jobject b) {
    (void)e;
    return (b && O(b)->kind == K_DIRECT) ? O(b)->cap : -1;
}

static const struct JNINativeInterface_ g_table = {
    GetArrayLength,     GetIntArrayRegion,     GetLongArrayRegion, GetByteArrayRegion,     SetIntArrayRegion,
    SetLongArrayRegion, SetByteArrayRegion,    GetStringUTFChars,  ReleaseStringUTFChars,  NewStringUTF,
    GetDirectBufferAddress, GetDirectBufferCapacity,
};
static JNIEnv g_env = &g_table;

/* ---- the binding's entry points (integration/owgs_jni.c) ---- */
#define JN(name) Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_##name
jlong JN(create)(JNIEnv*, jobject, jdouble, jdouble, jlong, jint, jint, jlong);
void JN(destroy)(JNIEnv*, jobject, jlong);
jint JN(updateInvokers)(JNIEnv*, jobject, jlong, jintArray, jlongArray, jbyteArray);
jint JN(updateCluster)(JNIEnv*, jobject, jlong, jint);
jint JN(registerAction)(JNIEnv*, jobject, jlong, jstring, jstring, jstring, jint, jint, jboolean);
jint JN(processBatch)(JNIEnv*, jobject, jlong, jobject, jobject, jint, jint, jint, jlong);
jint JN(releaseActions)(JNIEnv*, jobject, jlong, jintArray, jint);
jint JN(publishBatch)(JNIEnv*, jobject, jlong, jintArray, jlongArray, jint, jintArray, jbyteArray);
jint JN(releaseBatch)(JNIEnv*, jobject, jlong, jintArray, jintArray, jint, jbyteArray);
jstring JN(lastError)(JNIEnv*, jobject, jlong);

/* ---- ctypes surface ---- */
#define HX __attribute__((visibility("default")))
HX void* h_obj(int kind, void* data, int64_t len) {  /* kind 1 int[], 2 long[], 3 byte[], 4 String, 5 direct buffer */
    fake_obj* o = calloc(1, sizeof *o);
    if (!o) return NULL;
    o->kind = kind;
    o->data = data;
    o->len = kind == K_DIRECT ? 0 : (jsize)len;
    o->cap = kind == K_DIRECT ? (jlong)len : 0;
    return o;
}
HX void h_free(void* o) { free(o); }
HX long h_oob(void) { return g_oob; }
HX long h_strings_held(void) { return g_strings; }

HX int64_t h_create(double mf, double bf, int64_t min_mem, int32_t cluster, int32_t device, int64_t seed) {
    return JN(create)(&g_env, NULL, mf, bf, min_mem, cluster, device, seed);
}
HX void h_destroy(int64_t h) { JN(destroy)(&g_env, NULL, h); }
HX int32_t h_update_invokers(int64_t h, void* ids, void* mem, void* status) {
    return JN(updateInvokers)(&g_env, NULL, h, ids, mem, status);
}
HX int32_t h_update_cluster(int64_t h, int32_t n) { return JN(updateCluster)(&g_env, NULL, h, n); }
HX int32_t h_register_action(int64_t h, void* ns, void* path, void* key, int32_t mem, int32_t maxc, int32_t bb) {
    return JN(registerAction)(&g_env, NULL, h, ns, path, key, mem, maxc, (jboolean)(bb != 0));
}
HX int32_t h_process_batch(int64_t h, void* in, void* out, int32_t n_runs, int32_t n_rel, int32_t n_pub,
                           int64_t seq_base) {
    return JN(processBatch)(&g_env, NULL, h, in, out, n_runs, n_rel, n_pub, seq_base);
}
HX int32_t h_release_actions(int64_t h, void* handles, int32_t n) {
    return JN(releaseActions)(&g_env, NULL, h, handles, n);
}
HX int32_t h_publish_batch(int64_t h, void* actions, void* seq, int32_t n, void* out, void* flags) {
    return JN(publishBatch)(&g_env, NULL, h, actions, seq, n, out, flags);
}
HX int32_t h_release_batch(int64_t h, void* invokers, void* actions, int32_t n, void* flags) {
    return JN(releaseBatch)(&g_env, NULL, h, invokers, actions, n, flags);
}
HX const char* h_last_error(int64_t h) {
    jstring s = JN(lastError)(&g_env, NULL, h);
    return s ? (const char*)O(s)->data : "";
}
