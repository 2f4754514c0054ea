/*
 * harness.c -- TEST INFRASTRUCTURE: drives the JNI shim (java-rsync_amd/jni/rsync_hip_jni.c) without a JVM.
 *
 * No JDK exists in this image or on the GPU box, so the shim is compiled against tests/jni/jni.h (a test
 * double with the JDK's names) and linked into libjniharness.so together with this file, which implements
 * the JNIEnv functions over plain C objects and exports jh_* entry points for ctypes
 * (tests/test_jni_shim.py).  Arrays and direct buffers wrap caller memory; a "heap" buffer has no address
 * (GetDirectBufferAddress returns NULL, as for a JVM heap ByteBuffer); a thrown exception is recorded by
 * class name and read back with jh_exception().  Array region calls are bounds-checked like the JVM's
 * (ArrayIndexOutOfBoundsException) so that a shim that over-reads or over-writes a Java array shows up.
 */
#include <jni.h>
#include <stdlib.h>
#include <string.h>

#include "rsync_hip.h"

enum { K_DIRECT = 1, K_HEAP, K_INT, K_BYTE, K_LONG, K_OBJS, K_STR, K_CLASS };
struct _jobject {
    int kind;
    void* data;
    jlong len; /* elements (arrays), capacity (buffers) */
};
typedef struct _jobject fobj;

static __thread char g_exc[256];
static __thread char g_msg[256];

static jclass f_FindClass(JNIEnv* env, const char* name) {
    (void)env;
    static __thread fobj cls;
    static __thread char nm[256];
    strncpy(nm, name, sizeof(nm) - 1);
    cls.kind = K_CLASS;
    cls.data = nm;
    return &cls;
}
static jint f_ThrowNew(JNIEnv* env, jclass c, const char* msg) {
    (void)env;
    if (!g_exc[0]) { /* the first exception stays pending, as in a JVM */
        strncpy(g_exc, (const char*)c->data, sizeof(g_exc) - 1);
        strncpy(g_msg, msg ? msg : "", sizeof(g_msg) - 1);
    }
    return 0;
}
static void f_DeleteLocalRef(JNIEnv* env, jobject o) {
    (void)env;
    (void)o;
}
static void* f_GetDirectBufferAddress(JNIEnv* env, jobject b) {
    (void)env;
    return b && b->kind == K_DIRECT ? b->data : NULL;
}
static jlong f_GetDirectBufferCapacity(JNIEnv* env, jobject b) {
    (void)env;
    return b && b->kind == K_DIRECT ? b->len : -1;
}
static jsize f_GetArrayLength(JNIEnv* env, jarray a) {
    (void)env;
    return (jsize)a->len;
}
static jobject f_GetObjectArrayElement(JNIEnv* env, jobjectArray a, jsize i) {
    (void)env;
    return ((jobject*)a->data)[i];
}
static int in_bounds(jarray a, jsize start, jsize len) {
    if (start < 0 || len < 0 || (jlong)start + len > a->len) {
        f_ThrowNew(NULL, f_FindClass(NULL, "java/lang/ArrayIndexOutOfBoundsException"), "region");
        return 0;
    }
    return 1;
}
static void f_GetIntArrayRegion(JNIEnv* env, jintArray a, jsize s, jsize l, jint* buf) {
    (void)env;
    if (in_bounds(a, s, l)) memcpy(buf, (jint*)a->data + s, (size_t)l * 4);
}
static void f_SetIntArrayRegion(JNIEnv* env, jintArray a, jsize s, jsize l, const jint* buf) {
    (void)env;
    if (in_bounds(a, s, l)) memcpy((jint*)a->data + s, buf, (size_t)l * 4);
}
static void f_GetByteArrayRegion(JNIEnv* env, jbyteArray a, jsize s, jsize l, jbyte* buf) {
    (void)env;
    if (in_bounds(a, s, l)) memcpy(buf, (jbyte*)a->data + s, (size_t)l);
}
static void f_SetByteArrayRegion(JNIEnv* env, jbyteArray a, jsize s, jsize l, const jbyte* buf) {
    (void)env;
    if (in_bounds(a, s, l)) memcpy((jbyte*)a->data + s, buf, (size_t)l);
}
static void f_SetLongArrayRegion(JNIEnv* env, jlongArray a, jsize s, jsize l, const jlong* buf) {
    (void)env;
    if (in_bounds(a, s, l)) memcpy((jlong*)a->data + s, buf, (size_t)l * 8);
}
static void f_GetLongArrayRegion(JNIEnv* env, jlongArray a, jsize s, jsize l, jlong* buf) {
    (void)env;
    if (in_bounds(a, s, l)) memcpy(buf, (jlong*)a->data + s, (size_t)l * 8);
}
static jlongArray f_NewLongArray(JNIEnv* env, jsize len) {
    (void)env;
    fobj* o = (fobj*)calloc(1, sizeof(fobj));
    o->kind = K_LONG;
    o->len = len;
    o->data = calloc((size_t)(len > 0 ? len : 1), 8);
    return o;
}
static jlong* f_GetLongArrayElements(JNIEnv* env, jlongArray a, jboolean* c) {
    (void)env;
    if (c) *c = 0;
    return (jlong*)a->data;
}
static void f_ReleaseLongArrayElements(JNIEnv* env, jlongArray a, jlong* e, jint mode) {
    (void)env;
    (void)a;
    (void)e;
    (void)mode;
}
static const char* f_GetStringUTFChars(JNIEnv* env, jstring s, jboolean* c) {
    (void)env;
    if (c) *c = 0;
    return (const char*)s->data;
}
static void f_ReleaseStringUTFChars(JNIEnv* env, jstring s, const char* p) {
    (void)env;
    (void)s;
    (void)p;
}

static const struct JNINativeInterface_ g_fns = {
    f_FindClass, f_ThrowNew, f_DeleteLocalRef, f_GetDirectBufferAddress, f_GetDirectBufferCapacity, f_GetArrayLength,
    f_GetObjectArrayElement, f_GetIntArrayRegion, f_SetIntArrayRegion, f_GetByteArrayRegion, f_SetByteArrayRegion,
    f_SetLongArrayRegion, f_NewLongArray, f_GetLongArrayElements, f_ReleaseLongArrayElements, f_GetStringUTFChars,
    f_ReleaseStringUTFChars, f_GetLongArrayRegion,
};
static JNIEnv g_env = &g_fns;

/* the shim's natives (rsync_hip_jni.c) */
#define NC(name) Java_com_github_java_rsync_internal_session_NativeChecksum_##name
jlong NC(ctxCreate)(JNIEnv*, jclass, jint);
void NC(ctxDestroy)(JNIEnv*, jclass, jlong);
void NC(blockSums)(JNIEnv*, jclass, jlong, jobject, jlong, jintArray, jbyteArray, jintArray, jbyteArray);
void NC(blockSumsBuffers)(JNIEnv*, jclass, jlong, jobjectArray, jlong, jintArray, jbyteArray, jintArray, jbyteArray);
jlongArray NC(matchScan)(JNIEnv*, jclass, jlong, jobject, jlong, jintArray, jintArray, jbyteArray, jbyteArray,
                         jbyteArray, jlongArray);
jlongArray NC(matchScanBuffers)(JNIEnv*, jclass, jlong, jobjectArray, jlong, jintArray, jintArray, jbyteArray,
                                jbyteArray, jbyteArray, jlongArray);
void NC(blockSumsBatch)(JNIEnv*, jclass, jlong, jobjectArray, jintArray, jlongArray, jintArray, jbyteArray,
                        jobjectArray, jobjectArray);
jlongArray NC(matchScanBatch)(JNIEnv*, jclass, jlong, jobjectArray, jintArray, jlongArray, jintArray, jobjectArray,
                              jobjectArray, jbyteArray, jbyteArray, jlongArray);
void NC(blockSumsBatchMulti)(JNIEnv*, jclass, jlongArray, jobjectArray, jintArray, jlongArray, jintArray, jbyteArray,
                             jobjectArray, jobjectArray);
jlongArray NC(matchScanBatchMulti)(JNIEnv*, jclass, jlongArray, jobjectArray, jintArray, jlongArray, jintArray,
                                   jobjectArray, jobjectArray, jbyteArray, jbyteArray, jlongArray);
jboolean NC(receiverCombine)(JNIEnv*, jclass, jlong, jobject, jlong, jintArray, jobject, jlong, jboolean, jobject, jlong,
                             jlongArray, jbyteArray);

/* fake objects: cap < 0 = a heap buffer (no address); NULL data with len < 0 = a Java null */
#define OBJ(name, k, ptr, n) fobj name##_o = {k, (void*)(ptr), (n)}; jobject name = (n) < 0 && !(ptr) ? NULL : &name##_o
#define BUF(name, ptr, cap) fobj name##_o = {(cap) < 0 ? K_HEAP : K_DIRECT, (void*)(ptr), (cap)}; \
    jobject name = (ptr) || (cap) >= 0 ? &name##_o : NULL

static void reset(void) {
    g_exc[0] = 0;
    g_msg[0] = 0;
}

/* jh_set_multi(ctxs, n): the segment entry points below call the Multi natives (NativeChecksum's device set) with
 * these contexts as the long[] instead of the single context (n = 0: back to the single-context natives). */
static jlong g_multi[64];
static int g_nmulti = 0;
JNIEXPORT void jh_set_multi(const jlong* ctxs, int n) {
    g_nmulti = n < 0 ? 0 : n > 64 ? 64 : n;
    if (g_nmulti) memcpy(g_multi, ctxs, (size_t)g_nmulti * sizeof(jlong));
}

JNIEXPORT const char* jh_exception(void) { return g_exc; }
JNIEXPORT const char* jh_exception_message(void) { return g_msg; }

JNIEXPORT jlong jh_ctx_create(int device) {
    reset();
    return NC(ctxCreate)(&g_env, NULL, device);
}
JNIEXPORT void jh_ctx_destroy(jlong ctx) {
    reset();
    NC(ctxDestroy)(&g_env, NULL, ctx);
}

JNIEXPORT void jh_block_sums(jlong ctx, void* buf, jlong cap, jlong n, int32_t* hdr4, uint8_t* seed, jlong seed_len,
                             int32_t* weak, jlong weak_len, uint8_t* strong, jlong strong_len) {
    reset();
    BUF(b, buf, cap);
    OBJ(h, K_INT, hdr4, 4);
    OBJ(s, K_BYTE, seed, seed_len);
    OBJ(w, K_INT, weak, weak_len);
    OBJ(st, K_BYTE, strong, strong_len);
    NC(blockSums)(&g_env, NULL, ctx, b, n, h, s, w, st);
}

/* bufs[i] with caps[i] (< 0: heap buffer) */
static jobjectArray buffers(fobj* store, jobject* refs, void** bufs, const jlong* caps, int nb) {
    for (int i = 0; i < nb; ++i) {
        store[i].kind = caps[i] < 0 ? K_HEAP : K_DIRECT;
        store[i].data = bufs[i];
        store[i].len = caps[i];
        refs[i] = &store[i];
    }
    return NULL;
}

JNIEXPORT void jh_block_sums_buffers(jlong ctx, void** bufs, const jlong* caps, int nb, jlong n, int32_t* hdr4,
                                     uint8_t* seed, jlong seed_len, int32_t* weak, jlong weak_len, uint8_t* strong,
                                     jlong strong_len) {
    reset();
    fobj* store = (fobj*)calloc((size_t)nb + 1, sizeof(fobj));
    jobject* refs = (jobject*)calloc((size_t)nb + 1, sizeof(jobject));
    buffers(store, refs, bufs, caps, nb);
    fobj arr = {K_OBJS, refs, nb};
    OBJ(h, K_INT, hdr4, 4);
    OBJ(s, K_BYTE, seed, seed_len);
    OBJ(w, K_INT, weak, weak_len);
    OBJ(st, K_BYTE, strong, strong_len);
    NC(blockSumsBuffers)(&g_env, NULL, ctx, &arr, n, h, s, w, st);
    free(refs);
    free(store);
}

/* Copies the returned event longs into ev_out (up to ev_cap) and returns their count; -1 when the shim
 * returned null (an exception is then pending). */
static jlong events_back(jlongArray out, jlong* ev_out, jlong ev_cap) {
    if (!out) return -1;
    const jlong k = out->len < ev_cap ? out->len : ev_cap;
    if (k > 0) memcpy(ev_out, out->data, (size_t)k * 8);
    const jlong len = out->len;
    free(out->data);
    free(out);
    return len;
}

JNIEXPORT jlong jh_match_scan(jlong ctx, void* buf, jlong cap, jlong n, int32_t* hdr4, int32_t* weak, jlong weak_len,
                              uint8_t* strong, jlong strong_len, uint8_t* seed, jlong seed_len, uint8_t* md5,
                              jlong md5_len, jlong* sizes, jlong sizes_len, jlong* ev_out, jlong ev_cap) {
    reset();
    BUF(b, buf, cap);
    OBJ(h, K_INT, hdr4, 4);
    OBJ(w, K_INT, weak, weak_len);
    OBJ(st, K_BYTE, strong, strong_len);
    OBJ(s, K_BYTE, seed, seed_len);
    OBJ(m, K_BYTE, md5, md5_len);
    OBJ(z, K_LONG, sizes, sizes_len);
    return events_back(NC(matchScan)(&g_env, NULL, ctx, b, n, h, w, st, s, m, z), ev_out, ev_cap);
}

JNIEXPORT jlong jh_match_scan_buffers(jlong ctx, void** bufs, const jlong* caps, int nb, jlong n, int32_t* hdr4,
                                      int32_t* weak, jlong weak_len, uint8_t* strong, jlong strong_len, uint8_t* seed,
                                      jlong seed_len, uint8_t* md5, jlong md5_len, jlong* sizes, jlong sizes_len,
                                      jlong* ev_out, jlong ev_cap) {
    reset();
    fobj* store = (fobj*)calloc((size_t)nb + 1, sizeof(fobj));
    jobject* refs = (jobject*)calloc((size_t)nb + 1, sizeof(jobject));
    buffers(store, refs, bufs, caps, nb);
    fobj arr = {K_OBJS, refs, nb};
    OBJ(h, K_INT, hdr4, 4);
    OBJ(w, K_INT, weak, weak_len);
    OBJ(st, K_BYTE, strong, strong_len);
    OBJ(s, K_BYTE, seed, seed_len);
    OBJ(m, K_BYTE, md5, md5_len);
    OBJ(z, K_LONG, sizes, sizes_len);
    jlong r = events_back(NC(matchScanBuffers)(&g_env, NULL, ctx, &arr, n, h, w, st, s, m, z), ev_out, ev_cap);
    free(refs);
    free(store);
    return r;
}

JNIEXPORT int jh_receiver_combine(jlong ctx, void* tokens, jlong tok_cap, jlong tokens_len, int32_t* hdr4,
                                  void* replica, jlong rep_cap, jlong replica_len, int defer, void* target,
                                  jlong tgt_cap, jlong target_cap, jlong* result, uint8_t* md5) {
    reset();
    BUF(t, tokens, tok_cap);
    BUF(r, replica, rep_cap);
    BUF(o, target, tgt_cap);
    OBJ(h, K_INT, hdr4, 4);
    OBJ(res, K_LONG, result, 4);
    OBJ(m, K_BYTE, md5, 16);
    return NC(receiverCombine)(&g_env, NULL, ctx, t, tokens_len, h, r, replica_len, (jboolean)defer, o, target_cap,
                               res, m);
}

/* A segment (blockSumsBatch / matchScanBatch): nb buffers, nf files of file_pieces[f] buffers each; the per-file
 * Java arrays (int[][] / byte[][]) are arrs[f] with lens[f] elements (lens[f] < 0 with a NULL pointer: a Java
 * null element). */
static jobjectArray objs_of(fobj* store, jobject* refs, int kind, void** arrs, const jlong* lens, int n) {
    for (int i = 0; i < n; ++i) {
        store[i].kind = kind;
        store[i].data = arrs[i];
        store[i].len = lens[i];
        refs[i] = (lens[i] < 0 && !arrs[i]) ? NULL : &store[i];
    }
    return NULL;
}

JNIEXPORT void jh_block_sums_batch(jlong ctx, void** bufs, const jlong* caps, int nb, int32_t* file_pieces, int nf,
                                   jlong* sizes, int32_t* hdrs, uint8_t* seed, void** weak, const jlong* weak_lens,
                                   void** strong, const jlong* strong_lens) {
    reset();
    fobj* store = (fobj*)calloc((size_t)nb + 1, sizeof(fobj));
    jobject* refs = (jobject*)calloc((size_t)nb + 1, sizeof(jobject));
    buffers(store, refs, bufs, caps, nb);
    fobj arr = {K_OBJS, refs, nb};
    fobj* ws = (fobj*)calloc((size_t)nf + 1, sizeof(fobj));
    jobject* wr = (jobject*)calloc((size_t)nf + 1, sizeof(jobject));
    fobj* ss = (fobj*)calloc((size_t)nf + 1, sizeof(fobj));
    jobject* sr = (jobject*)calloc((size_t)nf + 1, sizeof(jobject));
    objs_of(ws, wr, K_INT, weak, weak_lens, nf);
    objs_of(ss, sr, K_BYTE, strong, strong_lens, nf);
    fobj wa = {K_OBJS, wr, nf}, sa = {K_OBJS, sr, nf};
    OBJ(fp, K_INT, file_pieces, nf);
    OBJ(sz, K_LONG, sizes, nf);
    OBJ(h, K_INT, hdrs, 4 * nf);
    OBJ(s, K_BYTE, seed, 4);
    fobj cs_o = {K_LONG, g_multi, g_nmulti};
    jobject cs = &cs_o;
    if (g_nmulti) NC(blockSumsBatchMulti)(&g_env, NULL, cs, &arr, fp, sz, h, s, &wa, &sa);
    else NC(blockSumsBatch)(&g_env, NULL, ctx, &arr, fp, sz, h, s, &wa, &sa);
    free(refs);
    free(store);
    free(ws);
    free(wr);
    free(ss);
    free(sr);
}

JNIEXPORT jlong jh_match_scan_batch(jlong ctx, void** bufs, const jlong* caps, int nb, int32_t* file_pieces, int nf,
                                    jlong* sizes, int32_t* hdrs, void** weak, const jlong* weak_lens, void** strong,
                                    const jlong* strong_lens, uint8_t* seed, uint8_t* md5, jlong md5_len,
                                    jlong* per_file, jlong per_len, jlong* ev_out, jlong ev_cap) {
    reset();
    fobj* store = (fobj*)calloc((size_t)nb + 1, sizeof(fobj));
    jobject* refs = (jobject*)calloc((size_t)nb + 1, sizeof(jobject));
    buffers(store, refs, bufs, caps, nb);
    fobj arr = {K_OBJS, refs, nb};
    fobj* ws = (fobj*)calloc((size_t)nf + 1, sizeof(fobj));
    jobject* wr = (jobject*)calloc((size_t)nf + 1, sizeof(jobject));
    fobj* ss = (fobj*)calloc((size_t)nf + 1, sizeof(fobj));
    jobject* sr = (jobject*)calloc((size_t)nf + 1, sizeof(jobject));
    objs_of(ws, wr, K_INT, weak, weak_lens, nf);
    objs_of(ss, sr, K_BYTE, strong, strong_lens, nf);
    fobj wa = {K_OBJS, wr, nf}, sa = {K_OBJS, sr, nf};
    OBJ(fp, K_INT, file_pieces, nf);
    OBJ(sz, K_LONG, sizes, nf);
    OBJ(h, K_INT, hdrs, 4 * nf);
    OBJ(s, K_BYTE, seed, 4);
    OBJ(m, K_BYTE, md5, md5_len);
    OBJ(pf, K_LONG, per_file, per_len);
    fobj cs_o = {K_LONG, g_multi, g_nmulti};
    jobject cs = &cs_o;
    jlongArray o = g_nmulti ? NC(matchScanBatchMulti)(&g_env, NULL, cs, &arr, fp, sz, h, &wa, &sa, s, m, pf)
                            : NC(matchScanBatch)(&g_env, NULL, ctx, &arr, fp, sz, h, &wa, &sa, s, m, pf);
    jlong r = events_back(o, ev_out, ev_cap);
    free(refs);
    free(store);
    free(ws);
    free(wr);
    free(ss);
    free(sr);
    return r;
}
