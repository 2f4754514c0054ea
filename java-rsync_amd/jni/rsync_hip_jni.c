/*
 * rsync_hip_jni.c -- JNI shim between java-rsync's core (Generator / Sender) and librsynchip.so.
 *
 * Binds the native methods of com.github.java.rsync.internal.session.NativeChecksum (source next to
 * this file; INTEGRATION.md shows the call sites it replaces).  Thin by design: it pins the Java
 * arrays / direct buffers, calls the C-ABI of include/rsync_hip.h and maps status codes onto the
 * exceptions the reference already throws:
 *   RSH_E_PROTOCOL -> com.github.java.rsync.RsyncProtocolException   (Connection.java:28-38)
 *   RSH_E_OVERFLOW -> ...internal.session.Checksum$ChunkOverflow     (Checksum.java:58-64,107-111)
 *   RSH_E_INVAL    -> java.lang.IllegalArgumentException
 *   RSH_E_NOMEM    -> java.lang.OutOfMemoryError
 *   RSH_E_BUSY     -> java.lang.IllegalStateException (a context shared across threads; use forThread())
 *   RSH_E_DEVICE   -> java.lang.IllegalStateException (caller falls back to the Java path only if it
 *                     chose to; the library itself never falls back)
 *   RSH_E_NOTFOUND -> ...internal.io.FileViewNotFound                (FileView.java:74-75)
 *   RSH_E_OPEN     -> ...internal.io.FileViewOpenFailed              (FileView.java:76-78)
 * A closed context (handle 0) is an IllegalStateException; a byte count larger than the direct buffer it
 * names is an IllegalArgumentException -- the library is never handed memory the buffer does not own.
 *
 * Three ways to hand over the file bytes:
 *   blockSums / matchScan              one direct ByteBuffer (files < 2 GiB: a buffer's capacity is an int);
 *   blockSumsBuffers / matchScanBuffers  an array of direct ByteBuffers, the file being their concatenation
 *                                      (any size; FileView streams any file, FileView.java:235-278);
 *   blockSumsFile / matchScanFile      a path: the library reads the file with FileView's semantics and
 *                                      reports a read error as a flag (the FileViewException of close());
 *   blockSumsBatch / matchScanBatch    a whole file-list segment in one call (Generator.itemizeSegment,
 *                                      Sender.sendFiles): every file's pieces, header and table at once;
 *   blockSumsBatchMulti / matchScanBatchMulti  the same over the calling thread's contexts on the node's GPUs
 *                                      (rsh_*_batch_multi: the segment's files split over them).
 * The Sender replays the returned events through its own sendDataFrom/putInt so channel framing is
 * untouched (Sender.java:794-809); INTEGRATION.md shows the replay for each form.
 *
 * Build (needs a JDK): make -C java-rsync_amd jni JAVA_HOME=/path/to/jdk
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include "rsync_hip.h"

static void throw_class(JNIEnv* env, const char* cls, const char* msg) {
    jclass c = (*env)->FindClass(env, cls);
    if (!c) return; /* NoClassDefFoundError already pending */
    (*env)->ThrowNew(env, c, msg);
}

static void throw_status(JNIEnv* env, int rc) {
    const char* cls;
    switch (rc) {
        case RSH_E_PROTOCOL: cls = "com/github/java/rsync/RsyncProtocolException"; break;
        case RSH_E_OVERFLOW: cls = "com/github/java/rsync/internal/session/Checksum$ChunkOverflow"; break;
        case RSH_E_INVAL: cls = "java/lang/IllegalArgumentException"; break;
        case RSH_E_NOMEM: cls = "java/lang/OutOfMemoryError"; break;
        case RSH_E_NOTFOUND: cls = "com/github/java/rsync/internal/io/FileViewNotFound"; break;
        case RSH_E_OPEN: cls = "com/github/java/rsync/internal/io/FileViewOpenFailed"; break;
        default: cls = "java/lang/IllegalStateException"; break;
    }
    throw_class(env, cls, rsh_strerror(rc));
}

/* The context of a live NativeChecksum; throws IllegalStateException for a closed one (handle 0). */
static rsh_ctx* ctx_of(JNIEnv* env, jlong ctx) {
    if (ctx == 0) throw_class(env, "java/lang/IllegalStateException", "NativeChecksum context is closed");
    return (rsh_ctx*)(intptr_t)ctx;
}

/* The contexts of a NativeChecksum device set (long[] of live handles, one per GPU): malloc'd array (free it), or
 * NULL with IllegalStateException (a closed context) / IllegalArgumentException (empty) thrown. */
static rsh_ctx** ctxs_of(JNIEnv* env, jlongArray hs, jint* n) {
    *n = hs ? (*env)->GetArrayLength(env, hs) : 0;
    if (*n < 1) {
        throw_class(env, "java/lang/IllegalArgumentException", "no NativeChecksum contexts");
        return NULL;
    }
    jlong* v = (jlong*)malloc(sizeof(jlong) * (size_t)*n);
    rsh_ctx** out = (rsh_ctx**)malloc(sizeof(rsh_ctx*) * (size_t)*n);
    if (!v || !out) {
        free(v);
        free(out);
        throw_status(env, RSH_E_NOMEM);
        return NULL;
    }
    (*env)->GetLongArrayRegion(env, hs, 0, *n, v);
    for (jint i = 0; i < *n; ++i) {
        if (!ctx_of(env, v[i])) {
            free(v);
            free(out);
            return NULL;
        }
        out[i] = (rsh_ctx*)(intptr_t)v[i];
    }
    free(v);
    return out;
}

/* The address of a direct buffer that holds at least `need` bytes; NULL (IllegalArgumentException thrown)
 * for a heap buffer, a negative count or a count past the buffer's capacity. */
static const uint8_t* direct_bytes(JNIEnv* env, jobject buf, jlong need) {
    if (!buf || need < 0) {
        throw_status(env, RSH_E_INVAL);
        return NULL;
    }
    const uint8_t* p = (const uint8_t*)(*env)->GetDirectBufferAddress(env, buf);
    const jlong cap = (*env)->GetDirectBufferCapacity(env, buf);
    if (!p || cap < need) {
        throw_class(env, "java/lang/IllegalArgumentException",
                    p ? "byte count exceeds the direct buffer's capacity" : "not a direct ByteBuffer");
        return NULL;
    }
    return p;
}

/* The pieces of a file handed over as ByteBuffer[]: every buffer's whole capacity in order, the last one
 * cut at n.  Returns the piece count (0 for n == 0), or -1 with IllegalArgumentException thrown when a
 * buffer is not direct or the buffers hold fewer than n bytes.  *out is malloc'd (free it). */
static jint pieces_from(JNIEnv* env, jobjectArray bufs, jlong n, rsh_piece** out) {
    *out = NULL;
    const jsize nb = bufs ? (*env)->GetArrayLength(env, bufs) : 0;
    if (n < 0 || (n > 0 && nb == 0)) {
        throw_status(env, RSH_E_INVAL);
        return -1;
    }
    rsh_piece* p = (rsh_piece*)malloc(sizeof(rsh_piece) * (size_t)(nb > 0 ? nb : 1));
    if (!p) {
        throw_status(env, RSH_E_NOMEM);
        return -1;
    }
    jlong left = n;
    jint k = 0;
    for (jsize i = 0; i < nb && left > 0; ++i) {
        jobject b = (*env)->GetObjectArrayElement(env, bufs, i);
        const uint8_t* a = b ? (const uint8_t*)(*env)->GetDirectBufferAddress(env, b) : NULL;
        const jlong cap = b ? (*env)->GetDirectBufferCapacity(env, b) : -1;
        if (b) (*env)->DeleteLocalRef(env, b);
        if (!a || cap < 0) {
            free(p);
            throw_class(env, "java/lang/IllegalArgumentException", "piece is not a direct ByteBuffer");
            return -1;
        }
        p[k].data = a;
        p[k].len = cap < left ? cap : left;
        left -= p[k].len;
        ++k;
    }
    if (left > 0) {
        free(p);
        throw_class(env, "java/lang/IllegalArgumentException", "the buffers hold fewer bytes than the file size");
        return -1;
    }
    *out = p;
    return k;
}

static int header_from(JNIEnv* env, jintArray hdr4, rsh_header* h) {
    if (!hdr4 || (*env)->GetArrayLength(env, hdr4) != 4) return RSH_E_INVAL;
    jint v[4];
    (*env)->GetIntArrayRegion(env, hdr4, 0, 4, v);
    h->chunk_count = v[0];   /* wire order of Connection.sendChecksumHeader (Connection.java:40-45) */
    h->block_length = v[1];
    h->digest_length = v[2];
    h->remainder = v[3];
    return RSH_OK;
}

static int seed_from(JNIEnv* env, jbyteArray seed, jbyte s4[4]) {
    if (!seed || (*env)->GetArrayLength(env, seed) != 4) return RSH_E_INVAL;
    (*env)->GetByteArrayRegion(env, seed, 0, 4, s4);
    return RSH_OK;
}

/* Generator outputs: weakOut[chunkCount], strongOut[chunkCount * digestLength]. */
static int sums_out_ok(JNIEnv* env, const rsh_header* h, jintArray weakOut, jbyteArray strongOut) {
    if (!weakOut || !strongOut || h->chunk_count < 0 || h->digest_length < 0) return RSH_E_INVAL;
    if ((*env)->GetArrayLength(env, weakOut) < h->chunk_count ||
        (*env)->GetArrayLength(env, strongOut) < (jlong)h->chunk_count * h->digest_length)
        return RSH_E_INVAL;
    return RSH_OK;
}

typedef int (*sums_fn)(rsh_ctx* c, const void* src, const rsh_header* h, const uint8_t* seed, int32_t* w,
                       uint8_t* st, void* arg);

/* Runs a Generator pass into native buffers (the call can run for seconds: no JNI critical region, which
 * would stall the GC) and copies the sums into the Java arrays. */
static void run_sums(JNIEnv* env, rsh_ctx* c, const void* src, const rsh_header* h, const jbyte* s4, jintArray weakOut,
                     jbyteArray strongOut, sums_fn fn, void* arg) {
    const size_t C = (size_t)h->chunk_count, dl = (size_t)h->digest_length;
    int32_t* w = (int32_t*)malloc(C * 4 + 4);
    uint8_t* st = (uint8_t*)malloc(C * dl + 1);
    int rc = (w && st) ? fn(c, src, h, (const uint8_t*)s4, w, st, arg) : RSH_E_NOMEM;
    if (rc == RSH_OK) {
        (*env)->SetIntArrayRegion(env, weakOut, 0, (jsize)C, (const jint*)w);
        (*env)->SetByteArrayRegion(env, strongOut, 0, (jsize)(C * dl), (const jbyte*)st);
    }
    free(st);
    free(w);
    if (rc != RSH_OK) throw_status(env, rc);
}

/* Events as a flat long[] of 4-tuples {kind, offset, length, index | (count << 32)}. */
static jlongArray events_to_java(JNIEnv* env, const rsh_event* ev, int64_t n_ev) {
    jlongArray out = (*env)->NewLongArray(env, (jsize)(4 * n_ev));
    if (!out) return NULL;
    jlong* o = (*env)->GetLongArrayElements(env, out, NULL);
    if (!o) return NULL;
    for (int64_t i = 0; i < n_ev; ++i) {
        o[4 * i + 0] = ev[i].kind;
        o[4 * i + 1] = ev[i].offset;
        o[4 * i + 2] = ev[i].length;
        o[4 * i + 3] = (jlong)(uint32_t)ev[i].index | ((jlong)ev[i].count << 32);
    }
    (*env)->ReleaseLongArrayElements(env, out, o, 0);
    return out;
}

typedef int (*scan_fn)(rsh_ctx* c, const void* src, const rsh_header* h, const int32_t* w, const uint8_t* st,
                       const uint8_t* seed, rsh_event* ev, int64_t cap, int64_t* n_ev, uint8_t md5[16], int64_t* lit,
                       int64_t* mat, void* arg);

/* Runs a Sender pass: copies the (small) received table out of the Java arrays (no critical region across
 * a long scan), sizes the event buffer, fetches the events again on RSH_E_NOSPACE (the context kept them:
 * not a rescan).  Returns the events, or NULL with an exception pending. */
static jlongArray run_scan(JNIEnv* env, rsh_ctx* c, const void* src, jlong n, const rsh_header* h, jintArray weak,
                           jbyteArray strong, const jbyte* s4, uint8_t md5[16], int64_t* lit, int64_t* mat, scan_fn fn,
                           void* arg) {
    /* one literal per flush interval plus a literal and a match run per chunk */
    int64_t cap = (n / (10 * (int64_t)(h->block_length > 0 ? h->block_length : 8192))) +
                  2 * (int64_t)(h->chunk_count > 0 ? h->chunk_count : 0) + 64;
    int64_t n_ev = 0;
    const jsize nw = weak ? (*env)->GetArrayLength(env, weak) : 0;
    const jsize ns = strong ? (*env)->GetArrayLength(env, strong) : 0;
    int rc = RSH_OK;
    if (h->chunk_count > 0 && (nw < h->chunk_count || (jlong)ns < (jlong)h->chunk_count * h->digest_length))
        rc = RSH_E_INVAL; /* received table shorter than its header says */
    rsh_event* ev = (rsh_event*)malloc((size_t)cap * sizeof(rsh_event));
    int32_t* w = (int32_t*)malloc((size_t)nw * 4 + 4);
    uint8_t* st = (uint8_t*)malloc((size_t)ns + 1);
    if (rc == RSH_OK && (!ev || !w || !st)) rc = RSH_E_NOMEM;
    if (rc == RSH_OK) {
        if (nw) (*env)->GetIntArrayRegion(env, weak, 0, nw, (jint*)w);
        if (ns) (*env)->GetByteArrayRegion(env, strong, 0, ns, (jbyte*)st);
        rc = fn(c, src, h, nw ? w : NULL, ns ? st : NULL, (const uint8_t*)s4, ev, cap, &n_ev, md5, lit, mat, arg);
        if (rc == RSH_E_NOSPACE) {
            rsh_event* grown = (rsh_event*)realloc(ev, (size_t)n_ev * sizeof(rsh_event));
            if (!grown) rc = RSH_E_NOMEM;
            else {
                ev = grown;
                rc = rsh_fetch_events(c, ev, n_ev, &n_ev);
            }
        }
    }
    free(st);
    free(w);
    jlongArray out = NULL;
    if (rc == RSH_OK) out = events_to_java(env, ev, n_ev);
    else throw_status(env, rc);
    free(ev);
    return out;
}

static void sizes_out(JNIEnv* env, jlongArray sizesOut, jbyteArray fileMd5Out, const uint8_t md5[16], jlong lit,
                      jlong mat, int with_error, jlong read_error) {
    jlong sizes[3] = {lit, mat, read_error};
    (*env)->SetByteArrayRegion(env, fileMd5Out, 0, 16, (const jbyte*)md5);
    (*env)->SetLongArrayRegion(env, sizesOut, 0, with_error ? 3 : 2, sizes);
}

static int scan_args_ok(JNIEnv* env, jintArray hdr4, rsh_header* h, jbyteArray seed, jbyte s4[4],
                        jbyteArray fileMd5Out, jlongArray sizesOut, jsize nsizes) {
    if (header_from(env, hdr4, h) != RSH_OK || seed_from(env, seed, s4) != RSH_OK || !fileMd5Out || !sizesOut ||
        (*env)->GetArrayLength(env, fileMd5Out) != 16 || (*env)->GetArrayLength(env, sizesOut) < nsizes)
        return RSH_E_INVAL;
    return RSH_OK;
}

JNIEXPORT jlong JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_ctxCreate(JNIEnv* env, jclass cls,
                                                                                           jint device) {
    (void)cls;
    rsh_ctx* ctx = NULL;
    int rc = rsh_ctx_create(device, &ctx);
    if (rc != RSH_OK) {
        throw_status(env, rc);
        return 0;
    }
    return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_ctxDestroy(JNIEnv* env, jclass cls,
                                                                                           jlong ctx) {
    (void)env;
    (void)cls;
    rsh_ctx_destroy((rsh_ctx*)(intptr_t)ctx); /* NULL is a no-op */
}

/* rsh_ctx_trim: the pass-sized buffers back to the allocators (throws on a device error). */
JNIEXPORT void JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_ctxTrim(JNIEnv* env, jclass cls,
                                                                                        jlong ctx) {
    (void)cls;
    const int rc = rsh_ctx_trim((rsh_ctx*)(intptr_t)ctx);
    if (rc != RSH_OK) throw_status(env, rc);
}

/* Generator.getBlockLengthFor / getDigestLength (Generator.java:198-212, :873). */
JNIEXPORT jint JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_blockLengthFor(JNIEnv* env, jclass c,
                                                                                               jlong size) {
    (void)env;
    (void)c;
    return rsh_block_length_for(size);
}

JNIEXPORT jint JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_digestLengthFor(
    JNIEnv* env, jclass c, jlong size, jint blen, jint min_dl) {
    (void)env;
    (void)c;
    return rsh_digest_length_for(size, blen, min_dl);
}

/* ---- Generator.sendItemizeAndChecksums hot loop (Generator.java:886-895) ---- */

static int sums_buffer(rsh_ctx* c, const void* src, const rsh_header* h, const uint8_t* seed, int32_t* w, uint8_t* st,
                       void* arg) {
    return rsh_block_sums(c, (const uint8_t*)src, *(const jlong*)arg, h, seed, w, st);
}

/* data: a direct ByteBuffer holding the whole basis file (n <= its capacity). */
JNIEXPORT void JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_blockSums(
    JNIEnv* env, jclass cls, jlong ctx, jobject data, jlong n, jintArray hdr4, jbyteArray seed, jintArray weakOut,
    jbyteArray strongOut) {
    (void)cls;
    rsh_ctx* c = ctx_of(env, ctx);
    if (!c) return;
    rsh_header h;
    jbyte s4[4];
    if (header_from(env, hdr4, &h) != RSH_OK || seed_from(env, seed, s4) != RSH_OK ||
        sums_out_ok(env, &h, weakOut, strongOut) != RSH_OK) {
        throw_status(env, RSH_E_INVAL);
        return;
    }
    const uint8_t* p = direct_bytes(env, data, n);
    if (!p) return;
    run_sums(env, c, p, &h, s4, weakOut, strongOut, sums_buffer, &n);
}

static int sums_pieces(rsh_ctx* c, const void* src, const rsh_header* h, const uint8_t* seed, int32_t* w,
                       uint8_t* st, void* arg) {
    return rsh_block_sums_pieces(c, (const rsh_piece*)src, *(const jint*)arg, h, seed, w, st);
}

/* As blockSums over the concatenation of direct ByteBuffers (each full to its capacity but the last). */
JNIEXPORT void JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_blockSumsBuffers(
    JNIEnv* env, jclass cls, jlong ctx, jobjectArray data, jlong n, jintArray hdr4, jbyteArray seed, jintArray weakOut,
    jbyteArray strongOut) {
    (void)cls;
    rsh_ctx* c = ctx_of(env, ctx);
    if (!c) return;
    rsh_header h;
    jbyte s4[4];
    if (header_from(env, hdr4, &h) != RSH_OK || seed_from(env, seed, s4) != RSH_OK ||
        sums_out_ok(env, &h, weakOut, strongOut) != RSH_OK) {
        throw_status(env, RSH_E_INVAL);
        return;
    }
    rsh_piece* pieces;
    jint np = pieces_from(env, data, n, &pieces);
    if (np < 0) return;
    run_sums(env, c, pieces, &h, s4, weakOut, strongOut, sums_pieces, &np);
    free(pieces);
}

/* ---- Sender.sendMatchesAndData / skipMatchSendData (Sender.java:1235-1327, 1386-1399) ----
 * Return the events as {kind, offset, length, index | (count << 32)} quadruples; fileMd5Out[16] receives
 * the whole-file digest and sizesOut = {sizeLiteral, sizeMatch[, readError]}. */

static int scan_buffer(rsh_ctx* c, const void* src, const rsh_header* h, const int32_t* w, const uint8_t* st,
                       const uint8_t* seed, rsh_event* ev, int64_t cap, int64_t* n_ev, uint8_t md5[16], int64_t* lit,
                       int64_t* mat, void* arg) {
    return rsh_match_scan(c, (const uint8_t*)src, *(const jlong*)arg, h, w, st, seed, ev, cap, n_ev, md5, lit, mat,
                          NULL);
}

JNIEXPORT jlongArray JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_matchScan(
    JNIEnv* env, jclass cls, jlong ctx, jobject src, jlong n, jintArray hdr4, jintArray weak, jbyteArray strong,
    jbyteArray seed, jbyteArray fileMd5Out, jlongArray sizesOut) {
    (void)cls;
    rsh_ctx* c = ctx_of(env, ctx);
    if (!c) return NULL;
    rsh_header h;
    jbyte s4[4];
    if (scan_args_ok(env, hdr4, &h, seed, s4, fileMd5Out, sizesOut, 2) != RSH_OK) {
        throw_status(env, RSH_E_INVAL);
        return NULL;
    }
    const uint8_t* p = direct_bytes(env, src, n);
    if (!p) return NULL;
    uint8_t md5[16];
    int64_t lit = 0, mat = 0;
    jlongArray out = run_scan(env, c, p, n, &h, weak, strong, s4, md5, &lit, &mat, scan_buffer, &n);
    if (out) sizes_out(env, sizesOut, fileMd5Out, md5, lit, mat, 0, 0);
    return out;
}

static int scan_pieces(rsh_ctx* c, const void* src, const rsh_header* h, const int32_t* w, const uint8_t* st,
                       const uint8_t* seed, rsh_event* ev, int64_t cap, int64_t* n_ev, uint8_t md5[16], int64_t* lit,
                       int64_t* mat, void* arg) {
    return rsh_match_scan_pieces(c, (const rsh_piece*)src, *(const jint*)arg, h, w, st, seed, ev, cap, n_ev, md5, lit,
                                 mat, NULL);
}

/* As matchScan over the concatenation of direct ByteBuffers: the source of any size.  The caller replays a
 * LIT(offset, length) event from the same buffers (sendDataFrom over ByteBuffer[]). */
JNIEXPORT jlongArray JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_matchScanBuffers(
    JNIEnv* env, jclass cls, jlong ctx, jobjectArray src, jlong n, jintArray hdr4, jintArray weak, jbyteArray strong,
    jbyteArray seed, jbyteArray fileMd5Out, jlongArray sizesOut) {
    (void)cls;
    rsh_ctx* c = ctx_of(env, ctx);
    if (!c) return NULL;
    rsh_header h;
    jbyte s4[4];
    if (scan_args_ok(env, hdr4, &h, seed, s4, fileMd5Out, sizesOut, 2) != RSH_OK) {
        throw_status(env, RSH_E_INVAL);
        return NULL;
    }
    rsh_piece* pieces;
    jint np = pieces_from(env, src, n, &pieces);
    if (np < 0) return NULL;
    uint8_t md5[16];
    int64_t lit = 0, mat = 0;
    jlongArray out = run_scan(env, c, pieces, n, &h, weak, strong, s4, md5, &lit, &mat, scan_pieces, &np);
    free(pieces);
    if (out) sizes_out(env, sizesOut, fileMd5Out, md5, lit, mat, 0, 0);
    return out;
}

/* ---- the same passes reading the file natively (rsh_*_file: FileView.java:51-80,187-278 semantics) ---- */

typedef struct {
    jlong size;
    int32_t read_error;
} file_arg;

static int sums_file(rsh_ctx* c, const void* src, const rsh_header* h, const uint8_t* seed, int32_t* w, uint8_t* st,
                     void* arg) {
    file_arg* a = (file_arg*)arg;
    return rsh_block_sums_file(c, (const char*)src, a->size, h, seed, w, st, &a->read_error);
}

/* Returns true when the file could not be read to `size` (zero-filled from there: FileViewException). */
JNIEXPORT jboolean JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_blockSumsFile(
    JNIEnv* env, jclass cls, jlong ctx, jstring path, jlong size, jintArray hdr4, jbyteArray seed, jintArray weakOut,
    jbyteArray strongOut) {
    (void)cls;
    rsh_ctx* c = ctx_of(env, ctx);
    if (!c) return JNI_FALSE;
    rsh_header h;
    jbyte s4[4];
    if (!path || header_from(env, hdr4, &h) != RSH_OK || seed_from(env, seed, s4) != RSH_OK ||
        sums_out_ok(env, &h, weakOut, strongOut) != RSH_OK) {
        throw_status(env, RSH_E_INVAL);
        return JNI_FALSE;
    }
    const char* cpath = (*env)->GetStringUTFChars(env, path, NULL);
    if (!cpath) return JNI_FALSE; /* OutOfMemoryError pending */
    file_arg a = {size, 0};
    run_sums(env, c, cpath, &h, s4, weakOut, strongOut, sums_file, &a);
    (*env)->ReleaseStringUTFChars(env, path, cpath);
    return a.read_error ? JNI_TRUE : JNI_FALSE;
}

static int scan_file(rsh_ctx* c, const void* src, const rsh_header* h, const int32_t* w, const uint8_t* st,
                     const uint8_t* seed, rsh_event* ev, int64_t cap, int64_t* n_ev, uint8_t md5[16], int64_t* lit,
                     int64_t* mat, void* arg) {
    file_arg* a = (file_arg*)arg;
    return rsh_match_scan_file(c, (const char*)src, a->size, h, w, st, seed, ev, cap, n_ev, md5, lit, mat, NULL,
                               &a->read_error);
}

/* As matchScan, reading the source natively; sizesOut[3] = {sizeLiteral, sizeMatch, readError}.  The caller
 * replays a LIT(offset, length) event with positional reads of the same file. */
JNIEXPORT jlongArray JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_matchScanFile(
    JNIEnv* env, jclass cls, jlong ctx, jstring path, jlong size, jintArray hdr4, jintArray weak, jbyteArray strong,
    jbyteArray seed, jbyteArray fileMd5Out, jlongArray sizesOut) {
    (void)cls;
    rsh_ctx* c = ctx_of(env, ctx);
    if (!c) return NULL;
    rsh_header h;
    jbyte s4[4];
    if (!path || scan_args_ok(env, hdr4, &h, seed, s4, fileMd5Out, sizesOut, 3) != RSH_OK) {
        throw_status(env, RSH_E_INVAL);
        return NULL;
    }
    const char* cpath = (*env)->GetStringUTFChars(env, path, NULL);
    if (!cpath) return NULL;
    uint8_t md5[16];
    int64_t lit = 0, mat = 0;
    file_arg a = {size, 0};
    jlongArray out = run_scan(env, c, cpath, size, &h, weak, strong, s4, md5, &lit, &mat, scan_file, &a);
    (*env)->ReleaseStringUTFChars(env, path, cpath);
    if (out) sizes_out(env, sizesOut, fileMd5Out, md5, lit, mat, 1, a.read_error);
    return out;
}

/* ---- a segment's files in one call (rsh_block_sums_batch / rsh_match_scan_batch) ----
 * Generator.itemizeSegment (Generator.java:558-614) and Sender.sendFiles (Sender.java:1098-1148) walk a
 * segment's files one by one; these natives take them all: data holds every file's direct buffers in file order,
 * filePieces[f] of them for file f (each full to its capacity but the file's last, which is cut at sizes[f]),
 * hdrs four ints per file in Connection.sendChecksumHeader order.  A failing file throws its exception, naming
 * the file; the reference would have thrown it from that file's call. */

typedef struct {
    rsh_piece* pieces; /* all files' pieces */
    int32_t* first;    /* file f: pieces[first[f] .. first[f] + count[f]) */
    int32_t* count;
    rsh_header* h;
    jint nf;
} segment_args;

static void segment_free(segment_args* a) {
    free(a->pieces);
    free(a->first);
    free(a->count);
    free(a->h);
}

/* Splits `bufs` into the files' piece lists and reads their headers; RSH_OK, or an exception thrown. */
static int segment_from(JNIEnv* env, jobjectArray bufs, jintArray filePieces, jlongArray sizes, jintArray hdrs,
                        segment_args* a) {
    memset(a, 0, sizeof(*a));
    const jsize nb = bufs ? (*env)->GetArrayLength(env, bufs) : 0;
    const jint nf = filePieces ? (*env)->GetArrayLength(env, filePieces) : -1;
    if (nf < 0 || !sizes || !hdrs || (*env)->GetArrayLength(env, sizes) < nf ||
        (*env)->GetArrayLength(env, hdrs) < 4 * (jlong)nf) {
        throw_status(env, RSH_E_INVAL);
        return RSH_E_INVAL;
    }
    a->nf = nf;
    a->pieces = (rsh_piece*)malloc(sizeof(rsh_piece) * (size_t)(nb + 1));
    a->first = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nf + 1));
    a->count = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nf + 1));
    a->h = (rsh_header*)malloc(sizeof(rsh_header) * (size_t)(nf + 1));
    jint* fp = (jint*)malloc(sizeof(jint) * (size_t)(nf + 1));
    jlong* sz = (jlong*)malloc(sizeof(jlong) * (size_t)(nf + 1));
    jint* hv = (jint*)malloc(sizeof(jint) * (size_t)(4 * nf + 1));
    int rc = (a->pieces && a->first && a->count && a->h && fp && sz && hv) ? RSH_OK : RSH_E_NOMEM;
    if (rc == RSH_OK && nf > 0) {
        (*env)->GetIntArrayRegion(env, filePieces, 0, nf, fp);
        (*env)->GetLongArrayRegion(env, sizes, 0, nf, sz);
        (*env)->GetIntArrayRegion(env, hdrs, 0, 4 * nf, hv);
    }
    const char* why = NULL;
    jsize b = 0;
    for (jint f = 0; rc == RSH_OK && f < nf; ++f) {
        a->h[f].chunk_count = hv[4 * f];
        a->h[f].block_length = hv[4 * f + 1];
        a->h[f].digest_length = hv[4 * f + 2];
        a->h[f].remainder = hv[4 * f + 3];
        if (fp[f] < 0 || sz[f] < 0 || (jlong)b + fp[f] > nb) {
            rc = RSH_E_INVAL;
            why = "file piece counts or sizes do not match the buffers";
            break;
        }
        a->first[f] = (int32_t)b;
        a->count[f] = 0;
        jlong left = sz[f];
        for (jint k = 0; k < fp[f]; ++k, ++b) {
            jobject o = (*env)->GetObjectArrayElement(env, bufs, b);
            const uint8_t* p = o ? (const uint8_t*)(*env)->GetDirectBufferAddress(env, o) : NULL;
            const jlong cap = o ? (*env)->GetDirectBufferCapacity(env, o) : -1;
            if (o) (*env)->DeleteLocalRef(env, o);
            if (!p || cap < 0) {
                rc = RSH_E_INVAL;
                why = "piece is not a direct ByteBuffer";
                break;
            }
            rsh_piece* pc = &a->pieces[a->first[f] + a->count[f]++];
            pc->data = p;
            pc->len = cap < left ? cap : left;
            left -= pc->len;
        }
        if (rc == RSH_OK && left > 0) {
            rc = RSH_E_INVAL;
            why = "a file's buffers hold fewer bytes than its size";
        }
    }
    free(fp);
    free(sz);
    free(hv);
    if (rc != RSH_OK) {
        segment_free(a);
        if (why) throw_class(env, "java/lang/IllegalArgumentException", why);
        else throw_status(env, rc);
    }
    return rc;
}

/* The exception of file f's status, the message naming the file. */
static void throw_file_status(JNIEnv* env, jint f, int rc) {
    char msg[160];
    snprintf(msg, sizeof(msg), "segment file %d: %s", (int)f, rsh_strerror(rc));
    const char* cls;
    switch (rc) {
        case RSH_E_PROTOCOL: cls = "com/github/java/rsync/RsyncProtocolException"; break;
        case RSH_E_OVERFLOW: cls = "com/github/java/rsync/internal/session/Checksum$ChunkOverflow"; break;
        case RSH_E_INVAL: cls = "java/lang/IllegalArgumentException"; break;
        case RSH_E_NOMEM: cls = "java/lang/OutOfMemoryError"; break;
        default: cls = "java/lang/IllegalStateException"; break;
    }
    throw_class(env, cls, msg);
}

/* weakOut[f] (int[chunkCount]) and strongOut[f] (byte[chunkCount * digestLength]) receive file f's sums. */
/* A segment's Generator pass over nctx contexts (rsh_block_sums_batch_multi; nctx 1: rsh_block_sums_batch). */
static void block_sums_segment(JNIEnv* env, rsh_ctx* const* ctxs, jint nctx, jobjectArray data, jintArray filePieces,
                               jlongArray sizes, jintArray hdrs, jbyteArray seed, jobjectArray weakOut,
                               jobjectArray strongOut) {
    jbyte s4[4];
    if (seed_from(env, seed, s4) != RSH_OK) {
        throw_status(env, RSH_E_INVAL);
        return;
    }
    segment_args a;
    if (segment_from(env, data, filePieces, sizes, hdrs, &a) != RSH_OK) return;
    const jint nf = a.nf;
    int rc = RSH_OK;
    if (!weakOut || !strongOut || (*env)->GetArrayLength(env, weakOut) < nf ||
        (*env)->GetArrayLength(env, strongOut) < nf)
        rc = RSH_E_INVAL;
    rsh_block_batch_job* jobs = (rsh_block_batch_job*)calloc((size_t)nf + 1, sizeof(rsh_block_batch_job));
    jobject* wo = (jobject*)calloc((size_t)nf + 1, sizeof(jobject));
    jobject* so = (jobject*)calloc((size_t)nf + 1, sizeof(jobject));
    if (rc == RSH_OK && (!jobs || !wo || !so)) rc = RSH_E_NOMEM;
    for (jint f = 0; rc == RSH_OK && f < nf; ++f) {
        wo[f] = (*env)->GetObjectArrayElement(env, weakOut, f);
        so[f] = (*env)->GetObjectArrayElement(env, strongOut, f);
        if (sums_out_ok(env, &a.h[f], (jintArray)wo[f], (jbyteArray)so[f]) != RSH_OK) {
            rc = RSH_E_INVAL;
            break;
        }
        const size_t C = (size_t)a.h[f].chunk_count, dl = (size_t)a.h[f].digest_length;
        jobs[f].pieces = a.pieces + a.first[f];
        jobs[f].npieces = a.count[f];
        jobs[f].h = a.h[f];
        jobs[f].weak_out = (int32_t*)malloc(C * 4 + 4);
        jobs[f].strong_out = (uint8_t*)malloc(C * dl + 1);
        if (!jobs[f].weak_out || !jobs[f].strong_out) rc = RSH_E_NOMEM;
    }
    if (rc == RSH_OK) {
        rc = rsh_block_sums_batch_multi(ctxs, nctx, jobs, nf, (const uint8_t*)s4);
        if (rc != RSH_OK) {
            jint f = 0;
            while (f < nf && jobs[f].status == RSH_OK) ++f;
            if (f < nf) throw_file_status(env, f, jobs[f].status);
            else throw_status(env, rc); /* the call failed before any file did: never zero sums as results */
        } else {
            for (jint f = 0; f < nf; ++f) {
                const jsize C = a.h[f].chunk_count;
                (*env)->SetIntArrayRegion(env, (jintArray)wo[f], 0, C, (const jint*)jobs[f].weak_out);
                (*env)->SetByteArrayRegion(env, (jbyteArray)so[f], 0, (jsize)((jlong)C * a.h[f].digest_length),
                                           (const jbyte*)jobs[f].strong_out);
            }
        }
    } else {
        throw_status(env, rc);
    }
    for (jint f = 0; jobs && f < nf; ++f) {
        free(jobs[f].weak_out);
        free(jobs[f].strong_out);
        if (wo && wo[f]) (*env)->DeleteLocalRef(env, wo[f]);
        if (so && so[f]) (*env)->DeleteLocalRef(env, so[f]);
    }
    free(jobs);
    free(wo);
    free(so);
    segment_free(&a);
}

JNIEXPORT void JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_blockSumsBatch(
    JNIEnv* env, jclass cls, jlong ctx, jobjectArray data, jintArray filePieces, jlongArray sizes, jintArray hdrs,
    jbyteArray seed, jobjectArray weakOut, jobjectArray strongOut) {
    (void)cls;
    rsh_ctx* c = ctx_of(env, ctx);
    if (!c) return;
    block_sums_segment(env, &c, 1, data, filePieces, sizes, hdrs, seed, weakOut, strongOut);
}

/* As blockSumsBatch over the thread's contexts on the node's GPUs: the files are split over them (rsh_shard_files). */
JNIEXPORT void JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_blockSumsBatchMulti(
    JNIEnv* env, jclass cls, jlongArray ctxs, jobjectArray data, jintArray filePieces, jlongArray sizes, jintArray hdrs,
    jbyteArray seed, jobjectArray weakOut, jobjectArray strongOut) {
    (void)cls;
    jint n = 0;
    rsh_ctx** cs = ctxs_of(env, ctxs, &n);
    if (!cs) return;
    block_sums_segment(env, cs, n, data, filePieces, sizes, hdrs, seed, weakOut, strongOut);
    free(cs);
}

/* An event buffer no scan of n bytes overflows (Sender.java:1251-1316):
 *  - a MATCH consumes its window, w = min(B, n - start) bytes (:1279-1287); w < B only when the window reaches the
 *    file's end, and then the match ends the scan, so M <= n / B + 1 (runs of consecutive matches are one event);
 *  - a flush (isFull, :1294-1302) emits exactly 10*B literal bytes and moves the mark past them: F <= n / (10 B);
 *  - every other LITERAL precedes a MATCH (:1270) or is the final one (:1313), and empty literals are not emitted.
 * So events <= 2 M + F + 1 <= 2 (n / B + 1) + n / (10 B) + 1 (tests/test_oracle.py::test_event_bound_adversarial
 * checks the bound on alternating match / literal / flush sources at small B). */
static int64_t event_bound(int64_t n, const rsh_header* h) {
    if (h->block_length <= 0) return n / 8192 + 2;
    return 2 * (n / h->block_length + 1) + n / (10 * (int64_t)h->block_length) + 4;
}

/* A file whose events outran event_bound (it cannot, by the argument above; this keeps the segment correct should
 * the bound ever be wrong) is scanned again alone into a buffer of the event count the first scan reported. */
static int rescan_nospace(rsh_ctx* c, rsh_scan_batch_job* jobs, jint nf, const uint8_t* seed) {
    int rc = RSH_OK;
    for (jint f = 0; f < nf; ++f) {
        if (jobs[f].status == RSH_OK) continue;
        if (jobs[f].status != RSH_E_NOSPACE) return jobs[f].status;
        rsh_event* ev = (rsh_event*)realloc(jobs[f].ev, (size_t)jobs[f].n_ev * sizeof(rsh_event) + sizeof(rsh_event));
        if (!ev) return RSH_E_NOMEM;
        jobs[f].ev = ev;
        jobs[f].ev_cap = jobs[f].n_ev;
        rc = rsh_match_scan_batch(c, &jobs[f], 1, seed, NULL);
        if (rc != RSH_OK) return rc;
    }
    return rc;
}

/* Returns every file's events, file after file, as {kind, offset, length, index | (count << 32)} quadruples;
 * perFileOut[3f..3f+2] = {event count, sizeLiteral, sizeMatch}, fileMd5Out[16f..16f+15] = file f's MD5. */
/* A segment's Sender pass over nctx contexts (rsh_match_scan_batch_multi; nctx 1: rsh_match_scan_batch). */
static jlongArray scan_segment(JNIEnv* env, rsh_ctx* const* ctxs, jint nctx, jobjectArray src, jintArray filePieces,
                               jlongArray sizes, jintArray hdrs, jobjectArray weak, jobjectArray strong, jbyteArray seed,
                               jbyteArray fileMd5Out, jlongArray perFileOut) {
    jbyte s4[4];
    if (seed_from(env, seed, s4) != RSH_OK) {
        throw_status(env, RSH_E_INVAL);
        return NULL;
    }
    segment_args a;
    if (segment_from(env, src, filePieces, sizes, hdrs, &a) != RSH_OK) return NULL;
    const jint nf = a.nf;
    int rc = RSH_OK;
    if (!weak || !strong || !fileMd5Out || !perFileOut || (*env)->GetArrayLength(env, weak) < nf ||
        (*env)->GetArrayLength(env, strong) < nf || (*env)->GetArrayLength(env, fileMd5Out) < 16 * (jlong)nf ||
        (*env)->GetArrayLength(env, perFileOut) < 3 * (jlong)nf)
        rc = RSH_E_INVAL;
    rsh_scan_batch_job* jobs = (rsh_scan_batch_job*)calloc((size_t)nf + 1, sizeof(rsh_scan_batch_job));
    if (rc == RSH_OK && !jobs) rc = RSH_E_NOMEM;
    for (jint f = 0; rc == RSH_OK && f < nf; ++f) {
        jobject wa = (*env)->GetObjectArrayElement(env, weak, f);
        jobject sa = (*env)->GetObjectArrayElement(env, strong, f);
        const jsize nw = wa ? (*env)->GetArrayLength(env, wa) : 0, ns = sa ? (*env)->GetArrayLength(env, sa) : 0;
        const rsh_header* h = &a.h[f];
        if (h->chunk_count > 0 && (nw < h->chunk_count || (jlong)ns < (jlong)h->chunk_count * h->digest_length))
            rc = RSH_E_INVAL; /* received table shorter than its header says */
        int64_t n = 0;
        for (int32_t k = 0; k < a.count[f]; ++k) n += a.pieces[a.first[f] + k].len;
        jobs[f].pieces = a.pieces + a.first[f];
        jobs[f].npieces = a.count[f];
        jobs[f].h = *h;
        jobs[f].ev_cap = event_bound(n, h);
        jobs[f].ev = (rsh_event*)malloc((size_t)jobs[f].ev_cap * sizeof(rsh_event));
        int32_t* w = (int32_t*)malloc((size_t)nw * 4 + 4);
        uint8_t* st = (uint8_t*)malloc((size_t)ns + 1);
        jobs[f].weak = w;
        jobs[f].strong = st;
        if (rc == RSH_OK && (!jobs[f].ev || !w || !st)) rc = RSH_E_NOMEM;
        if (rc == RSH_OK && nw) (*env)->GetIntArrayRegion(env, wa, 0, nw, (jint*)w);
        if (rc == RSH_OK && ns) (*env)->GetByteArrayRegion(env, sa, 0, ns, (jbyte*)st);
        if (wa) (*env)->DeleteLocalRef(env, wa);
        if (sa) (*env)->DeleteLocalRef(env, sa);
    }
    jlongArray out = NULL;
    if (rc == RSH_OK) {
        rc = rsh_match_scan_batch_multi(ctxs, nctx, jobs, nf, (const uint8_t*)s4, NULL);
        if (rc == RSH_E_NOSPACE) rc = rescan_nospace(ctxs[0], jobs, nf, (const uint8_t*)s4);
        if (rc != RSH_OK) {
            jint f = 0;
            while (f < nf && jobs[f].status == RSH_OK) ++f;
            if (f < nf) throw_file_status(env, f, jobs[f].status);
            else throw_status(env, rc); /* the call failed before any file did */
        } else {
            int64_t total = 0;
            for (jint f = 0; f < nf; ++f) total += jobs[f].n_ev;
            out = (*env)->NewLongArray(env, (jsize)(4 * total));
            jlong* o = out ? (*env)->GetLongArrayElements(env, out, NULL) : NULL;
            if (o) {
                int64_t q = 0;
                for (jint f = 0; f < nf; ++f) {
                    const rsh_event* ev = jobs[f].ev;
                    for (int64_t i = 0; i < jobs[f].n_ev; ++i, ++q) {
                        o[4 * q + 0] = ev[i].kind;
                        o[4 * q + 1] = ev[i].offset;
                        o[4 * q + 2] = ev[i].length;
                        o[4 * q + 3] = (jlong)(uint32_t)ev[i].index | ((jlong)ev[i].count << 32);
                    }
                    const jlong per[3] = {jobs[f].n_ev, jobs[f].literal, jobs[f].matched};
                    (*env)->SetLongArrayRegion(env, perFileOut, 3 * f, 3, per);
                    (*env)->SetByteArrayRegion(env, fileMd5Out, 16 * f, 16, (const jbyte*)jobs[f].file_md5);
                }
                (*env)->ReleaseLongArrayElements(env, out, o, 0);
            } else {
                out = NULL; /* OutOfMemoryError pending */
            }
        }
    } else {
        throw_status(env, rc);
    }
    for (jint f = 0; jobs && f < nf; ++f) {
        free(jobs[f].ev);
        free((void*)jobs[f].weak);
        free((void*)jobs[f].strong);
    }
    free(jobs);
    segment_free(&a);
    return out;
}

JNIEXPORT jlongArray JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_matchScanBatch(
    JNIEnv* env, jclass cls, jlong ctx, jobjectArray src, jintArray filePieces, jlongArray sizes, jintArray hdrs,
    jobjectArray weak, jobjectArray strong, jbyteArray seed, jbyteArray fileMd5Out, jlongArray perFileOut) {
    (void)cls;
    rsh_ctx* c = ctx_of(env, ctx);
    if (!c) return NULL;
    return scan_segment(env, &c, 1, src, filePieces, sizes, hdrs, weak, strong, seed, fileMd5Out, perFileOut);
}

/* As matchScanBatch over the thread's contexts on the node's GPUs (rsh_match_scan_batch_multi). */
JNIEXPORT jlongArray JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_matchScanBatchMulti(
    JNIEnv* env, jclass cls, jlongArray ctxs, jobjectArray src, jintArray filePieces, jlongArray sizes, jintArray hdrs,
    jobjectArray weak, jobjectArray strong, jbyteArray seed, jbyteArray fileMd5Out, jlongArray perFileOut) {
    (void)cls;
    jint n = 0;
    rsh_ctx** cs = ctxs_of(env, ctxs, &n);
    if (!cs) return NULL;
    jlongArray out = scan_segment(env, cs, n, src, filePieces, sizes, hdrs, weak, strong, seed, fileMd5Out, perFileOut);
    free(cs);
    return out;
}

/* ---- Receiver.combineDataToFile (Receiver.java:459-555) over direct buffers ----
 * tokens: the file's de-multiplexed token stream; replica may be null; target receives the file.
 * resultOut[4] = {tokensUsed, targetLength, sizeLiteral, sizeMatch}; md5Out[16] = the Receiver's digest.
 * Returns combineDataToFile's value (true: deferred write, the replica is the file). */
JNIEXPORT jboolean JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_receiverCombine(
    JNIEnv* env, jclass cls, jlong ctx, jobject tokens, jlong tokensLen, jintArray hdr4, jobject replica,
    jlong replicaLen, jboolean deferWrite, jobject target, jlong targetCap, jlongArray resultOut, jbyteArray md5Out) {
    (void)cls;
    rsh_ctx* c = ctx_of(env, ctx);
    if (!c) return JNI_FALSE;
    rsh_header h;
    if (header_from(env, hdr4, &h) != RSH_OK || !resultOut || !md5Out || (*env)->GetArrayLength(env, resultOut) < 4 ||
        (*env)->GetArrayLength(env, md5Out) != 16) {
        throw_status(env, RSH_E_INVAL);
        return JNI_FALSE;
    }
    const uint8_t* t = direct_bytes(env, tokens, tokensLen);
    if (!t) return JNI_FALSE;
    const uint8_t* r = NULL;
    if (replica && !(r = direct_bytes(env, replica, replicaLen))) return JNI_FALSE;
    uint8_t* o = NULL;
    if (target && !(o = (uint8_t*)direct_bytes(env, target, targetCap))) return JNI_FALSE;
    rsh_combine_result res;
    int rc = rsh_receiver_combine(c, t, tokensLen, &h, r, r ? replicaLen : 0, deferWrite ? 1 : 0, o, o ? targetCap : 0,
                                  &res);
    if (rc != RSH_OK) {
        throw_status(env, rc);
        return JNI_FALSE;
    }
    jlong vals[4] = {res.tokens_used, res.target_len, res.literal, res.matched};
    (*env)->SetLongArrayRegion(env, resultOut, 0, 4, vals);
    (*env)->SetByteArrayRegion(env, md5Out, 0, 16, (const jbyte*)res.md5);
    return res.intact ? JNI_TRUE : JNI_FALSE;
}
