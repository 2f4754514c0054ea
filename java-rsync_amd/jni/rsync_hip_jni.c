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
 * blockSums / matchScan take the file bytes from Java (FileView semantics incl. zero-fill after read
 * errors stay in Java, FileView.java:209-271); blockSumsFile / matchScanFile read the file natively with
 * the same semantics and report a read error as a flag (the FileViewException the Java code would get
 * at close()).  The Sender replays the returned events through its own sendDataFrom/putInt so channel
 * framing is untouched (Sender.java:794-809).
 *
 * Build (needs a JDK): make -C java-rsync_amd jni JAVA_HOME=/path/to/jdk
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rsync_hip.h"

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
    jclass c = (*env)->FindClass(env, cls);
    if (!c) return; /* NoClassDefFoundError already pending */
    (*env)->ThrowNew(env, c, rsh_strerror(rc));
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
    rsh_ctx_destroy((rsh_ctx*)(intptr_t)ctx);
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

/*
 * Generator.sendItemizeAndChecksums hot loop (Generator.java:886-895).
 * data: a direct ByteBuffer holding the whole basis file (n bytes).  weakOut[chunkCount],
 * strongOut[chunkCount * digestLength] are filled; Java then writes header + sums to the channel.
 */
JNIEXPORT void JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_blockSums(
    JNIEnv* env, jclass cls, jlong ctx, jobject data, jlong n, jintArray hdr4, jbyteArray seed, jintArray weakOut,
    jbyteArray strongOut) {
    (void)cls;
    rsh_header h;
    int rc = header_from(env, hdr4, &h);
    if (rc != RSH_OK) {
        throw_status(env, rc);
        return;
    }
    const uint8_t* p = (const uint8_t*)(*env)->GetDirectBufferAddress(env, data);
    if ((!p && n > 0) || (*env)->GetArrayLength(env, seed) != 4 ||
        (*env)->GetArrayLength(env, weakOut) < h.chunk_count ||
        (*env)->GetArrayLength(env, strongOut) < (jlong)h.chunk_count * h.digest_length) {
        throw_status(env, RSH_E_INVAL);
        return;
    }
    jbyte s4[4];
    (*env)->GetByteArrayRegion(env, seed, 0, 4, s4);
    /* the call can run for seconds: native buffers, not JNI critical regions (which would stall GC) */
    const size_t C = (size_t)(h.chunk_count > 0 ? h.chunk_count : 0), dl = (size_t)(h.digest_length > 0 ? h.digest_length : 0);
    int32_t* w = (int32_t*)malloc(C * 4 + 4);
    uint8_t* st = (uint8_t*)malloc(C * dl + 1);
    rc = (w && st) ? rsh_block_sums((rsh_ctx*)(intptr_t)ctx, p, n, &h, (const uint8_t*)s4, w, st) : RSH_E_NOMEM;
    if (rc == RSH_OK) {
        (*env)->SetIntArrayRegion(env, weakOut, 0, (jsize)C, (const jint*)w);
        (*env)->SetByteArrayRegion(env, strongOut, 0, (jsize)(C * dl), (const jbyte*)st);
    }
    free(st);
    free(w);
    if (rc != RSH_OK) throw_status(env, rc);
}

/*
 * Sender.sendMatchesAndData / skipMatchSendData (Sender.java:1235-1327, 1386-1399).
 * Returns the events as a flat long[] of 4-tuples {kind, offset, length, index | (count << 32)};
 * fileMd5Out[16] receives the whole-file digest and sizesOut[2] = {sizeLiteral, sizeMatch}.
 */
JNIEXPORT jlongArray JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_matchScan(
    JNIEnv* env, jclass cls, jlong ctx, jobject src, jlong n, jintArray hdr4, jintArray weak, jbyteArray strong,
    jbyteArray seed, jbyteArray fileMd5Out, jlongArray sizesOut) {
    (void)cls;
    rsh_header h;
    int rc = header_from(env, hdr4, &h);
    if (rc != RSH_OK) {
        throw_status(env, rc);
        return NULL;
    }
    const uint8_t* p = (const uint8_t*)(*env)->GetDirectBufferAddress(env, src);
    if ((!p && n > 0) || (*env)->GetArrayLength(env, seed) != 4 || (*env)->GetArrayLength(env, fileMd5Out) != 16 ||
        (*env)->GetArrayLength(env, sizesOut) < 2) {
        throw_status(env, RSH_E_INVAL);
        return NULL;
    }
    jbyte s4[4];
    (*env)->GetByteArrayRegion(env, seed, 0, 4, s4);
    /* one literal per flush interval plus a literal and a match run per chunk; a short buffer is not
       a rescan: the context keeps the events for rsh_fetch_events */
    int64_t cap = (n / (10 * (int64_t)(h.block_length > 0 ? h.block_length : 8192))) + 2 * (int64_t)h.chunk_count + 64;
    int64_t n_ev = 0, lit = 0, mat = 0;
    rsh_event* ev = (rsh_event*)malloc((size_t)cap * sizeof(rsh_event));
    uint8_t md5[16];
    if (!ev) {
        rc = RSH_E_NOMEM;
    } else {
        /* copies of the (small) received table: no JNI critical region across a long scan */
        const jsize nw = weak ? (*env)->GetArrayLength(env, weak) : 0;
        const jsize ns = strong ? (*env)->GetArrayLength(env, strong) : 0;
        int32_t* w = (int32_t*)malloc((size_t)nw * 4 + 4);
        uint8_t* st = (uint8_t*)malloc((size_t)ns + 1);
        if (!w || !st) {
            rc = RSH_E_NOMEM;
        } else if (h.chunk_count > 0 && (nw < h.chunk_count || (jlong)ns < (jlong)h.chunk_count * h.digest_length)) {
            rc = RSH_E_INVAL; /* received table shorter than its header says */
        } else {
            if (nw) (*env)->GetIntArrayRegion(env, weak, 0, nw, (jint*)w);
            if (ns) (*env)->GetByteArrayRegion(env, strong, 0, ns, (jbyte*)st);
            rc = rsh_match_scan((rsh_ctx*)(intptr_t)ctx, p, n, &h, nw ? w : NULL, ns ? st : NULL, (const uint8_t*)s4,
                                ev, cap, &n_ev, md5, &lit, &mat, NULL);
        }
        free(st);
        free(w);
        if (rc == RSH_E_NOSPACE) {
            rsh_event* grown = (rsh_event*)realloc(ev, (size_t)n_ev * sizeof(rsh_event));
            if (!grown) rc = RSH_E_NOMEM;
            else {
                ev = grown;
                rc = rsh_fetch_events((rsh_ctx*)(intptr_t)ctx, ev, n_ev, &n_ev);
            }
        }
    }
    if (rc != RSH_OK) {
        free(ev);
        throw_status(env, rc);
        return NULL;
    }
    jlongArray out = (*env)->NewLongArray(env, (jsize)(4 * n_ev));
    if (out) {
        jlong* o = (*env)->GetLongArrayElements(env, out, NULL);
        for (int64_t i = 0; i < n_ev; ++i) {
            o[4 * i + 0] = ev[i].kind;
            o[4 * i + 1] = ev[i].offset;
            o[4 * i + 2] = ev[i].length;
            o[4 * i + 3] = (jlong)(uint32_t)ev[i].index | ((jlong)ev[i].count << 32);
        }
        (*env)->ReleaseLongArrayElements(env, out, o, 0);
        (*env)->SetByteArrayRegion(env, fileMd5Out, 0, 16, (const jbyte*)md5);
        jlong sizes[2] = {lit, mat};
        (*env)->SetLongArrayRegion(env, sizesOut, 0, 2, sizes);
    }
    free(ev);
    return out;
}

/* ---- the same passes reading the file natively (rsh_*_file: FileView.java:51-80,187-278 semantics) ---- */

/* Returns true when the file could not be read to `size` (zero-filled from there: FileViewException). */
JNIEXPORT jboolean JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_blockSumsFile(
    JNIEnv* env, jclass cls, jlong ctx, jstring path, jlong size, jintArray hdr4, jbyteArray seed, jintArray weakOut,
    jbyteArray strongOut) {
    (void)cls;
    rsh_header h;
    int rc = header_from(env, hdr4, &h);
    if (rc != RSH_OK || !path || (*env)->GetArrayLength(env, seed) != 4 ||
        (*env)->GetArrayLength(env, weakOut) < h.chunk_count ||
        (*env)->GetArrayLength(env, strongOut) < (jlong)h.chunk_count * h.digest_length) {
        throw_status(env, rc != RSH_OK ? rc : RSH_E_INVAL);
        return JNI_FALSE;
    }
    jbyte s4[4];
    (*env)->GetByteArrayRegion(env, seed, 0, 4, s4);
    const size_t C = (size_t)(h.chunk_count > 0 ? h.chunk_count : 0), dl = (size_t)(h.digest_length > 0 ? h.digest_length : 0);
    int32_t* w = (int32_t*)malloc(C * 4 + 4);
    uint8_t* st = (uint8_t*)malloc(C * dl + 1);
    const char* cpath = (*env)->GetStringUTFChars(env, path, NULL);
    int32_t read_error = 0;
    rc = (w && st && cpath) ? rsh_block_sums_file((rsh_ctx*)(intptr_t)ctx, cpath, size, &h, (const uint8_t*)s4, w, st,
                                                  &read_error)
                            : RSH_E_NOMEM;
    if (cpath) (*env)->ReleaseStringUTFChars(env, path, cpath);
    if (rc == RSH_OK) {
        (*env)->SetIntArrayRegion(env, weakOut, 0, (jsize)C, (const jint*)w);
        (*env)->SetByteArrayRegion(env, strongOut, 0, (jsize)(C * dl), (const jbyte*)st);
    }
    free(st);
    free(w);
    if (rc != RSH_OK) throw_status(env, rc);
    return read_error ? JNI_TRUE : JNI_FALSE;
}

/* As matchScan, reading the source natively; sizesOut[3] = {sizeLiteral, sizeMatch, readError}. */
JNIEXPORT jlongArray JNICALL Java_com_github_java_rsync_internal_session_NativeChecksum_matchScanFile(
    JNIEnv* env, jclass cls, jlong ctx, jstring path, jlong size, jintArray hdr4, jintArray weak, jbyteArray strong,
    jbyteArray seed, jbyteArray fileMd5Out, jlongArray sizesOut) {
    (void)cls;
    rsh_header h;
    int rc = header_from(env, hdr4, &h);
    if (rc != RSH_OK || !path || (*env)->GetArrayLength(env, seed) != 4 ||
        (*env)->GetArrayLength(env, fileMd5Out) != 16 || (*env)->GetArrayLength(env, sizesOut) < 3) {
        throw_status(env, rc != RSH_OK ? rc : RSH_E_INVAL);
        return NULL;
    }
    jbyte s4[4];
    (*env)->GetByteArrayRegion(env, seed, 0, 4, s4);
    int64_t cap = (size / (10 * (int64_t)(h.block_length > 0 ? h.block_length : 8192))) + 2 * (int64_t)h.chunk_count + 64;
    int64_t n_ev = 0, lit = 0, mat = 0;
    int32_t read_error = 0;
    rsh_event* ev = (rsh_event*)malloc((size_t)cap * sizeof(rsh_event));
    const jsize nw = weak ? (*env)->GetArrayLength(env, weak) : 0;
    const jsize ns = strong ? (*env)->GetArrayLength(env, strong) : 0;
    int32_t* w = (int32_t*)malloc((size_t)nw * 4 + 4);
    uint8_t* st = (uint8_t*)malloc((size_t)ns + 1);
    const char* cpath = (*env)->GetStringUTFChars(env, path, NULL);
    uint8_t md5[16];
    if (!ev || !w || !st || !cpath) {
        rc = RSH_E_NOMEM;
    } else if (h.chunk_count > 0 && (nw < h.chunk_count || (jlong)ns < (jlong)h.chunk_count * h.digest_length)) {
        rc = RSH_E_INVAL;
    } else {
        if (nw) (*env)->GetIntArrayRegion(env, weak, 0, nw, (jint*)w);
        if (ns) (*env)->GetByteArrayRegion(env, strong, 0, ns, (jbyte*)st);
        rc = rsh_match_scan_file((rsh_ctx*)(intptr_t)ctx, cpath, size, &h, nw ? w : NULL, ns ? st : NULL,
                                 (const uint8_t*)s4, ev, cap, &n_ev, md5, &lit, &mat, NULL, &read_error);
        if (rc == RSH_E_NOSPACE) {
            rsh_event* grown = (rsh_event*)realloc(ev, (size_t)n_ev * sizeof(rsh_event));
            if (!grown) rc = RSH_E_NOMEM;
            else {
                ev = grown;
                rc = rsh_fetch_events((rsh_ctx*)(intptr_t)ctx, ev, n_ev, &n_ev);
            }
        }
    }
    if (cpath) (*env)->ReleaseStringUTFChars(env, path, cpath);
    free(st);
    free(w);
    jlongArray out = NULL;
    if (rc == RSH_OK) out = (*env)->NewLongArray(env, (jsize)(4 * n_ev));
    if (out) {
        jlong* o = (*env)->GetLongArrayElements(env, out, NULL);
        for (int64_t i = 0; i < n_ev; ++i) {
            o[4 * i + 0] = ev[i].kind;
            o[4 * i + 1] = ev[i].offset;
            o[4 * i + 2] = ev[i].length;
            o[4 * i + 3] = (jlong)(uint32_t)ev[i].index | ((jlong)ev[i].count << 32);
        }
        (*env)->ReleaseLongArrayElements(env, out, o, 0);
        (*env)->SetByteArrayRegion(env, fileMd5Out, 0, 16, (const jbyte*)md5);
        jlong sizes[3] = {lit, mat, read_error};
        (*env)->SetLongArrayRegion(env, sizesOut, 0, 3, sizes);
    }
    free(ev);
    if (rc != RSH_OK) throw_status(env, rc);
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
    rsh_header h;
    int rc = header_from(env, hdr4, &h);
    const uint8_t* t = tokens ? (const uint8_t*)(*env)->GetDirectBufferAddress(env, tokens) : NULL;
    const uint8_t* r = replica ? (const uint8_t*)(*env)->GetDirectBufferAddress(env, replica) : NULL;
    uint8_t* o = target ? (uint8_t*)(*env)->GetDirectBufferAddress(env, target) : NULL;
    if (rc != RSH_OK || !t || (replica && !r) || (*env)->GetArrayLength(env, resultOut) < 4 ||
        (*env)->GetArrayLength(env, md5Out) != 16) {
        throw_status(env, rc != RSH_OK ? rc : RSH_E_INVAL);
        return JNI_FALSE;
    }
    rsh_combine_result res;
    rc = rsh_receiver_combine((rsh_ctx*)(intptr_t)ctx, t, tokensLen, &h, r, r ? replicaLen : 0, deferWrite ? 1 : 0, o,
                              o ? targetCap : 0, &res);
    if (rc != RSH_OK) {
        throw_status(env, rc);
        return JNI_FALSE;
    }
    jlong vals[4] = {res.tokens_used, res.target_len, res.literal, res.matched};
    (*env)->SetLongArrayRegion(env, resultOut, 0, 4, vals);
    (*env)->SetByteArrayRegion(env, md5Out, 0, 16, (const jbyte*)res.md5);
    return res.intact ? JNI_TRUE : JNI_FALSE;
}
