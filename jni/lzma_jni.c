/*
 * lzma_jni.c -- JNI binding of the MI355X LZMA path (include/lzma_mi355x.h) for the
 * Java drop-in classes in java/SevenZip/Compression/LZMA/ (Encoder, Decoder, Native).
 *
 * Replaces, for the Java callers of rfalke/lzma-java, the hot path of
 *   Encoder.Code   src/main/java/SevenZip/Compression/LZMA/Encoder.java:1064-1077
 *   Decoder.Code   src/main/java/SevenZip/Compression/LZMA/Decoder.java:205-301
 * The setters' range checks stay in Java with the reference's return values.
 *
 * Build (needs a JDK; none exists in the build container or on the GPU box, so this
 * file is not compiled by the repository's own build): see jni/Makefile.
 *
 * One device context per process on the first device of the mask
 * -Dlzma.mi355x.devices (default 1 = device 0); encodeBatch deals a batch's streams
 * over every device of the mask (lzma_enc_batch_multi). The contexts keep their
 * device buffers between calls (no hipMalloc per Code call). Calls are serialised:
 * the reference's Encoder/Decoder instances are single-threaded, and so is a context.
 */
#include <jni.h>
#include <limits.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>

#include "lzma_mi355x.h"

static lzma_mctx *g_m;
static lzma_ctx *g_ctx;
static int g_dev0;   /* the first device of the mask (init) */
static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;

static void throw_io(JNIEnv *env, const char *msg) {
    jclass c = (*env)->FindClass(env, "java/io/IOException");
    if (c) (*env)->ThrowNew(env, c, msg);
}

/* static native boolean init(int deviceMask) */
JNIEXPORT jboolean JNICALL Java_SevenZip_Compression_LZMA_Native_init(JNIEnv *env, jclass cls, jint mask) {
    (void)env; (void)cls;
    uint32_t m = mask ? (uint32_t)mask : 1u;
    pthread_mutex_lock(&g_lock);
    int ok = g_ctx != NULL;
    if (!ok && lzma_mctx_create(m, &g_m) == LZMA_OK) {
        int first = 0;
        while (!(m >> first & 1u)) first++;
        ok = lzma_ctx_create(first, &g_ctx) == LZMA_OK;
        g_dev0 = first;
        if (!ok) {   /* no half-initialised state: the next init starts over */
            lzma_mctx_destroy(g_m);
            g_m = NULL;
            g_ctx = NULL;
        }
    }
    pthread_mutex_unlock(&g_lock);
    return ok ? JNI_TRUE : JNI_FALSE;
}

/* static native byte[] encode(byte[] in, int len, int dict, int fb, int mf, int lc, int lp, int pb,
 *                             boolean eos): Encoder.Code on in[0..len), the raw stream (no header) */
JNIEXPORT jbyteArray JNICALL Java_SevenZip_Compression_LZMA_Native_encode(
        JNIEnv *env, jclass cls, jbyteArray in, jint n, jint dict, jint fb, jint mf,
        jint lc, jint lp, jint pb, jboolean eos) {
    (void)cls;
    lzma_params p = {dict, fb, mf, lc, lp, pb, eos ? 1 : 0};
    uint64_t cap = lzma_enc_bound((uint64_t)n), len = 0;
    uint8_t *out = (uint8_t *)malloc(cap);
    if (!out) { throw_io(env, "out of memory"); return NULL; }
    jbyte *src = (*env)->GetPrimitiveArrayCritical(env, in, NULL);
    if (!src) { free(out); return NULL; }
    pthread_mutex_lock(&g_lock);
    int rc = lzma_encode(g_ctx, &p, (const uint8_t *)src, (uint64_t)n, out, cap, &len);
    (*env)->ReleasePrimitiveArrayCritical(env, in, src, JNI_ABORT);
    if (rc != LZMA_OK) {
        throw_io(env, lzma_last_error(g_ctx));
        pthread_mutex_unlock(&g_lock);
        free(out);
        return NULL;
    }
    pthread_mutex_unlock(&g_lock);
    if (len > (uint64_t)INT_MAX) { free(out); throw_io(env, "output longer than a Java array"); return NULL; }
    jbyteArray r = (*env)->NewByteArray(env, (jsize)len);
    if (r) (*env)->SetByteArrayRegion(env, r, 0, (jsize)len, (const jbyte *)out);
    free(out);
    return r;
}

/* static native byte[] decode(byte[] props5, byte[] in, int len, long outSize, int[] status):
 * Decoder.Code on in[0..len). status[0] = LZMA_OK or LZMA_E_DATA (Code returns false).
 * On LZMA_E_DATA the returned bytes are what the reference had written by then: the whole
 * windows OutWindow flushed (OutWindow.java:63-73), lzma_visible_on_error. outSize < 0
 * decodes until the end marker (Decoder.java:219): the output buffer grows on
 * LZMA_E_OVERFLOW and the stream is decoded again. */
JNIEXPORT jbyteArray JNICALL Java_SevenZip_Compression_LZMA_Native_decode(
        JNIEnv *env, jclass cls, jbyteArray props, jbyteArray in, jint n, jlong out_size, jintArray status) {
    (void)cls;
    uint8_t pr[5];
    (*env)->GetByteArrayRegion(env, props, 0, 5, (jbyte *)pr);
    const uint32_t dict = (uint32_t)pr[1] | ((uint32_t)pr[2] << 8) | ((uint32_t)pr[3] << 16) | ((uint32_t)pr[4] << 24);
    /* a match may run past outSize (CopyBlock copies whole matches): 273 bytes of slack;
     * a Java array holds at most INT_MAX bytes, so the capacity never exceeds that */
    if (out_size > (jlong)INT_MAX - 273) { throw_io(env, "output longer than a Java array"); return NULL; }
    uint64_t cap = out_size >= 0 ? (uint64_t)out_size + 273 : (uint64_t)n * 4 + 65536, len = 0;
    if (cap > (uint64_t)INT_MAX) cap = (uint64_t)INT_MAX;
    for (;;) {
        uint8_t *dst = (uint8_t *)malloc(cap ? cap : 1);
        if (!dst) { throw_io(env, "out of memory"); return NULL; }
        jbyte *src = (*env)->GetPrimitiveArrayCritical(env, in, NULL);
        if (!src) { free(dst); return NULL; }
        pthread_mutex_lock(&g_lock);
        int rc = lzma_decode(g_ctx, pr, (const uint8_t *)src, (uint64_t)n, (int64_t)out_size, dst, cap, &len);
        (*env)->ReleasePrimitiveArrayCritical(env, in, src, JNI_ABORT);
        if (rc == LZMA_E_OVERFLOW && out_size < 0 && cap < (uint64_t)INT_MAX) {
            pthread_mutex_unlock(&g_lock);
            free(dst);
            cap = cap > (uint64_t)INT_MAX / 2 ? (uint64_t)INT_MAX : cap * 2;
            continue;
        }
        if (rc == LZMA_E_OVERFLOW && out_size < 0) {   /* the end marker lies beyond INT_MAX bytes */
            pthread_mutex_unlock(&g_lock);
            free(dst);
            throw_io(env, "output longer than a Java array");
            return NULL;
        }
        if (rc != LZMA_OK && rc != LZMA_E_DATA) {
            throw_io(env, lzma_last_error(g_ctx));
            pthread_mutex_unlock(&g_lock);
            free(dst);
            return NULL;
        }
        pthread_mutex_unlock(&g_lock);
        if (rc == LZMA_E_DATA) len = lzma_visible_on_error(dict, len);
        if (len > (uint64_t)INT_MAX) { free(dst); throw_io(env, "output longer than a Java array"); return NULL; }
        jint st = rc;
        (*env)->SetIntArrayRegion(env, status, 0, 1, &st);
        jbyteArray r = (*env)->NewByteArray(env, (jsize)len);
        if (r) (*env)->SetByteArrayRegion(env, r, 0, (jsize)len, (const jbyte *)dst);
        free(dst);
        return r;
    }
}

/* static native long[] encodeBatch(byte[] in, long[] offs, byte[] out, int dict, int fb, int mf,
 *                                  int lc, int lp, int pb, boolean eos):
 * N independent chunks in[offs[i]..offs[i+1]) over the device mask; returns the packed
 * layout out_offs[N+1] of the encoded streams in out. */
JNIEXPORT jlongArray JNICALL Java_SevenZip_Compression_LZMA_Native_encodeBatch(
        JNIEnv *env, jclass cls, jbyteArray in, jlongArray offs, jbyteArray out,
        jint dict, jint fb, jint mf, jint lc, jint lp, jint pb, jboolean eos) {
    (void)cls;
    lzma_params p = {dict, fb, mf, lc, lp, pb, eos ? 1 : 0};
    jsize n = (*env)->GetArrayLength(env, offs) - 1;
    if (n < 0) { throw_io(env, "offs must hold N + 1 entries"); return NULL; }
    uint64_t *oo = (uint64_t *)malloc(sizeof(uint64_t) * ((size_t)n + 1));
    if (!oo) { throw_io(env, "out of memory"); return NULL; }
    jlong *o = (*env)->GetLongArrayElements(env, offs, NULL);
    jbyte *src = (*env)->GetPrimitiveArrayCritical(env, in, NULL);
    jbyte *dst = (*env)->GetPrimitiveArrayCritical(env, out, NULL);
    pthread_mutex_lock(&g_lock);
    int rc = (o && src && dst) ? lzma_enc_batch_multi(g_m, &p, (const uint8_t *)src, (const uint64_t *)o, n, (uint8_t *)dst,
                                                      (uint64_t)(*env)->GetArrayLength(env, out), oo)
                               : LZMA_E_NOMEM;
    if (dst) (*env)->ReleasePrimitiveArrayCritical(env, out, dst, 0);
    if (src) (*env)->ReleasePrimitiveArrayCritical(env, in, src, JNI_ABORT);
    if (o) (*env)->ReleaseLongArrayElements(env, offs, o, JNI_ABORT);
    if (rc != LZMA_OK) {
        throw_io(env, rc == LZMA_E_NOMEM && !(o && src && dst) ? "could not pin the Java arrays" : lzma_mctx_last_error(g_m));
        pthread_mutex_unlock(&g_lock);
        free(oo);
        return NULL;
    }
    pthread_mutex_unlock(&g_lock);
    jlongArray r = (*env)->NewLongArray(env, n + 1);
    if (r) (*env)->SetLongArrayRegion(env, r, 0, n + 1, (const jlong *)oo);
    free(oo);
    return r;
}

/* The sliced encode (lzma_enc_session_*) for Encoder.Code on a long stream: the drop-in's
 * Code loop steps it a slice at a time, writes each slice's final bytes to its OutputStream
 * and calls ICodeProgress.SetProgress between slices (Encoder.java:1069-1073 reports per
 * block). A session owns a context of its own (an open session refuses the context's other
 * calls), so other threads' Code calls keep the shared one. The handle is a jlong. */
typedef struct {
    lzma_ctx *ctx;
    lzma_enc_session *s;
} jsession;

/* static native long sessionBegin(byte[] in, int len, int dict, int fb, int mf, int lc, int lp, int pb, boolean eos) */
JNIEXPORT jlong JNICALL Java_SevenZip_Compression_LZMA_Native_sessionBegin(
        JNIEnv *env, jclass cls, jbyteArray in, jint n, jint dict, jint fb, jint mf,
        jint lc, jint lp, jint pb, jboolean eos) {
    (void)cls;
    lzma_params p = {dict, fb, mf, lc, lp, pb, eos ? 1 : 0};
    jsession *js = (jsession *)calloc(1, sizeof *js);
    if (!js) { throw_io(env, "out of memory"); return 0; }
    pthread_mutex_lock(&g_lock);
    const int dev = g_dev0;
    pthread_mutex_unlock(&g_lock);
    if (lzma_ctx_create(dev, &js->ctx) != LZMA_OK) { free(js); throw_io(env, "no MI355X device for the session"); return 0; }
    jbyte *src = (*env)->GetPrimitiveArrayCritical(env, in, NULL);
    if (!src) { lzma_ctx_destroy(js->ctx); free(js); return 0; }
    int rc = lzma_enc_session_begin_host(js->ctx, &p, (const uint8_t *)src, (uint64_t)n, &js->s);
    (*env)->ReleasePrimitiveArrayCritical(env, in, src, JNI_ABORT);
    if (rc != LZMA_OK) {
        throw_io(env, lzma_last_error(js->ctx));
        lzma_ctx_destroy(js->ctx);
        free(js);
        return 0;
    }
    return (jlong)(intptr_t)js;
}

/* static native boolean sessionStep(long h, long bytes, long[] pos): pos[0] = input consumed,
 * pos[1] = output bytes final so far; returns true once the stream is flushed */
JNIEXPORT jboolean JNICALL Java_SevenZip_Compression_LZMA_Native_sessionStep(
        JNIEnv *env, jclass cls, jlong h, jlong bytes, jlongArray pos) {
    (void)cls;
    jsession *js = (jsession *)(intptr_t)h;
    if (!js) { throw_io(env, "closed session"); return JNI_FALSE; }
    uint64_t ip = 0, ol = 0;
    int done = 0;
    int rc = lzma_enc_session_step(js->s, bytes > 0 ? (uint64_t)bytes : 1u, &ip, &ol, &done);
    if (rc != LZMA_OK) { throw_io(env, lzma_last_error(js->ctx)); return JNI_FALSE; }
    jlong v[2] = {(jlong)ip, (jlong)ol};
    (*env)->SetLongArrayRegion(env, pos, 0, 2, v);
    return done ? JNI_TRUE : JNI_FALSE;
}

/* static native void sessionOutput(long h, long from, byte[] dst, int len): final output bytes */
JNIEXPORT void JNICALL Java_SevenZip_Compression_LZMA_Native_sessionOutput(
        JNIEnv *env, jclass cls, jlong h, jlong from, jbyteArray dst, jint len) {
    (void)cls;
    jsession *js = (jsession *)(intptr_t)h;
    if (!js) { throw_io(env, "closed session"); return; }
    if (len <= 0) return;
    jbyte *d = (*env)->GetPrimitiveArrayCritical(env, dst, NULL);
    if (!d) return;
    int rc = lzma_enc_session_output(js->s, (uint64_t)from, (uint8_t *)d, (uint64_t)len);
    (*env)->ReleasePrimitiveArrayCritical(env, dst, d, 0);
    if (rc != LZMA_OK) throw_io(env, lzma_last_error(js->ctx));
}

/* static native void sessionEnd(long h) */
JNIEXPORT void JNICALL Java_SevenZip_Compression_LZMA_Native_sessionEnd(JNIEnv *env, jclass cls, jlong h) {
    (void)env; (void)cls;
    jsession *js = (jsession *)(intptr_t)h;
    if (!js) return;
    lzma_enc_session_end(js->s);
    lzma_ctx_destroy(js->ctx);
    free(js);
}
