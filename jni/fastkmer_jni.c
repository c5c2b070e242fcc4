/*
 * fastkmer_jni.c -- JNI binding of the C ABI (include/fastkmer.h) for the
 * Scala object skc.gpu.NativeKmerCounter (jni/skc/gpu/NativeKmerCounter.scala).
 *
 * It is the thin host layer a fastkmer maintainer adds so that
 * SparkBinKmerCounter.executeJob (src/main/scala/skc/SparkBinKmerCounter.scala:989)
 * calls the MI355X counter instead of the Spark map / reduceByKey / reduce closures
 * (:1033-1043).  Every native method maps to one fk_* call; a negative FK_E_* return
 * becomes a java.lang.RuntimeException carrying fk_last_error(), mirroring the
 * reference, whose failures are exceptions that fail the Spark task (require at
 * package.scala:182,185; ArrayIndexOutOfBounds for x = 0 at SBKC:508).
 *
 * Build (only where a JDK is installed; this image has none):
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *       jni/fastkmer_jni.c -Lfastkmer_amd/lib -lfastkmer -Wl,-rpath,'$ORIGIN' -o libfastkmer_jni.so
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "fastkmer.h"

static void throw_fk(JNIEnv *env, int rc) {
    char msg[768];
    snprintf(msg, sizeof msg, "fastkmer error %d: %s", rc, fk_last_error());
    jclass ex = (*env)->FindClass(env, "java/lang/RuntimeException");
    if (ex) (*env)->ThrowNew(env, ex, msg);
}

static fk_ctx *ctx_of(jlong h) { return (fk_ctx *)(intptr_t)h; }

/* def create(k, m, x, b, useHT, sequenceType, nRanks, rank, device): Long */
JNIEXPORT jlong JNICALL Java_skc_gpu_NativeKmerCounter_00024_create(JNIEnv *env, jobject self, jint k, jint m, jint x,
                                                                   jint b, jboolean use_ht, jint seq_type,
                                                                   jint n_ranks, jint rank, jint device) {
    (void)self;
    fk_config cfg;
    fk_config_init(&cfg);
    cfg.k = k;
    cfg.m = m;
    cfg.x = x;
    cfg.B = b;
    cfg.use_ht = use_ht ? 1 : 0;
    cfg.sequence_type = seq_type;
    cfg.n_ranks = n_ranks;
    cfg.rank = rank;
    cfg.device = device;
    fk_ctx *c = NULL;
    const int rc = fk_create(&cfg, &c);
    if (rc != FK_OK) {
        throw_fk(env, rc);
        return 0;
    }
    return (jlong)(intptr_t)c;
}

/* def ingest(h, fasta: java.nio.ByteBuffer (direct or file-mapped), n, last): Unit */
JNIEXPORT void JNICALL Java_skc_gpu_NativeKmerCounter_00024_ingest(JNIEnv *env, jobject self, jlong h, jobject buf,
                                                                  jlong n, jboolean last) {
    (void)self;
    const uint8_t *p = (const uint8_t *)(*env)->GetDirectBufferAddress(env, buf);
    const jlong cap = (*env)->GetDirectBufferCapacity(env, buf);
    if (!p || cap < n || n < 0) {
        jclass ex = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
        if (ex) (*env)->ThrowNew(env, ex, "ingest needs a direct ByteBuffer holding n bytes");
        return;
    }
    const int rc = fk_ingest(ctx_of(h), p, (size_t)n, last ? 1 : 0);
    if (rc != FK_OK) throw_fk(env, rc);
}

/* def ingestFileRange(h, path, world, rank, window): Unit -- the job's whole input: this rank's
 * split of the file (FASTdoop-style: whole records for sequenceType 0, the k - 1 overlap and a
 * header prefix for sequenceType 1; SBKC:993, 1009-1012), read by the library in pinned windows */
JNIEXPORT void JNICALL Java_skc_gpu_NativeKmerCounter_00024_ingestFileRange(JNIEnv *env, jobject self, jlong h,
                                                                           jstring path, jint world, jint rank,
                                                                           jlong window) {
    (void)self;
    const char *p = (*env)->GetStringUTFChars(env, path, NULL);
    if (!p) return;
    const int rc = fk_ingest_file_range(ctx_of(h), p, world, rank, window < 0 ? 0 : (uint64_t)window);
    (*env)->ReleaseStringUTFChars(env, path, p);
    if (rc != FK_OK) throw_fk(env, rc);
}

/* def balanceBinsFile(h, path, world, rank, fraction): Unit -- useCustomPartitioner (SBKC:1023-1026,
 * MultiprocessorSchedulingPartitioner.scala:35-69): `fraction` of this rank's split mapped (never
 * exchanged), the per-bin k-mer totals summed over the ranks, the LPT placement installed for the
 * job's exchange; collective, before ingestFileRange */
JNIEXPORT void JNICALL Java_skc_gpu_NativeKmerCounter_00024_balanceBinsFile(JNIEnv *env, jobject self, jlong h,
                                                                           jstring path, jint world, jint rank,
                                                                           jdouble fraction) {
    (void)self;
    const char *p = (*env)->GetStringUTFChars(env, path, NULL);
    if (!p) return;
    const int rc = fk_balance_bins_file(ctx_of(h), p, world, rank, fraction);
    (*env)->ReleaseStringUTFChars(env, path, p);
    if (rc != FK_OK) throw_fk(env, rc);
}

/* def finish(h): Unit -- map and count (one rank); with a communicator the last piece, the
 * exchange with the other ranks and the count of this rank's bins (collective) */
JNIEXPORT void JNICALL Java_skc_gpu_NativeKmerCounter_00024_finish(JNIEnv *env, jobject self, jlong h) {
    (void)self;
    const int rc = fk_finish(ctx_of(h));
    if (rc != FK_OK) throw_fk(env, rc);
}

/* def commUniqueId(): Array[Byte] -- a fresh RCCL unique id, made on one executor (e.g. the
 * driver) and handed to every rank of the job with the task closure */
JNIEXPORT jbyteArray JNICALL Java_skc_gpu_NativeKmerCounter_00024_commUniqueId(JNIEnv *env, jobject self) {
    (void)self;
    uint8_t id[FK_COMM_ID_BYTES];
    const int rc = fk_comm_unique_id(id);
    if (rc != FK_OK) {
        throw_fk(env, rc);
        return NULL;
    }
    jbyteArray out = (*env)->NewByteArray(env, FK_COMM_ID_BYTES);
    if (out) (*env)->SetByteArrayRegion(env, out, 0, FK_COMM_ID_BYTES, (const jbyte *)id);
    return out;
}

/* def commInit(h, id: Array[Byte]): Unit -- join the job's RCCL communicator (every rank) */
JNIEXPORT void JNICALL Java_skc_gpu_NativeKmerCounter_00024_commInit(JNIEnv *env, jobject self, jlong h,
                                                                    jbyteArray id) {
    (void)self;
    if (!id || (*env)->GetArrayLength(env, id) != FK_COMM_ID_BYTES) {
        jclass ex = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
        if (ex) (*env)->ThrowNew(env, ex, "an RCCL unique id has 128 bytes");
        return;
    }
    uint8_t buf[FK_COMM_ID_BYTES];
    (*env)->GetByteArrayRegion(env, id, 0, FK_COMM_ID_BYTES, (jbyte *)buf);
    const int rc = fk_comm_init(ctx_of(h), buf);
    if (rc != FK_OK) throw_fk(env, rc);
}

/* def binSizes(h): Array[Long] -- distinct k-mers per bin */
JNIEXPORT jlongArray JNICALL Java_skc_gpu_NativeKmerCounter_00024_binSizes(JNIEnv *env, jobject self, jlong h) {
    (void)self;
    const int32_t nb = fk_num_bins(ctx_of(h));
    jlongArray out = (*env)->NewLongArray(env, nb);
    if (!out || nb <= 0) return out;
    jlong *dst = (*env)->GetLongArrayElements(env, out, NULL);
    const int rc = fk_bin_sizes(ctx_of(h), (uint64_t *)dst);
    (*env)->ReleaseLongArrayElements(env, out, dst, 0);
    if (rc != FK_OK) throw_fk(env, rc);
    return out;
}

/* def writeBins(h, outDir): Unit -- the reference's bin<b> files */
JNIEXPORT void JNICALL Java_skc_gpu_NativeKmerCounter_00024_writeBins(JNIEnv *env, jobject self, jlong h,
                                                                     jstring dir) {
    (void)self;
    const char *d = (*env)->GetStringUTFChars(env, dir, NULL);
    if (!d) return;
    const int rc = fk_write_bins(ctx_of(h), d);
    (*env)->ReleaseStringUTFChars(env, dir, d);
    if (rc != FK_OK) throw_fk(env, rc);
}

/* def findBinSignatures(h, outDir): Unit -- executeFindBinSignaturesJob's
 * bin_signatures<b>.txt files (SBKC:956-986) for this context's input */
JNIEXPORT void JNICALL Java_skc_gpu_NativeKmerCounter_00024_findBinSignatures(JNIEnv *env, jobject self, jlong h,
                                                                             jstring dir) {
    (void)self;
    const char *d = (*env)->GetStringUTFChars(env, dir, NULL);
    if (!d) return;
    const int rc = fk_find_bin_signatures(ctx_of(h), d);
    (*env)->ReleaseStringUTFChars(env, dir, d);
    if (rc != FK_OK) throw_fk(env, rc);
}

/* def destroy(h): Unit */
JNIEXPORT void JNICALL Java_skc_gpu_NativeKmerCounter_00024_destroy(JNIEnv *env, jobject self, jlong h) {
    (void)env;
    (void)self;
    fk_destroy(ctx_of(h));
}
