/*
 * jni.h -- TEST DOUBLE of the JDK's <jni.h>, for compiling java-rsync_amd/jni/rsync_hip_jni.c where no JDK
 * exists (this image and the GPU box have none).  It declares only the types, macros and JNIEnv functions
 * the shim uses, with the JDK's names and calling convention ((*env)->Fn(env, ...)), so the shim source
 * compiles unchanged against either header.  tests/jni/harness.c implements these functions over plain C
 * objects; the result is a test of the shim's own logic (argument checks, buffer bounds, exception mapping,
 * event packing), not of a JVM.  The binary layout of this JNIEnv is NOT the JDK's: never load a shim built
 * against this header into a JVM.
 */
#ifndef RSH_TEST_JNI_H
#define RSH_TEST_JNI_H
#include <stdint.h>

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;

typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jintArray;
typedef jarray jbyteArray;
typedef jarray jlongArray;
typedef jarray jobjectArray;

#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
    jclass (*FindClass)(JNIEnv* env, const char* name);
    jint (*ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
    void (*DeleteLocalRef)(JNIEnv* env, jobject obj);
    void* (*GetDirectBufferAddress)(JNIEnv* env, jobject buf);
    jlong (*GetDirectBufferCapacity)(JNIEnv* env, jobject buf);
    jsize (*GetArrayLength)(JNIEnv* env, jarray array);
    jobject (*GetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index);
    void (*GetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, jint* buf);
    void (*SetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, const jint* buf);
    void (*GetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, jbyte* buf);
    void (*SetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, const jbyte* buf);
    void (*SetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, const jlong* buf);
    jlongArray (*NewLongArray)(JNIEnv* env, jsize len);
    jlong* (*GetLongArrayElements)(JNIEnv* env, jlongArray array, jboolean* isCopy);
    void (*ReleaseLongArrayElements)(JNIEnv* env, jlongArray array, jlong* elems, jint mode);
    const char* (*GetStringUTFChars)(JNIEnv* env, jstring str, jboolean* isCopy);
    void (*ReleaseStringUTFChars)(JNIEnv* env, jstring str, const char* chars);
    void (*GetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, jlong* buf);
};

#endif
