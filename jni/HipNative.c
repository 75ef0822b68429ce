/*
 * HipNative.c — JNI shim between the Java host (dev.demir.vulkan.engine.HipEngine)
 * and the C ABI of librtamd.so (include/rtamd.h).  It replaces the LWJGL-Vulkan
 * calls VulkanEngine makes for the render path (VulkanEngine.java:120-185,
 * 318-431): direct buffers go to the C ABI as plain pointers, a non-zero
 * status becomes a RuntimeException carrying rt_last_error(), as the
 * reference's Vulkan errors are (e.g. VulkanEngine.java:596-598).
 *
 * Build (a host with a JDK; none exists in this repo's build image):
 *   make -C jni JAVA_HOME=/path/to/jdk
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include "rtamd.h"

static void throw_rt(JNIEnv* env, int rc) {
    jclass ex = (*env)->FindClass(env, "java/lang/RuntimeException");
    char msg[1200];
    snprintf(msg, sizeof msg, "rtamd error %d: %s", rc, rt_last_error());
    (*env)->ThrowNew(env, ex, msg);
}

/* long create(int[] deviceIds) */
JNIEXPORT jlong JNICALL Java_dev_demir_vulkan_engine_HipNative_create(JNIEnv* env, jclass c, jintArray ids) {
    /* the library must have this shim's struct layouts (rtamd.h RT_ABI_VERSION) */
    size_t sb = 0, cb = 0;
    if (rt_abi_version(&sb, &cb) != RT_ABI_VERSION || sb != sizeof(rt_stats) || cb != sizeof(rt_camera_ubo)) {
        jclass ex = (*env)->FindClass(env, "java/lang/RuntimeException");
        if (ex) (*env)->ThrowNew(env, ex, "librtamd ABI version differs from the shim's (include/rtamd.h)");
        return 0;
    }
    jsize n = (*env)->GetArrayLength(env, ids);
    jint* p = (*env)->GetIntArrayElements(env, ids, NULL);
    rt_ctx* ctx = NULL;
    int rc = rt_create((const int*)p, (int)n, &ctx);
    (*env)->ReleaseIntArrayElements(env, ids, p, JNI_ABORT);
    if (rc) { throw_rt(env, rc); return 0; }
    return (jlong)(intptr_t)ctx;
}

/* void uploadScene(long ctx, ByteBuffer v, long vBytes, ByteBuffer m, long mBytes, ByteBuffer bvh, long bvhBytes)
 * Direct buffers only (LWJGL memAllocFloat / ByteBuffer.allocateDirect, as SceneBuilder makes them).
 * Byte counts are remaining()*4 / remaining(), as VulkanEngine.java:337,345,353 computes them. */
JNIEXPORT void JNICALL Java_dev_demir_vulkan_engine_HipNative_uploadScene(JNIEnv* env, jclass c, jlong ctx,
        jobject v, jlong vb, jobject m, jlong mb, jobject bvh, jlong bb) {
    int rc = rt_upload_scene((rt_ctx*)(intptr_t)ctx,
                             (*env)->GetDirectBufferAddress(env, v), (size_t)vb,
                             (*env)->GetDirectBufferAddress(env, m), (size_t)mb,
                             (*env)->GetDirectBufferAddress(env, bvh), (size_t)bb);
    if (rc) throw_rt(env, rc);
}

/* void render(long ctx, ByteBuffer ubo80, int w, int h, int maxBounces, ByteBuffer outRgba) */
JNIEXPORT void JNICALL Java_dev_demir_vulkan_engine_HipNative_render(JNIEnv* env, jclass c, jlong ctx,
        jobject ubo, jint w, jint h, jint maxBounces, jobject out) {
    int rc = rt_render((rt_ctx*)(intptr_t)ctx, (const rt_camera_ubo*)(*env)->GetDirectBufferAddress(env, ubo),
                       w, h, maxBounces, (uint8_t*)(*env)->GetDirectBufferAddress(env, out), NULL, NULL);
    if (rc) throw_rt(env, rc);
}

/* Pipelined frames: pinned frame buffers the copy stream writes asynchronously. */
JNIEXPORT jobject JNICALL Java_dev_demir_vulkan_engine_HipNative_allocFrame(JNIEnv* env, jclass c, jlong bytes) {
    void* p = rt_host_alloc((size_t)bytes);
    if (!p) { throw_rt(env, RT_ERR_OOM); return NULL; }
    return (*env)->NewDirectByteBuffer(env, p, bytes);
}
JNIEXPORT void JNICALL Java_dev_demir_vulkan_engine_HipNative_freeFrame(JNIEnv* env, jclass c, jobject buf) {
    rt_host_free((*env)->GetDirectBufferAddress(env, buf));
}
/* long renderAsync(long ctx, ByteBuffer ubo80, int w, int h, int maxBounces, ByteBuffer pinnedOut) */
JNIEXPORT jlong JNICALL Java_dev_demir_vulkan_engine_HipNative_renderAsync(JNIEnv* env, jclass c, jlong ctx,
        jobject ubo, jint w, jint h, jint maxBounces, jobject out) {
    uint64_t t = 0;
    int rc = rt_render_async((rt_ctx*)(intptr_t)ctx, (const rt_camera_ubo*)(*env)->GetDirectBufferAddress(env, ubo),
                             w, h, maxBounces, (uint8_t*)(*env)->GetDirectBufferAddress(env, out), &t);
    if (rc) throw_rt(env, rc);
    return (jlong)t;
}
JNIEXPORT void JNICALL Java_dev_demir_vulkan_engine_HipNative_waitFrame(JNIEnv* env, jclass c, jlong ctx, jlong t) {
    int rc = rt_render_wait((rt_ctx*)(intptr_t)ctx, (uint64_t)t);
    if (rc) throw_rt(env, rc);
}
/* boolean pollFrame(long ctx, long ticket): true when the frame is complete (never blocks) */
JNIEXPORT jboolean JNICALL Java_dev_demir_vulkan_engine_HipNative_pollFrame(JNIEnv* env, jclass c, jlong ctx, jlong t) {
    int done = 0;
    int rc = rt_render_poll((rt_ctx*)(intptr_t)ctx, (uint64_t)t, &done);
    if (rc) { throw_rt(env, rc); return JNI_FALSE; }
    return done ? JNI_TRUE : JNI_FALSE;
}

/* Extension: void uploadSpheres(long ctx, float[] spheres8n) — centre.xyz, radius, albedo.rgb, type per sphere.
 * Then setOption(ctx, "extensions", 8) turns them on. */
JNIEXPORT void JNICALL Java_dev_demir_vulkan_engine_HipNative_uploadSpheres(JNIEnv* env, jclass c, jlong ctx,
        jfloatArray s) {
    jsize n = (*env)->GetArrayLength(env, s);
    jfloat* p = (*env)->GetFloatArrayElements(env, s, NULL);
    int rc = rt_upload_spheres((rt_ctx*)(intptr_t)ctx, (const float*)p, (int)(n / 8));
    (*env)->ReleaseFloatArrayElements(env, s, p, JNI_ABORT);
    if (rc) throw_rt(env, rc);
}

/* void setOption(long ctx, String name, long value) — schedule and extension options (rtamd.h rt_set_option) */
JNIEXPORT void JNICALL Java_dev_demir_vulkan_engine_HipNative_setOption(JNIEnv* env, jclass c, jlong ctx,
        jstring name, jlong value) {
    const char* n = (*env)->GetStringUTFChars(env, name, NULL);
    int rc = rt_set_option((rt_ctx*)(intptr_t)ctx, n, (int64_t)value);
    (*env)->ReleaseStringUTFChars(env, name, n);
    if (rc) throw_rt(env, rc);
}

/* long getOption(long ctx, String name) — e.g. "queues_short": 1 when the async slots lack hardware queues */
JNIEXPORT jlong JNICALL Java_dev_demir_vulkan_engine_HipNative_getOption(JNIEnv* env, jclass c, jlong ctx,
        jstring name) {
    const char* n = (*env)->GetStringUTFChars(env, name, NULL);
    int64_t v = 0;
    int rc = rt_get_option((rt_ctx*)(intptr_t)ctx, n, &v);
    (*env)->ReleaseStringUTFChars(env, name, n);
    if (rc) throw_rt(env, rc);
    return (jlong)v;
}

JNIEXPORT void JNICALL Java_dev_demir_vulkan_engine_HipNative_destroy(JNIEnv* env, jclass c, jlong ctx) {
    rt_destroy((rt_ctx*)(intptr_t)ctx);
}
