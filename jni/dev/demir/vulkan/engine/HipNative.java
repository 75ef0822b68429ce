package dev.demir.vulkan.engine;

import java.nio.ByteBuffer;

/** JNI entry points of jni/HipNative.c over librtamd.so (include/rtamd.h). */
final class HipNative {
    static { System.loadLibrary("hipnative"); }
    static native long create(int[] deviceIds);
    static native void uploadScene(long ctx, ByteBuffer v, long vBytes, ByteBuffer m, long mBytes,
                                   ByteBuffer bvh, long bvhBytes);
    static native void render(long ctx, ByteBuffer ubo80, int w, int h, int maxBounces, ByteBuffer outRgba);
    static native void destroy(long ctx);
    static native ByteBuffer allocFrame(long bytes);            // pinned (rt_host_alloc)
    static native void freeFrame(ByteBuffer frame);
    static native long renderAsync(long ctx, ByteBuffer ubo80, int w, int h, int maxBounces, ByteBuffer pinnedOut);
    static native void waitFrame(long ctx, long ticket);
    static native boolean pollFrame(long ctx, long ticket);       // rt_render_poll: never blocks
    static native void uploadSpheres(long ctx, float[] spheres8n);   // extension (option "extensions" bit 8)
    static native void setOption(long ctx, String name, long value);
    static native long getOption(long ctx, String name);
}
