package dev.demir.vulkan.engine;

import dev.demir.vulkan.renderer.BuiltCpuData;
import dev.demir.vulkan.renderer.FrameData;
import dev.demir.vulkan.scene.Camera;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.concurrent.ConcurrentLinkedQueue;
import java.util.concurrent.atomic.AtomicReference;
import static org.lwjgl.system.MemoryUtil.memFree;

/**
 * Drop-in for VulkanEngine (VulkanEngine.java:120-185): the same public API and
 * render thread, rendering through jni/HipNative.c into librtamd.so.
 */
public class HipEngine implements Runnable {
    private static final int WIDTH = 1280, HEIGHT = 720, MAX_BOUNCES = 10;   // VulkanEngine.java:45-46, .comp:44
    private volatile boolean isRunning = true;
    private final Thread thread;
    private final AtomicReference<FrameData> frameQueue;
    private final ConcurrentLinkedQueue<BuiltCpuData> sceneQueue = new ConcurrentLinkedQueue<>();
    private final ConcurrentLinkedQueue<Camera> cameraQueue = new ConcurrentLinkedQueue<>();
    private final ConcurrentLinkedQueue<Boolean> skyToggleQueue = new ConcurrentLinkedQueue<>();
    private final ByteBuffer ubo = ByteBuffer.allocateDirect(80).order(ByteOrder.nativeOrder());
    private long ctx = 0;
    private boolean haveScene = false;
    private ByteBuffer[] slots = null;
    private static final int IN_FLIGHT = 4;                               // rt option async_slots (default 4)
    private final long[] tickets = new long[IN_FLIGHT];
    private long submitted = 0;
    private Camera currentCamera = null;
    private int isSkyEnabled = 1;

    public HipEngine(AtomicReference<FrameData> frameQueue) {
        this.frameQueue = frameQueue;
        this.thread = new Thread(this, "HIP-Engine-Thread");
        this.thread.setDaemon(true);
    }
    public void start() { isRunning = true; thread.start(); }
    public void stop() {
        isRunning = false;
        try { thread.join(5000); } catch (InterruptedException e) { Thread.currentThread().interrupt(); }
    }
    public void submitScene(BuiltCpuData d) { sceneQueue.add(d); }
    public void submitCameraUpdate(Camera c) { cameraQueue.add(c); }
    public void submitSkyToggle(boolean on) { skyToggleQueue.add(on); }

    @Override public void run() {
        try {
            ctx = HipNative.create(new int[]{0});
            if (HipNative.getOption(ctx, "queues_short") != 0)             // rtamd.h: async_slots + 2 > hw_queues
                System.err.println("WARN (HIP): GPU_MAX_HW_QUEUES=" + HipNative.getOption(ctx, "hw_queues")
                                   + " is too few for " + IN_FLIGHT + " frames in flight: start the JVM with "
                                   + "GPU_MAX_HW_QUEUES=16, or the frames' traces run one after another");
            while (isRunning) {
                BuiltCpuData d = sceneQueue.poll();                       // one scene per pass (:281-285)
                if (d != null) {
                    HipNative.uploadScene(ctx, memByteBufferOf(d.modelVertexData), d.modelVertexData.remaining() * 4L,
                                          memByteBufferOf(d.modelMaterialData), d.modelMaterialData.remaining() * 4L,
                                          d.flatBvhData, d.flatBvhData.remaining());
                    memFree(d.modelVertexData);                           // as VulkanEngine.java:343,351
                    memFree(d.modelMaterialData);
                    haveScene = true;
                }
                Camera c, latest = null;                                  // drain to the latest (:288-298)
                while ((c = cameraQueue.poll()) != null) latest = c;
                if (latest != null) currentCamera = latest;
                Boolean s, sky = null;
                while ((s = skyToggleQueue.poll()) != null) sky = s;
                if (sky != null) isSkyEnabled = sky ? 1 : 0;
                if (!haveScene || currentCamera == null) { Thread.sleep(16); continue; }
                currentCamera.getOrigin().store(0, ubo);                  // same bytes as :387-395
                currentCamera.getLowerLeft().store(16, ubo);
                currentCamera.getHorizontal().store(32, ubo);
                currentCamera.getVertical().store(48, ubo);
                ubo.putInt(64, currentCamera.getFrameCount());
                ubo.putInt(68, isSkyEnabled);
                // IN_FLIGHT (= the library's async_slots, default 4) frames in
                // flight, each tracing on its own stream: the frames' traces
                // overlap each other and every readback overlaps later traces.
                // Start the JVM with GPU_MAX_HW_QUEUES=16 so each stream gets a
                // hardware queue of its own (HIP's default is 4 per process).
                if (slots == null) {
                    slots = new ByteBuffer[IN_FLIGHT];
                    for (int i = 0; i < IN_FLIGHT; i++) slots[i] = HipNative.allocFrame(WIDTH * HEIGHT * 4L);
                }
                int k = (int)(submitted++ % IN_FLIGHT);
                tickets[k] = HipNative.renderAsync(ctx, ubo, WIDTH, HEIGHT, MAX_BOUNCES, slots[k]);
                if (submitted >= IN_FLIGHT) {
                    int j = (int)(submitted % IN_FLIGHT);                 // the oldest frame in flight
                    HipNative.waitFrame(ctx, tickets[j]);
                    ByteBuffer px = ByteBuffer.allocateDirect(WIDTH * HEIGHT * 4);   // a fresh buffer per frame (:421)
                    px.put(slots[j].duplicate()).flip();
                    frameQueue.set(new FrameData(px));
                }
            }
        } catch (Exception e) {
            System.err.println("FATAL (HIP): HipEngine thread crashed!");
            e.printStackTrace();
            isRunning = false;
        } finally {
            if (ctx != 0) HipNative.destroy(ctx);                         // waits for frames in flight
            if (slots != null) for (ByteBuffer b : slots) HipNative.freeFrame(b);
        }
    }

    private static ByteBuffer memByteBufferOf(java.nio.FloatBuffer f) {
        return org.lwjgl.system.MemoryUtil.memByteBuffer(f);
    }
}
