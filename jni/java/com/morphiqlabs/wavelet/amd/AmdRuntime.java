package com.morphiqlabs.wavelet.amd;

/**
 * The JVM's engine context: one vw_ctx on device {@code vectorwave.amd.device} (default 0), created on
 * first use and destroyed at JVM exit.  Every facade of this package ({@link AmdBatchMODWT},
 * {@link AmdMultiLevelMODWT}, {@link AmdSwt}, {@link AmdMODWTOptimizer}) enqueues on it; the engine
 * serialises the calls of one context, so the facades are thread-safe.
 *
 * <p>Accumulation: EXACT by default (separate multiply and add in the reference's tap order, results
 * bit-identical to vectorwave-core's scalar path); {@code -Dvectorwave.amd.fma=true} selects fused
 * multiply-add (max-abs error below 1e-12, the engine's fastest mode).
 */
public final class AmdRuntime {
    static final int DEVICE = Integer.getInteger("vectorwave.amd.device", 0);
    static final int FMA = Boolean.getBoolean("vectorwave.amd.fma") ? AmdNative.FLAG_FMA : 0;

    private AmdRuntime() {}

    private static final class Holder {
        static final long CTX = AmdNative.LOADED ? AmdNative.ctxCreate(DEVICE) : 0L;

        static {
            if (CTX != 0L) {
                Runtime.getRuntime().addShutdownHook(new Thread(() -> AmdNative.ctxDestroy(CTX)));
            }
        }
    }

    /** True when the native library loaded and a context exists on the configured device. */
    public static boolean isAvailable() {
        try {
            return AmdNative.LOADED && Holder.CTX != 0L;
        } catch (Throwable t) {
            return false;
        }
    }

    /** The context handle; throws IllegalStateException when the engine is unavailable. */
    static long ctx() {
        if (!isAvailable()) {
            throw new IllegalStateException("vectorwave_amd engine unavailable (library not loaded or no device "
                    + DEVICE + ")");
        }
        return Holder.CTX;
    }

    /** Device number of the context. */
    public static int device() {
        return DEVICE;
    }
}
