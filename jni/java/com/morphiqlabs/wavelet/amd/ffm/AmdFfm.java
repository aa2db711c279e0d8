package com.morphiqlabs.wavelet.amd.ffm;

import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.SymbolLookup;
import java.lang.foreign.ValueLayout;
import java.lang.invoke.MethodHandle;
import java.nio.file.Path;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

/**
 * Foreign Function &amp; Memory binding (java.lang.foreign, final since Java 22; vectorwave-extensions targets
 * Java 24) of the engine's C-ABI, include/vectorwave_amd.h -- no JNI glue, no copies: the engine reads and
 * writes the caller's off-heap {@link MemorySegment}s directly (host memory, staged by the engine through
 * its per-context device pool), or device buffers the caller keeps resident across calls
 * ({@link DeviceBatch}: the zero-copy route for batches that stay on the GPU between a forward and an
 * inverse, the north_star hot path).
 *
 * <p>Entry points bound here, each replacing the Java method named in the header's comment:
 * vw_modwt_forward_f64 / vw_modwt_inverse_f64 (MultiLevelMODWTTransform.decompose / reconstruct,
 * BatchMODWT.multiLevelAoS / inverseMultiLevelAoS), vw_swt_denoise_f64 (VectorWaveSwtAdapter.denoise),
 * the pipelined round trips (vw_pipeline_*), context / device-memory utilities.  Status codes are mapped
 * to exceptions by {@link #check(int)} (same table as AmdNative.check, INTEGRATION.md section 3).
 *
 * <p>Not built or run in this repository (no JDK in its build image); the signatures follow the header
 * one to one (int64_t = JAVA_LONG, int / unsigned = JAVA_INT, pointers = ADDRESS).
 */
public final class AmdFfm implements AutoCloseable {
    public static final int FLAG_CORE_LEVELS = 1, FLAG_VALIDATE = 1 << 1, FLAG_FFT_SWITCH = 1 << 2, FLAG_FMA = 1 << 3,
            FLAG_HOST_MEMORY = 1 << 4, FLAG_SYNC = 1 << 5, FLAG_REF_NONFINITE = 1 << 8;
    public static final int PERIODIC = 0, SYMMETRIC = 1, ZERO_PADDING = 2;

    private static final Linker LINKER = Linker.nativeLinker();

    private final SymbolLookup lib;
    private final MethodHandle ctxCreate, ctxDestroy, ctxSync, lastError, forward, inverse, denoise, devAlloc,
            devFree, memcpy, pipeCreate, pipeRun, pipeJoin, pipeDestroy;
    private final MemorySegment ctx;

    /** Loads {@code libvectorwave_amd.so} from {@code libraryPath} and creates a context on {@code device}. */
    public AmdFfm(Path libraryPath, int device) {
        lib = SymbolLookup.libraryLookup(libraryPath, Arena.global());
        ctxCreate = fn("vw_ctx_create", FunctionDescriptor.of(JAVA_INT, JAVA_INT, ADDRESS));
        ctxDestroy = fn("vw_ctx_destroy", FunctionDescriptor.of(JAVA_INT, ADDRESS));
        ctxSync = fn("vw_ctx_synchronize", FunctionDescriptor.of(JAVA_INT, ADDRESS));
        lastError = fn("vw_last_error", FunctionDescriptor.of(ADDRESS));
        // vw_modwt_forward_f64(ctx, x, B, N, ldx, lo, hi, L, wavelet_id, boundary, J, flags, details, approx)
        forward = fn("vw_modwt_forward_f64", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, JAVA_LONG,
                JAVA_LONG, ADDRESS, ADDRESS, JAVA_INT, JAVA_INT, JAVA_INT, JAVA_INT, JAVA_INT, ADDRESS, ADDRESS));
        // vw_modwt_inverse_f64(ctx, details, approx, B, N, lo, hi, L, wavelet_id, boundary, J, detail_mask,
        //                      approx_zero, flags, y)
        inverse = fn("vw_modwt_inverse_f64", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, JAVA_LONG,
                JAVA_LONG, ADDRESS, ADDRESS, JAVA_INT, JAVA_INT, JAVA_INT, JAVA_INT, JAVA_INT, JAVA_INT, JAVA_INT,
                ADDRESS));
        // vw_swt_denoise_f64(ctx, x, B, N, ldx, lo, hi, L, wavelet_id, boundary, J, threshold, soft, flags, y, thr)
        denoise = fn("vw_swt_denoise_f64", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, JAVA_LONG,
                JAVA_LONG, ADDRESS, ADDRESS, JAVA_INT, JAVA_INT, JAVA_INT, JAVA_INT, ValueLayout.JAVA_DOUBLE, JAVA_INT,
                JAVA_INT, ADDRESS, ADDRESS));
        devAlloc = fn("vw_device_alloc", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, ADDRESS));
        devFree = fn("vw_device_free", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
        memcpy = fn("vw_memcpy", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, JAVA_LONG, JAVA_INT));
        // vw_pipeline_create(fwd_ctx, inv_ctx, elem_bytes, sets, x[], details[], approx[], y[], B, N, lo, hi, L,
        //                    wavelet_id, boundary, J, flags, out)
        pipeCreate = fn("vw_pipeline_create", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, JAVA_INT,
                ADDRESS, ADDRESS, ADDRESS, ADDRESS, JAVA_LONG, JAVA_LONG, ADDRESS, ADDRESS, JAVA_INT, JAVA_INT,
                JAVA_INT, JAVA_INT, JAVA_INT, ADDRESS));
        pipeRun = fn("vw_pipeline_run", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG));
        pipeJoin = fn("vw_pipeline_join", FunctionDescriptor.of(JAVA_INT, ADDRESS));
        pipeDestroy = fn("vw_pipeline_destroy", FunctionDescriptor.of(JAVA_INT, ADDRESS));
        try (Arena a = Arena.ofConfined()) {
            MemorySegment out = a.allocate(ADDRESS);
            check((int) ctxCreate.invokeExact(device, out));
            ctx = out.get(ADDRESS, 0);
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    private MethodHandle fn(String name, FunctionDescriptor d) {
        return LINKER.downcallHandle(lib.find(name).orElseThrow(
                () -> new UnsatisfiedLinkError(name + " not exported by libvectorwave_amd.so")), d);
    }

    /**
     * MultiLevelMODWTTransform.decompose / BatchMODWT.multiLevelAoS over B signals of length N in the
     * caller's HOST memory (off-heap segments): x [B][N], details [J][B][N], approx [B][N], row-major
     * doubles.  The engine stages through its device pool and returns when the results are written.
     */
    public void forwardHost(MemorySegment x, long B, long N, double[] lo, double[] hi, int waveletId, int boundary,
                            int J, int flags, MemorySegment details, MemorySegment approx) {
        requireBytes(x, B * N, "x");
        requireBytes(details, J * B * N, "details");
        requireBytes(approx, B * N, "approx");
        try (Arena a = Arena.ofConfined()) {
            check((int) forward.invokeExact(ctx, x, B, N, N, taps(a, lo), taps(a, hi), lo.length, waveletId, boundary,
                    J, flags | FLAG_HOST_MEMORY | FLAG_SYNC, details, approx));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    /** MultiLevelMODWTTransform.reconstruct over host segments (details [J][B][N], approx [B][N] -> y [B][N]). */
    public void inverseHost(MemorySegment details, MemorySegment approx, long B, long N, double[] lo, double[] hi,
                            int waveletId, int boundary, int J, int flags, MemorySegment y) {
        requireBytes(details, J * B * N, "details");
        requireBytes(approx, B * N, "approx");
        requireBytes(y, B * N, "y");
        try (Arena a = Arena.ofConfined()) {
            check((int) inverse.invokeExact(ctx, details, approx, B, N, taps(a, lo), taps(a, hi), lo.length, waveletId,
                    boundary, J, -1, 0, flags | FLAG_HOST_MEMORY | FLAG_SYNC, y));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    /** VectorWaveSwtAdapter.denoise over host segments; thresholdsOut (B doubles) may be NULL. */
    public void denoiseHost(MemorySegment x, long B, long N, double[] lo, double[] hi, int waveletId, int boundary,
                            int J, double threshold, boolean soft, int flags, MemorySegment y,
                            MemorySegment thresholdsOut) {
        requireBytes(x, B * N, "x");
        requireBytes(y, B * N, "y");
        try (Arena a = Arena.ofConfined()) {
            check((int) denoise.invokeExact(ctx, x, B, N, N, taps(a, lo), taps(a, hi), lo.length, waveletId, boundary, J,
                    threshold, soft ? 1 : 0, flags | FLAG_HOST_MEMORY | FLAG_SYNC, y,
                    thresholdsOut == null ? MemorySegment.NULL : thresholdsOut));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    /**
     * A batch resident on the device: x [B][N], details [J][B][N], approx [B][N], y [B][N] allocated once;
     * {@link #upload} / {@link #download} move data, {@link #forward} / {@link #inverse} run on the device
     * buffers with no staging (asynchronous on the context's stream; {@link #synchronize} waits).
     */
    public final class DeviceBatch implements AutoCloseable {
        public final long B, N;
        public final int J;
        final MemorySegment x, det, app, y;

        DeviceBatch(long B, long N, int J) {
            this.B = B;
            this.N = N;
            this.J = J;
            x = alloc(B * N * 8);
            det = alloc(J * B * N * 8);
            app = alloc(B * N * 8);
            y = alloc(B * N * 8);
        }

        public void upload(MemorySegment hostX) {
            requireBytes(hostX, B * N, "x");
            copy(x, hostX, B * N * 8, 0);
        }

        public void forward(double[] lo, double[] hi, int waveletId, int boundary, int flags) {
            try (Arena a = Arena.ofConfined()) {
                check((int) forward.invokeExact(ctx, x, B, N, N, taps(a, lo), taps(a, hi), lo.length, waveletId,
                        boundary, J, flags & ~(FLAG_HOST_MEMORY | FLAG_SYNC), det, app));
                // the engine reads the taps during the call (kernel arguments), so `a` may close now
            } catch (Throwable t) {
                throw rethrow(t);
            }
        }

        public void inverse(double[] lo, double[] hi, int waveletId, int boundary, int flags) {
            try (Arena a = Arena.ofConfined()) {
                check((int) inverse.invokeExact(ctx, det, app, B, N, taps(a, lo), taps(a, hi), lo.length, waveletId,
                        boundary, J, -1, 0, flags & ~(FLAG_HOST_MEMORY | FLAG_SYNC), y));
            } catch (Throwable t) {
                throw rethrow(t);
            }
        }

        /** Reconstructed signals y [B][N] into host memory. */
        public void download(MemorySegment hostY) {
            requireBytes(hostY, B * N, "y");
            copy(hostY, y, B * N * 8, 1);
        }

        /** Details [J][B][N] and approximation [B][N] into host memory. */
        public void downloadCoefficients(MemorySegment hostDetails, MemorySegment hostApprox) {
            requireBytes(hostDetails, J * B * N, "details");
            requireBytes(hostApprox, B * N, "approx");
            copy(hostDetails, det, J * B * N * 8, 1);
            copy(hostApprox, app, B * N * 8, 1);
        }

        @Override
        public void close() {
            for (MemorySegment p : new MemorySegment[] {x, det, app, y}) free(p);
        }
    }

    /** Waits for everything enqueued on this context (vw_ctx_synchronize). */
    public void synchronize() {
        try {
            check((int) ctxSync.invokeExact(ctx));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    public DeviceBatch deviceBatch(long B, long N, int J) {
        return new DeviceBatch(B, N, J);
    }

    /**
     * Pipelined round trips over R device batches (vw_pipeline_*): step i = forward then inverse of batch
     * i mod R, step i + 1's forward overlapping step i's inverse, every step issued by the engine.  Uses
     * this context for the forwards and {@code inverseCtx} (another AmdFfm on the same device) for the
     * inverses.  Returns a handle for {@link #pipelineRun} / {@link #pipelineJoin} / {@link #pipelineClose}.
     */
    public MemorySegment pipeline(AmdFfm inverseCtx, DeviceBatch[] sets, double[] lo, double[] hi, int waveletId,
                                  int boundary, int flags) {
        final int R = sets.length;
        try (Arena a = Arena.ofConfined()) {
            MemorySegment xs = a.allocate(ADDRESS, R), ds = a.allocate(ADDRESS, R), as = a.allocate(ADDRESS, R),
                    ys = a.allocate(ADDRESS, R), out = a.allocate(ADDRESS);
            for (int r = 0; r < R; r++) {
                xs.setAtIndex(ADDRESS, r, sets[r].x);
                ds.setAtIndex(ADDRESS, r, sets[r].det);
                as.setAtIndex(ADDRESS, r, sets[r].app);
                ys.setAtIndex(ADDRESS, r, sets[r].y);
            }
            check((int) pipeCreate.invokeExact(ctx, inverseCtx.ctx, 8, R, xs, ds, as, ys, sets[0].B, sets[0].N,
                    taps(a, lo), taps(a, hi), lo.length, waveletId, boundary, sets[0].J, flags, out));
            return out.get(ADDRESS, 0);
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    public void pipelineRun(MemorySegment p, long steps) {
        try {
            check((int) pipeRun.invokeExact(p, steps));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    public void pipelineJoin(MemorySegment p) {
        try {
            check((int) pipeJoin.invokeExact(p));
            check((int) ctxSync.invokeExact(ctx));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    public void pipelineClose(MemorySegment p) {
        try {
            check((int) pipeDestroy.invokeExact(p));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    private MemorySegment alloc(long bytes) {
        try (Arena a = Arena.ofConfined()) {
            MemorySegment out = a.allocate(ADDRESS);
            check((int) devAlloc.invokeExact(ctx, bytes, out));
            return out.get(ADDRESS, 0);
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    private void free(MemorySegment p) {
        try {
            check((int) devFree.invokeExact(ctx, p));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    private void copy(MemorySegment dst, MemorySegment src, long bytes, int kind) {
        try {
            check((int) memcpy.invokeExact(ctx, dst, src, bytes, kind));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    private static MemorySegment taps(Arena a, double[] t) {
        MemorySegment s = a.allocate(ValueLayout.JAVA_DOUBLE, t.length);
        MemorySegment.copy(t, 0, s, ValueLayout.JAVA_DOUBLE, 0, t.length);
        return s;
    }

    private static void requireBytes(MemorySegment s, long doubles, String what) {
        if (s == null) throw new NullPointerException(what + " cannot be null");
        if (s.byteSize() < doubles * 8) {
            throw new IllegalArgumentException(what + " holds " + s.byteSize() + " bytes, needs " + doubles * 8);
        }
    }

    /** include/vectorwave_amd.h status -> the exception the reference throws for the same condition. */
    private void check(int st) {
        if (st == 0) return;
        String msg;
        try {
            msg = ((MemorySegment) lastError.invokeExact()).reinterpret(4096).getString(0);
        } catch (Throwable t) {
            msg = "status " + st;
        }
        switch (st) {
            case 1: throw new NullPointerException(msg);
            case 2: case 3: case 4: case 5: case 6: case 7: throw new IllegalArgumentException(msg + " [status " + st + "]");
            case 9: throw new UnsupportedOperationException(msg);
            case 10: throw new IllegalStateException(msg);
            default: throw new RuntimeException(msg + " [status " + st + "]");
        }
    }

    private static RuntimeException rethrow(Throwable t) {
        if (t instanceof RuntimeException r) return r;
        if (t instanceof Error e) throw e;
        return new RuntimeException(t);
    }

    @Override
    public void close() {
        try {
            check((int) ctxDestroy.invokeExact(ctx));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }
}
