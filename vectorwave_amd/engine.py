"""Device engine: one C-ABI context per GPU, array plumbing for numpy (host) and torch (device).

numpy inputs go through the engine's host-memory path (VW_FLAG_HOST_MEMORY: staged H2D, computed,
copied back -- what a JNI caller gets); torch CUDA tensors are passed as device pointers and the
work is enqueued on torch's current stream, so results stay resident in HBM.

Nothing here computes on the CPU: every transform is a call into libvectorwave_amd.so.
"""
from __future__ import annotations

import ctypes
import threading
from ctypes import byref, c_double, c_int64, c_void_p
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _native as nat
from .errors import raise_for_status

try:  # torch is plumbing only (device memory, streams); optional for host-memory use
    import torch
except Exception:  # pragma: no cover
    torch = None


def _is_device_tensor(a) -> bool:
    return torch is not None and isinstance(a, torch.Tensor) and a.is_cuda


def _check(status: int) -> None:
    if status != 0:
        raise_for_status(status, nat.last_error(), nat.last_error_index())


class Engine:
    """Per-device context (vw_ctx).  ``Engine.get(device)`` returns the process-wide instance."""

    _instances = {}
    _lock = threading.Lock()

    def __init__(self, device: int = 0):
        self.lib = nat.load()
        self.device = device
        ctx = c_void_p()
        _check(self.lib.vw_ctx_create(device, byref(ctx)))
        self.ctx = ctx
        self._ext_stream = None
        self._keep = None   # during capture(): device tensors the recorded calls allocate or convert

    @classmethod
    def get(cls, device: Optional[int] = None) -> "Engine":
        if device is None:
            device = torch.cuda.current_device() if (torch is not None and torch.cuda.is_available()) else 0
        with cls._lock:
            eng = cls._instances.get(device)
            if eng is None:
                eng = cls(device)
                cls._instances[device] = eng
            return eng

    def close(self) -> None:
        """Destroy this context (vw_ctx_destroy: drains its stream, invalidates its graphs).  Not for the
        shared instance of ``Engine.get``."""
        if self.ctx:
            with Engine._lock:
                if Engine._instances.get(self.device) is self:
                    del Engine._instances[self.device]
            _check(self.lib.vw_ctx_destroy(self.ctx))
            self.ctx = None

    # -- streams ------------------------------------------------------------------------------
    def bind_torch_stream(self) -> None:
        """Enqueue on torch's current stream of this device (orders engine work with torch ops)."""
        s = torch.cuda.current_stream(self.device).cuda_stream
        if s != self._ext_stream:
            # torch's default stream has handle 0 (the null stream), which vw_ctx_set_stream would read
            # as "use your own stream" -- unordered with torch's work
            _check(self.lib.vw_ctx_use_null_stream(self.ctx) if s == 0 else
                   self.lib.vw_ctx_set_stream(self.ctx, c_void_p(s)))
            self._ext_stream = s

    def set_option(self, key: str, value: int) -> None:
        """Kernel-path switch of this context (vw_ctx_set_option); value < 0 = default."""
        _check(self.lib.vw_ctx_set_option(self.ctx, key.encode(), int(value)))

    def options(self, **kv):
        """Context manager: set switches (VW_... = int) for the block, restore the defaults after."""
        import contextlib

        @contextlib.contextmanager
        def cm():
            for k, v in kv.items():
                self.set_option(k, v)
            try:
                yield self
            finally:
                for k in kv:
                    self.set_option(k, -1)
        return cm()

    def synchronize(self) -> None:
        _check(self.lib.vw_ctx_synchronize(self.ctx))

    def enable_timing(self, on: bool = True) -> None:
        _check(self.lib.vw_ctx_enable_timing(self.ctx, 1 if on else 0))

    def reset_timing(self) -> None:
        _check(self.lib.vw_ctx_reset_timing(self.ctx))

    def kernel_time(self, family: str) -> Tuple[float, int]:
        ms = c_double()
        n = c_int64()
        _check(self.lib.vw_ctx_kernel_time(self.ctx, family.encode(), byref(ms), byref(n)))
        return ms.value, n.value

    def kernel_spans(self, family: str, ref_event, max_n: int = 4096):
        """[(start_ms, end_ms)] of the uncollected timed launches of `family`, relative to `ref_event`
        (a torch.cuda.Event recorded before them); call before kernel_time (vw_ctx_kernel_spans)."""
        st = (c_double * max_n)()
        en = (c_double * max_n)()
        n = c_int64()
        _check(self.lib.vw_ctx_kernel_spans(self.ctx, family.encode(), c_void_p(ref_event.cuda_event), max_n, st, en,
                                            byref(n)))
        return [(st[i], en[i]) for i in range(min(n.value, max_n))]

    # -- array helpers ------------------------------------------------------------------------
    def _prep(self, x, dtype=None):
        """Returns (array, is_device, ptr, dtype_is_f32)."""
        if _is_device_tensor(x):
            # an f64-only entry point (dtype=float64) must never get an f32 buffer: the kernel would
            # read and write 8-byte elements over a 4-byte allocation
            if dtype is not None:
                want = torch.float32 if np.dtype(dtype) == np.float32 else torch.float64
                if x.dtype != want:
                    x = x.to(want)
            elif x.dtype not in (torch.float64, torch.float32):
                x = x.to(torch.float64)
            if not x.is_contiguous():
                x = x.contiguous()
            if x.device.index != self.device:
                raise ValueError(f"tensor on cuda:{x.device.index}, engine on cuda:{self.device}")
            self.bind_torch_stream()
            if self._keep is not None:
                self._keep.append(x)   # a recorded graph reads this storage on every replay
            return x, True, c_void_p(x.data_ptr()), x.dtype == torch.float32
        if torch is not None and isinstance(x, torch.Tensor):
            x = x.detach().numpy()
        a = np.asarray(x)
        if dtype is None:
            dtype = np.float32 if a.dtype == np.float32 else np.float64
        a = np.ascontiguousarray(a, dtype=dtype)
        return a, False, a.ctypes.data_as(c_void_p), a.dtype == np.float32

    def _empty(self, like, is_dev, shape):
        if is_dev:
            t = torch.empty(shape, dtype=like.dtype, device=like.device)
            if self._keep is not None:
                self._keep.append(t)   # a recorded graph writes this storage on every replay
            return t
        return np.empty(shape, dtype=like.dtype)

    @staticmethod
    def _ptr(a, is_dev):
        if a is None:
            return None
        return c_void_p(a.data_ptr()) if is_dev else a.ctypes.data_as(c_void_p)

    @staticmethod
    def _flags(flags: int, is_dev: bool) -> int:
        return flags if is_dev else flags | nat.FLAG_HOST_MEMORY

    # -- transforms ---------------------------------------------------------------------------
    def forward(self, x, lo: Sequence[float], hi: Sequence[float], wavelet_id: int, boundary: int, levels: int,
                flags: int):
        """Multi-level forward.  x: [N] or [B,N] -> (details [J,(B,)N], approx [(B,)N])."""
        xa, dev, xp, f32 = self._prep(x)
        one = xa.ndim == 1
        B, N = (1, xa.shape[0]) if one else xa.shape
        det = self._empty(xa, dev, (levels, N) if one else (levels, B, N))
        app = self._empty(xa, dev, (N,) if one else (B, N))
        fn = self.lib.vw_modwt_forward_f32 if f32 else self.lib.vw_modwt_forward_f64
        _check(fn(self.ctx, xp, B, N, N, nat.taps_array(lo), nat.taps_array(hi), len(lo), wavelet_id, boundary,
                  levels, self._flags(flags, dev), self._ptr(det, dev), self._ptr(app, dev)))
        return det, app

    def inverse(self, details, approx, lo, hi, wavelet_id: int, boundary: int, levels: int, flags: int,
                detail_mask: int = 0xFFFFFFFF, approx_zero: bool = False, shape=None):
        ref = approx if approx is not None else details
        ra, dev, _, f32 = self._prep(ref)
        da = dp = None
        if details is not None:
            da, _, dp, _ = self._prep(details, np.float32 if f32 else np.float64)
        aa = ap = None
        if approx is not None:
            aa, _, ap, _ = self._prep(approx, np.float32 if f32 else np.float64)
        if shape is None:
            shape = tuple(aa.shape if aa is not None else da.shape[1:])
        one = len(shape) == 1
        B, N = (1, shape[0]) if one else shape
        y = self._empty(ra, dev, shape)
        fn = self.lib.vw_modwt_inverse_f32 if f32 else self.lib.vw_modwt_inverse_f64
        _check(fn(self.ctx, dp, ap, B, N, nat.taps_array(lo), nat.taps_array(hi), len(lo), wavelet_id, boundary, levels,
                  detail_mask & 0xFFFFFFFF, 1 if approx_zero else 0, self._flags(flags, dev), self._ptr(y, dev)))
        return y

    def forward1(self, x, lo, hi, boundary: int, flags: int):
        xa, dev, xp, f32 = self._prep(x, np.float64)
        one = xa.ndim == 1
        B, N = (1, xa.shape[0]) if one else xa.shape
        app = self._empty(xa, dev, xa.shape)
        det = self._empty(xa, dev, xa.shape)
        _check(self.lib.vw_modwt1_forward_f64(self.ctx, xp, B, N, N, nat.taps_array(lo), nat.taps_array(hi), len(lo),
                                              boundary, self._flags(flags, dev), self._ptr(app, dev),
                                              self._ptr(det, dev)))
        return app, det

    def inverse1(self, approx, detail, lo, hi, boundary: int, flags: int):
        aa, dev, ap, _ = self._prep(approx, np.float64)
        da, _, dp, _ = self._prep(detail, np.float64)
        one = aa.ndim == 1
        B, N = (1, aa.shape[0]) if one else aa.shape
        y = self._empty(aa, dev, aa.shape)
        _check(self.lib.vw_modwt1_inverse_f64(self.ctx, ap, dp, B, N, nat.taps_array(lo), nat.taps_array(hi), len(lo),
                                              boundary, self._flags(flags, dev), self._ptr(y, dev)))
        return y

    def denoise(self, x, lo, hi, wavelet_id: int, boundary: int, levels: int, threshold: float, soft: bool,
                flags: int, want_thresholds: bool = False):
        xa, dev, xp, _ = self._prep(x, np.float64)
        one = xa.ndim == 1
        B, N = (1, xa.shape[0]) if one else xa.shape
        y = self._empty(xa, dev, xa.shape)
        thr = self._empty(xa, dev, (B,)) if want_thresholds else None
        _check(self.lib.vw_swt_denoise_f64(self.ctx, xp, B, N, N, nat.taps_array(lo), nat.taps_array(hi), len(lo),
                                           wavelet_id, boundary, levels, float(threshold), 1 if soft else 0,
                                           self._flags(flags, dev), self._ptr(y, dev), self._ptr(thr, dev)))
        return (y, thr) if want_thresholds else y

    def wavelet_denoise(self, x, lo, hi, wavelet_id: int, boundary: int, levels: int, method: int, fixed: float,
                        soft: bool, flags: int, want_thresholds: bool = False):
        """vw_wavelet_denoise_f64 (WaveletDenoiser); thresholds [max(levels,1), B]."""
        xa, dev, xp, _ = self._prep(x, np.float64)
        one = xa.ndim == 1
        B, N = (1, xa.shape[0]) if one else xa.shape
        y = self._empty(xa, dev, xa.shape)
        thr = self._empty(xa, dev, (max(levels, 1), B)) if want_thresholds else None
        _check(self.lib.vw_wavelet_denoise_f64(self.ctx, xp, B, N, N, nat.taps_array(lo), nat.taps_array(hi), len(lo),
                                               wavelet_id, boundary, levels, method, float(fixed), 1 if soft else 0,
                                               self._flags(flags, dev), self._ptr(y, dev), self._ptr(thr, dev)))
        return (y, thr) if want_thresholds else y

    def transpose(self, a, rows: int, cols: int):
        """out[c][r] = a[r][c] (a: rows*cols elements, any shape) -> flat [cols*rows] array."""
        aa, dev, ap, f32 = self._prep(a)
        if (aa.numel() if dev else aa.size) != rows * cols:
            raise ValueError("transpose: size mismatch")
        out = self._empty(aa, dev, (rows * cols,))
        fn = self.lib.vw_transpose_f32 if f32 else self.lib.vw_transpose_f64
        _check(fn(self.ctx, ap, rows, cols, self._flags(0, dev), self._ptr(out, dev)))
        return out

    def noise_sigma(self, coeffs):
        ca, dev, cp, _ = self._prep(coeffs, np.float64)
        one = ca.ndim == 1
        B, N = (1, ca.shape[0]) if one else ca.shape
        sig = self._empty(ca, dev, (B,))
        _check(self.lib.vw_noise_sigma_f64(self.ctx, cp, B, N, self._flags(0, dev), self._ptr(sig, dev)))
        return sig

    def threshold_inplace(self, coeffs, thresholds, soft: bool):
        """In-place threshold of a device tensor or numpy array [B,N] (or [N]) with per-row thresholds."""
        ca, dev, cp, _ = self._prep(coeffs, np.float64)
        one = ca.ndim == 1
        B, N = (1, ca.shape[0]) if one else ca.shape
        ta, _, tp, _ = self._prep(thresholds, np.float64)
        _check(self.lib.vw_threshold_f64(self.ctx, cp, B, N, tp, 1 if soft else 0, self._flags(0, dev)))
        if ca is not coeffs:  # _prep made a converted / contiguous copy: write the result back in place
            if dev:
                coeffs.copy_(ca)
            else:
                np.copyto(coeffs, ca)
        return coeffs

    # -- captured steps (vw_capture_begin / vw_capture_end / vw_graph_launch) --------------------
    def capture(self, fn) -> "Graph":
        """Record the engine calls ``fn()`` makes (device tensors, no validation) into one HIP graph.
        The engine must be bound to a non-default torch stream (``bind_torch_stream``).

        Every device tensor the recorded calls allocate (outputs) or convert (inputs made contiguous /
        cast) is kept alive by the returned Graph, so the caching allocator never hands that storage to
        another tensor while replays still write it; ``Graph.result`` is ``fn()``'s return value, whose
        tensors every replay rewrites.  If ``fn()`` raises, the partial graph is destroyed."""
        self.bind_torch_stream()
        _check(self.lib.vw_capture_begin(self.ctx))
        self._keep = []
        done = False
        result = None
        try:
            result = fn()
            done = True
        finally:
            keep, self._keep = self._keep, None
            g = c_void_p()
            st = self.lib.vw_capture_end(self.ctx, byref(g))
            if not done and st == 0:
                self.lib.vw_graph_destroy(g)
        _check(st)
        return Graph(self, g, keep=keep, result=result)

    def fill_uniform(self, x, seed: int, offset: int = 0):
        """Device generator of the bench input: x = 2u-1, u = (splitmix64(seed ^ (offset+i)) >> 11) 2^-53."""
        if not _is_device_tensor(x):
            raise TypeError("fill_uniform needs a CUDA tensor")
        self.bind_torch_stream()
        fn = self.lib.vw_fill_uniform_f32 if x.dtype == torch.float32 else self.lib.vw_fill_uniform_f64
        _check(fn(self.ctx, c_void_p(x.data_ptr()), x.numel(), ctypes.c_uint64(seed), offset))
        return x


class Graph:
    """An executable HIP graph of recorded engine calls; ``launch(count)`` replays it on the stream."""

    def __init__(self, engine: Engine, handle: c_void_p, keep=None, result=None):
        self.engine = engine
        self.handle = handle
        self._keep = keep or []   # storage the recorded kernels read / write (see Engine.capture)
        self.result = result

    def launch(self, count: int = 1) -> None:
        _check(self.engine.lib.vw_graph_launch(self.handle, int(count)))

    def close(self) -> None:
        if self.handle:
            _check(self.engine.lib.vw_graph_destroy(self.handle))
            self.handle = None
        self._keep = []

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def version() -> str:
    return nat.load().vw_version().decode()


def max_levels(N: int, L: int) -> int:
    return int(nat.load().vw_max_levels(N, L))
