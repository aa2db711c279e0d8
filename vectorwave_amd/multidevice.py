"""One batch over several device contexts, one host thread per context.

The reference parallelises a single batch call inside one JVM (BatchMODWT.multiLevelAoS over the
batch, ext/extensions/modwt/BatchMODWT.java:90-111; the VectorWaveSwtAdapter executor,
core/swt/VectorWaveSwtAdapter.java:210-267).  ``DeviceGroup`` is that call spread over GPUs: the batch
is split into contiguous row blocks (``shard.shard_rows``), block k runs on context k from its own
host thread, with no exchange between devices.

* Host arrays (numpy, the JNI/FFM caller's ``double[][]``): one C call,
  ``vw_modwt_forward_multi_f64`` / ``vw_modwt_inverse_multi_f64``, whose std::threads stage each
  block through its own context.
* Device tensors (one per context, already on that context's device): one C call,
  ``vw_modwt_forward_multi_dev_f64`` / ``vw_modwt_inverse_multi_dev_f64``, whose std::threads enqueue
  each shard on its own context's stream -- no staging, nothing crosses PCIe.

Contexts may share a device (several ``Engine`` instances on cuda:0 -- what the tests do on a one-GPU
box) or sit on different devices.
"""
from __future__ import annotations

import ctypes
from ctypes import c_void_p
from typing import List, Optional, Sequence

import numpy as np

from . import _native as nat
from .engine import Engine, _check
from .errors import InvalidArgumentException
from .shard import shard_rows
from .wavelets import Wavelet


class DeviceGroup:
    """``DeviceGroup(devices=[0, 1, ...])``: one context per entry (repeat a device for several contexts
    on it).  ``forward`` / ``inverse`` take a whole host batch and return whole host arrays."""

    def __init__(self, devices: Sequence[int] = (0,), engines: Optional[List[Engine]] = None):
        self.engines = list(engines) if engines else [Engine(d) for d in devices]
        if not self.engines:
            raise InvalidArgumentException("DeviceGroup needs at least one context")
        self._own = engines is None
        self._ctxs = (c_void_p * len(self.engines))(*[e.ctx.value for e in self.engines])

    def __len__(self) -> int:
        return len(self.engines)

    def blocks(self, B: int):
        """Row blocks [(start, rows)] in context order (min(len, B) of them)."""
        n = min(len(self.engines), B)
        return [shard_rows(B, n, k) for k in range(n)]

    # -- host batch: one C call, one std::thread per context ------------------------------------
    def forward(self, x, wavelet: Wavelet, levels: int, boundary: int = nat.PERIODIC, fma: bool = False,
                core_levels: bool = False):
        """x [B][N] host -> (details [J][B][N], approx [B][N]) host (BatchMODWT.multiLevelAoS semantics;
        ``core_levels``: MultiLevelMODWTTransform's level cap)."""
        a = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
        if a.ndim != 2 or a.shape[0] == 0 or a.shape[1] == 0:
            raise InvalidArgumentException("signals must be a non-empty [batch][length] array")
        B, N = a.shape
        det = np.empty((levels, B, N))
        app = np.empty((B, N))
        lo, hi = wavelet.lowPassDecomposition(), wavelet.highPassDecomposition()
        flags = nat.FLAG_HOST_MEMORY | (nat.FLAG_FMA if fma else 0) | (nat.FLAG_CORE_LEVELS if core_levels else 0)
        lib = nat.load()
        _check(lib.vw_modwt_forward_multi_f64(self._ctxs, len(self.engines), a.ctypes.data_as(c_void_p), B, N, N,
                                              nat.taps_array(lo), nat.taps_array(hi), len(lo), wavelet.wavelet_id,
                                              boundary, levels, flags, det.ctypes.data_as(c_void_p),
                                              app.ctypes.data_as(c_void_p)))
        return det, app

    def inverse(self, details, approx, wavelet: Wavelet, boundary: int = nat.PERIODIC, fma: bool = False):
        """details [J][B][N], approx [B][N] host -> y [B][N] host (MultiLevelMODWTTransform.reconstruct)."""
        d = np.ascontiguousarray(np.asarray(details, dtype=np.float64))
        ap = np.ascontiguousarray(np.asarray(approx, dtype=np.float64))
        if d.ndim != 3 or tuple(d.shape[1:]) != tuple(ap.shape):
            raise InvalidArgumentException("details must be [levels][batch][length] matching approx")
        J, B, N = d.shape
        y = np.empty((B, N))
        lo, hi = wavelet.lowPassReconstruction(), wavelet.highPassReconstruction()
        flags = nat.FLAG_HOST_MEMORY | (nat.FLAG_FMA if fma else 0)
        _check(nat.load().vw_modwt_inverse_multi_f64(self._ctxs, len(self.engines), d.ctypes.data_as(c_void_p),
                                                     ap.ctypes.data_as(c_void_p), B, N, nat.taps_array(lo),
                                                     nat.taps_array(hi), len(lo), wavelet.wavelet_id, boundary, J,
                                                     0xFFFFFFFF, 0, flags, y.ctypes.data_as(c_void_p)))
        return y

    # -- device tensors: one C call, one std::thread per context, no staging ----------------------
    def _dev_ptrs(self, ts):
        return (c_void_p * len(self.engines))(*[t.data_ptr() for t in ts])

    def _sync_devices(self):
        import torch
        for d in sorted({e.device for e in self.engines}):
            torch.cuda.synchronize(d)

    def forward_device(self, xs, wavelet: Wavelet, levels: int, boundary: int = nat.PERIODIC, fma: bool = False,
                       core_levels: bool = False):
        """xs: one [B_k][N] float64 CUDA tensor per context, on that context's device (a batch already
        sharded across GPUs) -> [(details [J][B_k][N], approx [B_k][N])], allocated on the same devices.
        One ``vw_modwt_forward_multi_dev_f64`` call: context k's host thread enqueues its shard on its own
        stream, nothing crosses PCIe; returns when every shard is done."""
        import torch
        if len(xs) != len(self.engines):
            raise InvalidArgumentException("one tensor per context")
        xs = [x.contiguous() for x in xs]
        N = xs[0].shape[-1]
        for k, x in enumerate(xs):
            if x.dtype != torch.float64 or x.ndim != 2 or x.shape[1] != N or not x.is_cuda \
                    or x.device.index != self.engines[k].device:
                raise InvalidArgumentException(f"xs[{k}] must be a [rows][{N}] float64 tensor on cuda:"
                                               f"{self.engines[k].device}")
        outs = [(torch.empty((levels, x.shape[0], N), dtype=torch.float64, device=x.device),
                 torch.empty_like(x)) for x in xs]
        rows = (ctypes.c_int64 * len(xs))(*[x.shape[0] for x in xs])
        lo, hi = wavelet.lowPassDecomposition(), wavelet.highPassDecomposition()
        flags = nat.FLAG_SYNC | (nat.FLAG_FMA if fma else 0) | (nat.FLAG_CORE_LEVELS if core_levels else 0)
        self._sync_devices()  # the inputs were written on torch's streams
        _check(nat.load().vw_modwt_forward_multi_dev_f64(
            self._ctxs, len(xs), self._dev_ptrs(xs), rows, N, N, nat.taps_array(lo), nat.taps_array(hi), len(lo),
            wavelet.wavelet_id, boundary, levels, flags, self._dev_ptrs([d for d, _ in outs]),
            self._dev_ptrs([a for _, a in outs])))
        return outs

    def inverse_device(self, parts, wavelet: Wavelet, boundary: int = nat.PERIODIC, fma: bool = False):
        """parts: [(details [J][B_k][N], approx [B_k][N])] per context, on its device -> [y [B_k][N]]."""
        import torch
        if len(parts) != len(self.engines):
            raise InvalidArgumentException("one (details, approx) pair per context")
        parts = [(d.contiguous(), a.contiguous()) for d, a in parts]
        d0 = parts[0][0]
        if d0.ndim != 3:
            raise InvalidArgumentException("details must be [levels][rows][length]")
        J, _, N = d0.shape
        # every shard is checked before any launch: the engine reads these as float64
        # [J][rows][N] / [rows][N] buffers on context k's device, so a mismatch would be an out-of-bounds
        # access, not an error
        for k, (d, a) in enumerate(parts):
            dev = self.engines[k].device
            ok = (d.dtype == torch.float64 and a.dtype == torch.float64 and d.ndim == 3 and a.ndim == 2
                  and d.shape[0] == J and d.shape[2] == N and a.shape[1] == N and d.shape[1] == a.shape[0]
                  and d.is_cuda and a.is_cuda and d.device.index == dev and a.device.index == dev)
            if not ok:
                raise InvalidArgumentException(
                    f"parts[{k}] must be float64 details [{J}][rows][{N}] and approx [rows][{N}] on cuda:{dev}, got "
                    f"{tuple(d.shape)} {d.dtype} {d.device} / {tuple(a.shape)} {a.dtype} {a.device}")
        ys = [torch.empty_like(a) for _, a in parts]
        rows = (ctypes.c_int64 * len(parts))(*[a.shape[0] for _, a in parts])
        lo, hi = wavelet.lowPassReconstruction(), wavelet.highPassReconstruction()
        flags = nat.FLAG_SYNC | (nat.FLAG_FMA if fma else 0)
        self._sync_devices()
        _check(nat.load().vw_modwt_inverse_multi_dev_f64(
            self._ctxs, len(parts), self._dev_ptrs([d for d, _ in parts]), self._dev_ptrs([a for _, a in parts]),
            rows, N, nat.taps_array(lo), nat.taps_array(hi), len(lo), wavelet.wavelet_id, boundary, J, 0xFFFFFFFF,
            0, flags, self._dev_ptrs(ys)))
        return ys

    def close(self) -> None:
        if self._own:
            for e in self.engines:
                if e.ctx:
                    _check(e.lib.vw_ctx_destroy(e.ctx))
                    e.ctx = None
        self.engines = []

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
