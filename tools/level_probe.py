"""Probe: forward / inverse pass time of one config as a function of the level count J (1..Jmax), so the
per-level cost is the difference between consecutive rows.  Direct C-ABI launches on one context, events
around K launches of each pass, FMA.
  python tools/level_probe.py coif5 8192 65536 f32 6 [K]"""
import sys
from ctypes import c_void_p

import torch

sys.path.insert(0, ".")
import vectorwave_amd as vw
from vectorwave_amd import _native as nat

name, N, B, dt, JM = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], int(sys.argv[5])
K = int(sys.argv[6]) if len(sys.argv) > 6 else 10
f32 = dt == "f32"
tdt = torch.float32 if f32 else torch.float64
from vectorwave_amd.wavelets import get_wavelet  # noqa: E402
w = get_wavelet(name)
lo, hi = w.lowPassDecomposition(), w.highPassDecomposition()
L = len(lo)
lo_a, hi_a = nat.taps_array(lo), nat.taps_array(hi)
eng = vw.Engine(0)
eng.bind_torch_stream()
lib = eng.lib
fwd = lib.vw_modwt_forward_f32 if f32 else lib.vw_modwt_forward_f64
inv = lib.vw_modwt_inverse_f32 if f32 else lib.vw_modwt_inverse_f64
P = lambda t: c_void_p(t.data_ptr())  # noqa: E731
x = torch.empty((B, N), dtype=tdt, device="cuda")
eng.fill_uniform(x, 42)
y = torch.empty_like(x)
app = torch.empty_like(x)
det = torch.empty((JM, B, N), dtype=tdt, device="cuda")


def ok(st):
    if st:
        raise RuntimeError(nat.last_error())


def timed(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(K):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / K


prev = (0.0, 0.0)
print(f"# {name} N={N} B={B} {dt} L={L} K={K}: J fwd_ms inv_ms d_fwd d_inv", flush=True)
for J in range(1, JM + 1):
    tf = timed(lambda: ok(fwd(eng.ctx, P(x), B, N, N, lo_a, hi_a, L, w.wavelet_id, nat.PERIODIC, J, nat.FLAG_FMA,
                              P(det), P(app))))
    ti = timed(lambda: ok(inv(eng.ctx, P(det), P(app), B, N, lo_a, hi_a, L, w.wavelet_id, nat.PERIODIC, J,
                              0xFFFFFFFF, 0, nat.FLAG_FMA, P(y))))
    print(f"{J} {tf:.4f} {ti:.4f} {tf - prev[0]:+.4f} {ti - prev[1]:+.4f}", flush=True)
    prev = (tf, ti)
