#!/usr/bin/env python3
"""Per-step HIP-event trace of the db4 fwd+inv step, fresh process (diagnoses clock ramp).

    python tools/step_trace.py [--steps 60] [--batch 4096] [--settle 0]

Prints one line per step: forward ms, inverse ms (events on the engine stream around each launch),
plus the wall time since the first launch, so the first steps of a short bench run are visible.
"""
import argparse
import os
import sys
import time
from ctypes import c_void_p

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--levels", type=int, default=6)
    ap.add_argument("--wavelet", default="db4")
    ap.add_argument("--settle", type=float, default=0.0, help="seconds of untimed steps first")
    a = ap.parse_args()
    import torch
    import vectorwave_amd as vw
    from vectorwave_amd import _native as nat

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    eng = vw.Engine.get(0)
    w = vw.get_wavelet(a.wavelet)
    lo, hi = w.lowPassDecomposition(), w.highPassDecomposition()
    B, N, J = a.batch, a.n, a.levels
    x = torch.empty((B, N), dtype=torch.float64, device=dev)
    eng.fill_uniform(x, 42)
    det = torch.empty((J, B, N), dtype=torch.float64, device=dev)
    app = torch.empty((B, N), dtype=torch.float64, device=dev)
    y = torch.empty((B, N), dtype=torch.float64, device=dev)
    eng.bind_torch_stream()
    lo_a, hi_a = nat.taps_array(lo), nat.taps_array(hi)
    lib = eng.lib
    xp, dp, ap_, yp = (c_void_p(t.data_ptr()) for t in (x, det, app, y))

    def fwd():
        assert lib.vw_modwt_forward_f64(eng.ctx, xp, B, N, N, lo_a, hi_a, len(lo), w.wavelet_id, 0, J,
                                        nat.FLAG_FMA, dp, ap_) == 0

    def inv():
        assert lib.vw_modwt_inverse_f64(eng.ctx, dp, ap_, B, N, lo_a, hi_a, len(lo), w.wavelet_id, 0, J,
                                        0xFFFFFFFF, 0, nat.FLAG_FMA, yp) == 0

    torch.cuda.synchronize()
    if a.settle > 0:
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < a.settle:
            for _ in range(20):
                fwd(); inv()
            torch.cuda.synchronize()
            n += 20
        print(f"settle: {n} steps in {time.perf_counter() - t0:.2f} s")
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    t0 = time.perf_counter()
    for e0, e1, e2 in ev:
        e0.record(); fwd(); e1.record(); inv(); e2.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    tf = ti = 0.0
    for k, (e0, e1, e2) in enumerate(ev):
        f, i = e0.elapsed_time(e1), e1.elapsed_time(e2)
        tf += f; ti += i
        print(f"step {k:3d}  fwd {f:.4f}  inv {i:.4f}  since0 {ev[0][0].elapsed_time(e2):8.3f} ms")
    n = len(ev)
    print(f"mean fwd {tf / n:.4f} inv {ti / n:.4f} wall/step {wall / n * 1e3:.4f} ms "
          f"-> {B * N / (wall / n) / 1e6:.0f} Msamples/s (wall)")


if __name__ == "__main__":
    main()
