"""Probe: the headline step (db4 J=6 fwd+inv over 4096 x 4096 fp64) issued by K contexts on one GPU, each
owning a contiguous block of rows on its own stream (graph replay per context), timed by events on a
main stream that forks to and joins the K streams.  Prints ms/step and Msamples/s per K."""
import sys
import time
from ctypes import c_void_p

import torch

sys.path.insert(0, ".")
import vectorwave_amd as vw
from vectorwave_amd import _native as nat

B, N, J, STEPS = 4096, 4096, 6, int(sys.argv[1]) if len(sys.argv) > 1 else 50
w = vw.Daubechies.DB4
lo, hi = nat.taps_array(w.lowPassDecomposition()), nat.taps_array(w.highPassDecomposition())
P = lambda t: c_void_p(t.data_ptr())  # noqa: E731


def run(K):
    main = torch.cuda.Stream()
    subs = []
    for k in range(K):
        eng = vw.Engine(0)
        s = torch.cuda.Stream()
        rows = B // K
        with torch.cuda.stream(s):
            x = torch.empty((rows, N), dtype=torch.float64, device="cuda")
            eng.fill_uniform(x, 42, offset=k * rows * N)
            det = torch.empty((J, rows, N), dtype=torch.float64, device="cuda")
            app = torch.empty((rows, N), dtype=torch.float64, device="cuda")
            y = torch.empty((rows, N), dtype=torch.float64, device="cuda")
            eng.bind_torch_stream()

            def step(eng=eng, x=x, det=det, app=app, y=y, rows=rows):
                assert eng.lib.vw_modwt_forward_f64(eng.ctx, P(x), rows, N, N, lo, hi, 8, w.wavelet_id, 0, J,
                                                    nat.FLAG_FMA, P(det), P(app)) == 0
                assert eng.lib.vw_modwt_inverse_f64(eng.ctx, P(det), P(app), rows, N, lo, hi, 8, w.wavelet_id, 0, J,
                                                    0xFFFFFFFF, 0, nat.FLAG_FMA, P(y)) == 0
            step()
            torch.cuda.synchronize()
            g = eng.capture(lambda step=step: [step() for _ in range(STEPS)])
        subs.append((s, g, eng, (x, det, app, y)))
    torch.cuda.synchronize()

    def once():
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(main):
            e0.record()
        ends = []
        for s, g, eng, _ in subs:
            s.wait_event(e0)
            with torch.cuda.stream(s):
                g.launch(1)
                ee = torch.cuda.Event()
                ee.record()
            ends.append(ee)
        with torch.cuda.stream(main):
            for ee in ends:
                main.wait_event(ee)
            e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)
    t0 = time.time()
    while time.time() - t0 < 1.0:
        once()
    ms = min(once() for _ in range(5)) / STEPS
    for s, g, eng, _ in subs:
        g.close()
    return ms


for K in (1, 2, 4, 1, 2):
    ms = run(K)
    print(f"K={K} ms/step={ms:.4f} Msamples/s={B * N / ms / 1e3:.1f}", flush=True)
