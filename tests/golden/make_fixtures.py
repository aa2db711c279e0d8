#!/usr/bin/env python3
"""Generate tests/golden/modwt_fixtures.npz: inputs + restatement outputs of the MODWT hot path.

The outputs come from oracle/ (the C restatement of vectorwave-core's scalar loops, itself pinned to
the reference's known answers and fixtures by tests/test_oracle_golden.py).  Committing them lets the
GPU parity tests (tests/test_golden_fixtures.py) compare the HIP engine with fixed vectors, and pins
the restatement against drift.  Inputs are the counter-based generator (seed 42, offset = case index
<< 32), so they are reproducible on host and device.

    python tests/golden/make_fixtures.py        # rewrites tests/golden/modwt_fixtures.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from vectorwave_amd.wavelets import get_wavelet  # noqa: E402

WAVELETS = ["haar", "db4", "db8", "sym8", "coif5"]
BOUNDARIES = {"periodic": O.PERIODIC, "symmetric": O.SYMMETRIC, "zero": O.ZERO_PADDING}
SIZES = [7, 64, 129, 512]
B = 2


def cases():
    i = 0
    for wn in WAVELETS:
        w = get_wavelet(wn)
        L = len(w.lowPassDecomposition())
        for bn, bc in BOUNDARIES.items():
            for n in SIZES:
                J = min(3, O.max_levels(n, L))
                if J < 1:
                    continue
                yield i, wn, w, bn, bc, n, J
                i += 1


def main():
    out = {}
    names = []
    for i, wn, w, bn, bc, n, J in cases():
        lo, hi = w.lowPassDecomposition(), w.highPassDecomposition()
        x = O.fill_uniform(B * n, 42, offset=i << 32).reshape(B, n)
        det = np.empty((J, B, n))
        app = np.empty((B, n))
        y = np.empty((B, n))
        for b in range(B):
            d, a = O.decompose(x[b], lo, hi, bc, J)
            det[:, b, :] = d
            app[b] = a
            y[b] = O.reconstruct(d, a, lo, hi, bc, w.wavelet_id)
        key = f"{wn}_{bn}_n{n}_j{J}"
        names.append(key)
        out[key + "_x"] = x
        out[key + "_details"] = det
        out[key + "_approx"] = app
        out[key + "_y"] = y
    out["cases"] = np.array(names)
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "modwt_fixtures.npz")
    np.savez_compressed(path, **out)
    print(f"{len(names)} cases -> {path} ({os.path.getsize(path) / 1024:.0f} KiB)")


if __name__ == "__main__":
    main()
