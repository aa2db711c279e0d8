"""Non-finite samples on the reference's unvalidated paths (VW_FLAG_REF_NONFINITE, vectorwave_amd/csrc/vw_ref.hip).

BatchMODWT.multiLevelAoS (no finite check, BatchMODWT.java:201-212) multiplies every tap of the upsampled
filters, zeros included (BatchSIMDMODWT.java:384-424); so do MultiLevelMODWTTransform.reconstruct (K4-K6,
:554-645, which BatchMODWT.inverseMultiLevelAoS calls per signal) and VectorWaveSwtAdapter.forwardParallel
(:210-335; the branch config 3 takes: N >= 4096 and J > 2) / inverse (:435-487).  A NaN or +-Inf sample
therefore turns every output whose window reaches it through a zero tap into NaN (0 * Inf).  The bar here is
full identity with the restatement (oracle/vw_oracle.c, which multiplies the zero taps as the reference
does): NaN masks equal, +-Inf equal, every other value bit-equal (signed zeros included).
"""
import numpy as np
import pytest

from oracle import oracle as O
import vectorwave_amd as vw
from vectorwave_amd.wavelets import Daubechies, Symlet

pytestmark = pytest.mark.gpu


def signals(B, n, seed):
    return np.stack([O.java_random_signal(n, seed + b) for b in range(B)])


def lohi(w):
    return w.lowPassDecomposition(), w.highPassDecomposition()


def same(got, ref, what=""):
    """Identity: NaN where the reference has NaN, and the same 64 bits everywhere else."""
    got, ref = np.asarray(got, dtype=np.float64), np.asarray(ref, dtype=np.float64)
    assert got.shape == ref.shape, what
    gn, rn = np.isnan(got), np.isnan(ref)
    if not np.array_equal(gn, rn):
        bad = np.argwhere(gn != rn)
        raise AssertionError(f"{what}: NaN masks differ at {len(bad)} positions, first {bad[:4].tolist()}")
    gb, rb = got[~gn].view(np.int64), ref[~rn].view(np.int64)
    if not np.array_equal(gb, rb):
        i = int(np.argmax(gb != rb))
        raise AssertionError(f"{what}: value {got[~gn][i]!r} != reference {ref[~rn][i]!r}")


def poisoned(B, n, seed):
    """Rows: 0 +Inf, 1 NaN, 2 -Inf next to +Inf (Inf - Inf inside the sums), 3 clean, 4 NaN at both ends."""
    x = signals(B, n, seed)
    x[0, n // 5] = np.inf
    x[1, 7] = np.nan
    x[2, n // 2] = -np.inf
    x[2, n // 2 + 1] = np.inf
    if B > 4:
        x[4, 0] = np.nan
        x[4, n - 1] = np.nan
    return x


@pytest.mark.parametrize("case", [(Daubechies.DB4, 512, 4), (Symlet.SYM8, 1024, 5), (Daubechies.DB4, 4096, 6)],
                         ids=["db4-512-J4", "sym8-1024-J5", "db4-4096-J6"])
@pytest.mark.parametrize("device", [False, True], ids=["host", "device"])
def test_batch_modwt_nonfinite_identity(engine, case, device):
    import torch
    w, n, J = case
    x = poisoned(5, n, 51)
    xin = torch.from_numpy(x).cuda() if device else x
    m = vw.BatchMODWT.multiLevelAoS(w, xin, J)
    det = m.detailPerLevel.cpu().numpy() if device else m.detailPerLevel
    app = m.finalApprox.cpu().numpy() if device else m.finalApprox
    y = vw.BatchMODWT.inverseMultiLevelAoS(w, m.detailPerLevel, m.finalApprox)
    y = y.cpu().numpy() if device else y
    for b in range(5):
        d_ref, a_ref = O.decompose(x[b], *lohi(w), O.PERIODIC, J, core=False)
        same(det[:, b, :], d_ref, f"details row {b}")
        same(app[b], a_ref, f"approx row {b}")
        if b < 3:
            assert np.isnan(d_ref).any()  # the zero taps spread the sample as NaN
        same(y[b], O.reconstruct(d_ref, a_ref, w.lowPassReconstruction(), w.highPassReconstruction(), O.PERIODIC),
             f"inverse row {b}")


def test_batch_modwt_nonfinite_under_fma(engine):
    # FMA accumulation: the flagged rows run the reference's arithmetic (identical), the clean row stays
    # within the FMA tolerance
    w, n, J = Daubechies.DB4, 512, 5
    x = poisoned(4, n, 77)
    m = vw.BatchMODWT.multiLevelAoS(w, x, J, fma=True)
    for b in range(4):
        d_ref, a_ref = O.decompose(x[b], *lohi(w), O.PERIODIC, J, core=False)
        if b < 3:
            same(m.detailPerLevel[:, b, :], d_ref, f"row {b}")
            same(m.finalApprox[b], a_ref, f"row {b}")
        else:
            assert np.max(np.abs(m.detailPerLevel[:, b, :] - d_ref)) <= 1e-12
            assert np.max(np.abs(m.finalApprox[b] - a_ref)) <= 1e-12


def test_batch_modwt_overflow_inside_the_cascade(engine):
    # finite input whose sums overflow to +-Inf at some level: the next level's zero taps turn it into NaN
    w, n, J = Daubechies.DB4, 512, 5
    x = signals(3, n, 5)
    x[0, 100:140] = 1.7e308
    x[1, 10:20] = -1.7e308
    m = vw.BatchMODWT.multiLevelAoS(w, x, J)
    y = vw.BatchMODWT.inverseMultiLevelAoS(w, m.detailPerLevel, m.finalApprox)
    for b in range(3):
        d_ref, a_ref = O.decompose(x[b], *lohi(w), O.PERIODIC, J, core=False)
        same(m.detailPerLevel[:, b, :], d_ref, f"row {b}")
        same(m.finalApprox[b], a_ref, f"row {b}")
        same(y[b], O.reconstruct(d_ref, a_ref, w.lowPassReconstruction(), w.highPassReconstruction(), O.PERIODIC),
             f"inverse row {b}")
    assert not np.isfinite(m.finalApprox[0]).all()


def test_batch_inverse_of_nonfinite_coefficients(engine):
    # inverseMultiLevelAoS on coefficients the caller poisoned directly (core reconstruct validates nothing)
    w, n, J = Symlet.SYM8, 2048, 4
    x = signals(3, n, 9)
    m = vw.BatchMODWT.multiLevelAoS(w, x, J)
    det, app = m.detailPerLevel.copy(), m.finalApprox.copy()
    det[2, 0, 500] = np.nan
    app[1, 1000] = -np.inf
    det[0, 2, 3] = np.inf
    y = vw.BatchMODWT.inverseMultiLevelAoS(w, det, app)
    for b in range(3):
        same(y[b], O.reconstruct(det[:, b, :], app[b], w.lowPassReconstruction(), w.highPassReconstruction(),
                                 O.PERIODIC), f"row {b}")


@pytest.mark.parametrize("soft", [True, False], ids=["soft", "hard"])
def test_swt_denoise_parallel_branch_nonfinite_config3(engine, soft):
    # config 3's shape and branch: sym8 J = 8, N = 16384 (forwardParallel: no validation), universal threshold
    w, n, J = Symlet.SYM8, 16384, 8
    x = poisoned(4, n, 123)
    swt = vw.VectorWaveSwtAdapter(w, vw.BoundaryMode.PERIODIC)
    y, thr = swt.denoise(x, J, soft=soft, return_thresholds=True)
    for b in range(4):
        y_ref, t_ref = O.swt_denoise(x[b], *lohi(w), O.PERIODIC, J, soft=soft, wavelet_id=w.wavelet_id)
        same(thr[b], t_ref, f"threshold row {b}")
        same(y[b], y_ref, f"denoised row {b}")


@pytest.mark.parametrize("boundary", [O.SYMMETRIC, O.ZERO_PADDING], ids=["S", "Z"])
@pytest.mark.parametrize("soft", [True, False], ids=["soft", "hard"])
def test_swt_denoise_nonperiodic_nonfinite(engine, boundary, soft):
    # the parallel branch on the other boundaries: forward convolution chunks (:303-335), universal
    # thresholds, core reconstruct K5 / K6 -- 64 rows so the sequential inverse probes its output
    w, n, J, B = Symlet.SYM8, 4096, 4, 64
    x = O.fill_uniform(B * n, 29).reshape(B, n)
    x[0, 0] = np.nan
    x[31, 2000] = np.inf
    x[B - 1, n - 1] = -np.inf
    swt = vw.VectorWaveSwtAdapter(w, vw.BoundaryMode(boundary))
    y, thr = swt.denoise(x, J, soft=soft, return_thresholds=True)
    for b in (0, 1, 31, B - 1):
        y_ref, t_ref = O.swt_denoise(x[b], *lohi(w), boundary, J, soft=soft, wavelet_id=w.wavelet_id)
        same(thr[b], t_ref, f"threshold row {b}")
        same(y[b], y_ref, f"denoised row {b}")


def test_config3_kernels_flag_their_own_rows(engine):
    # config 3 runs the register-blocked kernels (k_forward_blk / k_inverse_blk), which probe their details /
    # output in-line: no scan of the call's planes (timing family "ref_nonfinite", not "..._scan")
    w, n, J = Symlet.SYM8, 16384, 8
    x = poisoned(3, n, 7)
    swt = vw.VectorWaveSwtAdapter(w, vw.BoundaryMode.PERIODIC)
    engine.enable_timing(True)
    engine.reset_timing()
    try:
        y = swt.denoise(x, J)
        assert engine.kernel_time("ref_nonfinite_scan")[1] == 0
        assert engine.kernel_time("ref_nonfinite")[1] == 2
    finally:
        engine.enable_timing(False)
    for b in range(3):
        y_ref, _ = O.swt_denoise(x[b], *lohi(w), O.PERIODIC, J, soft=True, wavelet_id=w.wavelet_id)
        same(y[b], y_ref, f"denoised row {b}")


@pytest.mark.parametrize("boundary", [O.PERIODIC, O.SYMMETRIC, O.ZERO_PADDING], ids=["P", "S", "Z"])
def test_swt_parallel_forward_inverse_nonfinite(engine, boundary):
    # forwardParallel's three chunk loops (:282-335) and the matching inverse (reconstructPeriodic, or core
    # reconstruct K5 / K6 with the symmetric alignment)
    w, n, J = Daubechies.DB4, 4096, 4
    x = poisoned(5, n, 31)
    swt = vw.VectorWaveSwtAdapter(w, vw.BoundaryMode(boundary))
    res = swt.forward(x, J)
    det, app = res.details_array, res.approximation_array
    y = swt.inverse(res)
    for b in range(5):
        d_ref, a_ref = O.swt_forward(x[b], *lohi(w), boundary, J)
        same(det[:, b, :], d_ref, f"details row {b}")
        same(app[b], a_ref, f"approx row {b}")
        if boundary == O.PERIODIC:
            y_ref = O.swt_reconstruct_periodic(d_ref, a_ref, w.lowPassReconstruction(), w.highPassReconstruction())
        else:
            y_ref = O.reconstruct(d_ref, a_ref, w.lowPassReconstruction(), w.highPassReconstruction(), boundary,
                                  wavelet_id=w.wavelet_id)
        same(y[b], y_ref, f"inverse row {b}")


@pytest.mark.parametrize("boundary", [O.ZERO_PADDING, O.SYMMETRIC], ids=["Z", "S"])
@pytest.mark.parametrize("blk", [256, 16], ids=["blk256", "blk16-shorter-than-history"])
def test_streaming_history_blocks_nonfinite(engine, boundary, blk):
    # BatchStreamingMODWT ZERO / SYMMETRIC: the history convolution multiplies every upsampled tap
    # (BatchSIMDMODWT.java:447-507), so a NaN / +-Inf spreads through the zero taps of this block AND, via
    # the history it leaves, into later blocks; the recomputed rows rewrite their histories.  First
    # block (history initialised from the block), later blocks, blocks shorter than the deepest history
    # (carry), and the flush tail -- identity with the restatement for every row and block.
    w, J, B = Daubechies.DB4, 4, 4
    x = signals(B, blk * 4, 3)
    x[0, 5] = np.nan                      # first block
    x[1, blk + blk // 2] = np.inf         # second block
    x[2, 3 * blk - 1] = -np.inf           # end of the third block: only the history carries it on
    st = vw.BatchStreamingMODWT(w, vw.BoundaryMode(boundary), J)
    refs = [O.StreamRestatement(*lohi(w), boundary, J) for _ in range(B)]
    for k in range(4):
        out = st.processMultiLevel(x[:, k * blk:(k + 1) * blk])
        for b in range(B):
            d_ref, a_ref = refs[b].process(x[b, k * blk:(k + 1) * blk])
            same(out.detailPerLevel[:, b, :], d_ref, f"block {k} details row {b}")
            same(out.finalApprox[b], a_ref, f"block {k} approx row {b}")
    assert not np.isfinite(out.detailPerLevel[:, 2, :]).all()  # block 4 of row 2: only its history is poisoned
    tl = st.getMinFlushTailLength()
    tail = st.flushMultiLevel(tl)
    for b in range(B):
        d_ref, a_ref = refs[b].flush(tl)
        same(tail.detailPerLevel[:, b, :], d_ref, f"flush details row {b}")
        same(tail.finalApprox[b], a_ref, f"flush approx row {b}")
    st.close()


def test_streaming_periodic_blocks_nonfinite(engine):
    # BatchStreamingMODWT PERIODIC blocks are independent BatchMODWT blocks (BatchStreamingMODWT.java:110-116)
    w, n, J = Daubechies.DB4, 1024, 4
    x = poisoned(3, n, 17)
    with vw.BatchStreamingMODWT(w, vw.BoundaryMode.PERIODIC, J) as s:
        r = s.processMultiLevel(x)
    for b in range(3):
        d_ref, a_ref = O.decompose(x[b], *lohi(w), O.PERIODIC, J, core=False)
        same(r.detailPerLevel[:, b, :], d_ref, f"row {b}")
        same(r.finalApprox[b], a_ref, f"row {b}")


def test_validated_paths_still_reject(engine):
    # the validated entry points keep the reference's InvalidSignalException (VAL_003), first bad index
    x = signals(1, 512, 3)[0]
    x[77] = np.nan
    with pytest.raises(vw.InvalidSignalException):
        vw.MultiLevelMODWTTransform(Daubechies.DB4, vw.BoundaryMode.PERIODIC).decompose(x, 3)
    with pytest.raises(vw.InvalidSignalException):  # decomposeSWT branch (N < 4096)
        vw.VectorWaveSwtAdapter(Daubechies.DB4, vw.BoundaryMode.PERIODIC).forward(x, 3)


def test_headline_kernels_flag_their_own_rows(engine):
    # db4 J = 6, N = 4096, fp64 FMA at 640 rows (> 2 per CU): the persistent forward and the one-buffer
    # sequential inverse -- the headline's kernels -- probe their own outputs / inputs (no scan pass,
    # timing family "ref_nonfinite", not "ref_nonfinite_scan").  Poisoned rows: the reference's bits;
    # clean rows: the fast kernels' bits (the same as without the flag); the flags are clear afterwards.
    import torch
    from vectorwave_amd import _native as nat
    w, n, J, B = Daubechies.DB4, 4096, 6, 640
    x = O.fill_uniform(B * n, 23).reshape(B, n)
    x[0, 9] = np.inf
    x[317, 2048] = np.nan
    x[B - 1, n - 1] = -np.inf
    x[B - 1, 0] = np.inf
    lo, hi = lohi(w)
    lr, hr = w.lowPassReconstruction(), w.highPassReconstruction()
    F, REF = nat.FLAG_FMA, nat.FLAG_FMA | nat.FLAG_REF_NONFINITE
    xt = torch.from_numpy(x).cuda()
    engine.enable_timing(True)
    engine.reset_timing()
    try:
        d1, a1 = engine.forward(xt, lo, hi, w.wavelet_id, O.PERIODIC, J, REF)
        det = d1.clone()
        app = a1.clone()
        det[2, 100, 7] = float("nan")  # poisoned coefficients of clean rows 100 and 200
        app[200, 5] = float("inf")
        y1 = engine.inverse(det, app, lr, hr, w.wavelet_id, O.PERIODIC, J, REF)
        torch.cuda.synchronize()
        assert engine.kernel_time("ref_nonfinite")[1] == 2
        assert engine.kernel_time("ref_nonfinite_scan")[1] == 0
    finally:
        engine.enable_timing(False)
    d0, a0 = engine.forward(xt, lo, hi, w.wavelet_id, O.PERIODIC, J, F)
    y0 = engine.inverse(det, app, lr, hr, w.wavelet_id, O.PERIODIC, J, F)
    d1, a1, y1 = d1.cpu().numpy(), a1.cpu().numpy(), y1.cpu().numpy()
    d0, a0, y0 = d0.cpu().numpy(), a0.cpu().numpy(), y0.cpu().numpy()
    dh, ah = det.cpu().numpy(), app.cpu().numpy()
    for b in (0, 317, B - 1):
        d_ref, a_ref = O.decompose(x[b], lo, hi, O.PERIODIC, J, core=False)
        same(d1[:, b, :], d_ref, f"details row {b}")
        same(a1[b], a_ref, f"approx row {b}")
    for b in (0, 100, 200, 317, B - 1):
        same(y1[b], O.reconstruct(dh[:, b, :], ah[b], lr, hr, O.PERIODIC), f"inverse row {b}")
    clean = np.setdiff1d(np.arange(B), [0, 317, B - 1])
    assert np.array_equal(d1[:, clean, :].view(np.int64), d0[:, clean, :].view(np.int64))
    assert np.array_equal(a1[clean].view(np.int64), a0[clean].view(np.int64))
    clean_y = np.setdiff1d(clean, [100, 200])
    assert np.array_equal(y1[clean_y].view(np.int64), y0[clean_y].view(np.int64))
    # flags cleared: a clean call with the flag gives the fast kernels' bits everywhere
    xc = torch.from_numpy(np.nan_to_num(x, nan=0.0, posinf=0.0, neginf=0.0)).cuda()
    d2, a2 = engine.forward(xc, lo, hi, w.wavelet_id, O.PERIODIC, J, REF)
    d3, a3 = engine.forward(xc, lo, hi, w.wavelet_id, O.PERIODIC, J, F)
    y2 = engine.inverse(d2, a2, lr, hr, w.wavelet_id, O.PERIODIC, J, REF)
    y3 = engine.inverse(d3, a3, lr, hr, w.wavelet_id, O.PERIODIC, J, F)
    assert torch.equal(d2.view(torch.int64), d3.view(torch.int64)) and torch.equal(a2.view(torch.int64), a3.view(torch.int64))
    assert torch.equal(y2.view(torch.int64), y3.view(torch.int64))


def test_ref_nonfinite_in_a_captured_graph(engine):
    # the row flags are allocated by the first call and cleared by the fix-up kernels, so a recorded
    # forward + inverse with VW_FLAG_REF_NONFINITE replays correctly whether or not a replay meets a NaN
    import torch
    from ctypes import c_void_p
    from vectorwave_amd import _native as nat
    w, B, N, J = Daubechies.DB4, 640, 4096, 6
    F = nat.FLAG_FMA | nat.FLAG_REF_NONFINITE
    lo, hi = nat.taps_array(w.lowPassDecomposition()), nat.taps_array(w.highPassDecomposition())
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        x = torch.empty((B, N), dtype=torch.float64, device="cuda")
        det = torch.empty((J, B, N), dtype=torch.float64, device="cuda")
        app, y = torch.empty_like(x), torch.empty_like(x)
        engine.fill_uniform(x, 7)
        lib, ctx = engine.lib, engine.ctx
        P = lambda t: c_void_p(t.data_ptr())  # noqa: E731

        def step():
            assert lib.vw_modwt_forward_f64(ctx, P(x), B, N, N, lo, hi, len(lo), w.wavelet_id, 0, J, F,
                                            P(det), P(app)) == 0
            assert lib.vw_modwt_inverse_f64(ctx, P(det), P(app), B, N, lo, hi, len(lo), w.wavelet_id, 0, J,
                                            0xFFFFFFFF, 0, F, P(y)) == 0

        step()
        torch.cuda.synchronize()
        d0, a0, y0 = det.clone(), app.clone(), y.clone()
        g = engine.capture(step)
        x[411, 1000] = float("nan")
        g.launch(1)
        torch.cuda.synchronize()
        xh = x.cpu().numpy()
        d_ref, a_ref = O.decompose(xh[411], w.lowPassDecomposition(), w.highPassDecomposition(), O.PERIODIC, J,
                                   core=False)
        same(det[:, 411].cpu().numpy(), d_ref, "replayed details row 411")
        same(app[411].cpu().numpy(), a_ref, "replayed approx row 411")
        same(y[411].cpu().numpy(), O.reconstruct(d_ref, a_ref, w.lowPassReconstruction(), w.highPassReconstruction(),
                                                 O.PERIODIC), "replayed inverse row 411")
        engine.fill_uniform(x, 7)  # the clean input again
        g.launch(2)
        torch.cuda.synchronize()
        assert torch.equal(det.view(torch.int64), d0.view(torch.int64))
        assert torch.equal(app.view(torch.int64), a0.view(torch.int64))
        assert torch.equal(y.view(torch.int64), y0.view(torch.int64))
        g.close()


def test_ref_nonfinite_fp32_headline_kernels(engine):
    # the fp32 persistent forward / sequential inverse probe their rows too; the reference has no fp32 path,
    # so the bar is the fp64 restatement's NaN / +-Inf positions and the FMA path's fp32 tolerance elsewhere
    import torch
    from vectorwave_amd import _native as nat
    w, n, J, B = Daubechies.DB4, 4096, 6, 640
    x = O.fill_uniform(B * n, 31).reshape(B, n).astype(np.float32)
    x[5, 77] = np.nan
    x[600, 4000] = -np.inf
    lo, hi = lohi(w)
    lr, hr = w.lowPassReconstruction(), w.highPassReconstruction()
    xt = torch.from_numpy(x).cuda()
    d, a = engine.forward(xt, lo, hi, w.wavelet_id, O.PERIODIC, J, nat.FLAG_FMA | nat.FLAG_REF_NONFINITE)
    y = engine.inverse(d, a, lr, hr, w.wavelet_id, O.PERIODIC, J, nat.FLAG_FMA | nat.FLAG_REF_NONFINITE)
    d0, a0 = engine.forward(xt, lo, hi, w.wavelet_id, O.PERIODIC, J, nat.FLAG_FMA)
    d, a, y = d.cpu().numpy(), a.cpu().numpy(), y.cpu().numpy()
    tol = 1e-5 * J
    for b in (5, 600):
        d_ref, a_ref = O.decompose(x[b].astype(np.float64), lo, hi, O.PERIODIC, J, core=False)
        y_ref = O.reconstruct(d_ref, a_ref, lr, hr, O.PERIODIC)
        for got, ref, what in ((d[:, b, :], d_ref, "details"), (a[b], a_ref, "approx"), (y[b], y_ref, "y")):
            assert np.array_equal(np.isnan(got), np.isnan(ref)), (b, what)
            assert np.array_equal(np.isposinf(got), np.isposinf(ref)) and np.array_equal(np.isneginf(got),
                                                                                         np.isneginf(ref)), (b, what)
            f = np.isfinite(ref)
            assert np.max(np.abs(got[f] - ref[f]), initial=0.0) <= tol, (b, what)
    clean = np.setdiff1d(np.arange(B), [5, 600])
    assert np.array_equal(d[:, clean, :], d0.cpu().numpy()[:, clean, :])
    assert np.array_equal(a[clean], a0.cpu().numpy()[clean])


@pytest.mark.parametrize("boundary", [O.PERIODIC, O.SYMMETRIC], ids=["P", "S"])
def test_swt_full_batch_rows_probe_themselves(engine, boundary):
    # 640 rows (> 2 per CU): the kernels that probe their own rows (persistent forward; one-buffer sequential
    # inverse for the K6 symmetric reconstruction) instead of the scan pass
    w, n, J, B = Daubechies.DB4, 4096, 4, 640
    x = O.fill_uniform(B * n, 13).reshape(B, n)
    x[3, 0] = np.nan
    x[320, 2047] = np.inf
    x[B - 1, n - 1] = -np.inf
    swt = vw.VectorWaveSwtAdapter(w, vw.BoundaryMode(boundary))
    res = swt.forward(x, J)
    y = swt.inverse(res)
    for b in (3, 4, 320, B - 1):
        d_ref, a_ref = O.swt_forward(x[b], *lohi(w), boundary, J)
        same(res.details_array[:, b, :], d_ref, f"details row {b}")
        same(res.approximation_array[b], a_ref, f"approx row {b}")
        if boundary == O.PERIODIC:
            y_ref = O.swt_reconstruct_periodic(d_ref, a_ref, w.lowPassReconstruction(), w.highPassReconstruction())
        else:
            y_ref = O.reconstruct(d_ref, a_ref, w.lowPassReconstruction(), w.highPassReconstruction(), boundary,
                                  wavelet_id=w.wavelet_id)
        same(y[b], y_ref, f"inverse row {b}")


@pytest.mark.parametrize("fma", [False, True], ids=["exact", "fma"])
def test_long_rows_probe_their_final_output(engine, fma):
    # config 4's row shape (db8 J = 10, 2^20 samples): multi-level tiles + the deep forward launch, chained
    # column sweeps + multi-level inverse tiles.  The launches that write a_J / y probe it in registers (no
    # scan of the plane); the poisoned row is the reference's bits, the clean one the fast kernels' bits.
    import torch
    from vectorwave_amd import _native as nat
    from vectorwave_amd.wavelets import Daubechies as D
    w, n, J, B = D.DB8, 1 << 20, 10, 2
    x = O.fill_uniform(B * n, 5).reshape(B, n)
    x[1, 777] = np.nan
    lo, hi = lohi(w)
    lr, hr = w.lowPassReconstruction(), w.highPassReconstruction()
    xt = torch.from_numpy(x).cuda()
    F = nat.FLAG_FMA if fma else 0
    R = nat.FLAG_REF_NONFINITE | F
    engine.enable_timing(True)
    engine.reset_timing()
    try:
        d1, a1 = engine.forward(xt, lo, hi, w.wavelet_id, O.PERIODIC, J, R)
        y1 = engine.inverse(d1, a1, lr, hr, w.wavelet_id, O.PERIODIC, J, R)
        torch.cuda.synchronize()
        scans = engine.kernel_time("ref_nonfinite_scan")[1]
        probed = engine.kernel_time("ref_nonfinite")[1]
    finally:
        engine.enable_timing(False)
    assert (probed, scans) == (2, 0), (probed, scans)
    d0, a0 = engine.forward(xt, lo, hi, w.wavelet_id, O.PERIODIC, J, F)
    y0 = engine.inverse(d0, a0, lr, hr, w.wavelet_id, O.PERIODIC, J, F)
    d1, a1, y1 = d1.cpu().numpy(), a1.cpu().numpy(), y1.cpu().numpy()
    assert np.array_equal(d1[:, 0].view(np.int64), d0[:, 0].cpu().numpy().view(np.int64))
    assert np.array_equal(y1[0].view(np.int64), y0[0].cpu().numpy().view(np.int64))
    d_ref, a_ref = O.decompose(x[1], lo, hi, O.PERIODIC, J, core=False)
    same(d1[:, 1, :], d_ref, "details row 1")
    same(a1[1], a_ref, "approx row 1")
    same(y1[1], O.reconstruct(d_ref, a_ref, lr, hr, O.PERIODIC), "inverse row 1")
