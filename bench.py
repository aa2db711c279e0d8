#!/usr/bin/env python3
"""bench.py -- MODWT fwd+inv throughput on MI355X (BASELINE.json metric), one process per GPU.

Default workload (BASELINE.json configs[1]): db4, J=6, forward + inverse of a 4096 x 4096 fp64 batch
per GPU (weak scaling: every rank owns its own shard of signals; no collective on the data path).
A "step" = one fused multi-level forward launch + one fused multi-level inverse launch over the
rank's batch, inputs already resident in HBM (generated on device by the counter-based generator).

Prints ONE JSON line (rank 0) with value = Msamples/s over all ranks, a `roofline` object for the
dominant kernel (algorithmic bytes per launch / its HIP-event-measured average duration) and a
`cpu_baseline` object (the C restatement of vectorwave-core's scalar loops, timed on a bounded
sample on this host's cores).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config db4|sym8-denoise|db8-stream|coif5-f32]
"""
import argparse
import ctypes
import json
import os
import sys
import time
from ctypes import c_void_p

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ACC_NAME = {
    True: "fma (fused multiply-add per tap; max-abs error vs vectorwave-core < 1e-12, tests/test_gpu_parity.py)",
    False: "exact (separate multiply and add in the reference's tap order; bit-identical to vectorwave-core)",
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (/opt/skills/guides/MI355X_MICROARCH.md)

CONFIGS = {
    # name: (wavelet, levels, batch per GPU, N, dtype, pipeline)
    "db4": ("db4", 6, 4096, 4096, "f64", "fwd+inv"),
    "sym8-denoise": ("sym8", 8, 16384, 16384, "f64", "denoise"),
    "db8-stream": ("db8", 10, 32, 1 << 20, "f64", "fwd+inv"),
    "coif5-f32": ("coif5", 6, 65536 // 8, 8192, "f32", "fwd+inv"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)   # ~0.1 s timed: long enough for stable clocks
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--config", default="db4", choices=sorted(CONFIGS))
    p.add_argument("--batch", type=int, default=0, help="override signals per GPU")
    p.add_argument("--wavelet", default="", help="override the config's wavelet (experiments)")
    p.add_argument("--exact", action="store_true",
                   help="headline in EXACT accumulation (bit-identical to vectorwave-core) instead of FMA")
    p.add_argument("--fma", action="store_true", help="(default) FMA accumulation, max-abs error < 1e-12")
    p.add_argument("--no-alt", action="store_true", help="skip the timing of the other accumulation mode")
    p.add_argument("--events", default="separate", choices=["inline", "separate"],
                   help="HIP events around each kernel inside the timed region, or in a replay after it")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=6.0, help="target wall time of the CPU baseline sample")
    return p.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
        local = 0

    import vectorwave_amd as vw
    from vectorwave_amd import _native as nat

    wname, J, Bg, N, dtype, pipeline = CONFIGS[args.config]
    if args.batch:
        Bg = args.batch
    if args.wavelet:
        wname = args.wavelet
    w = vw.get_wavelet(wname)
    lo, hi = w.lowPassDecomposition(), w.highPassDecomposition()
    L = len(lo)
    eng = vw.Engine.get(local)
    lib = eng.lib
    tdt = torch.float32 if dtype == "f32" else torch.float64
    esz = 4 if dtype == "f32" else 8
    dev = torch.device("cuda", local)

    # weak scaling: the global batch is world*Bg signals; rank r owns its shard_rows() block
    # (distinct data per rank, generated on device from the global row index), no exchange
    from vectorwave_amd.shard import shard_rows
    start, Bg = shard_rows(world * Bg, world, rank)
    # all work on one dedicated (non-default) stream: the engine binds to it, torch allocations order on it
    torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    x = torch.empty((Bg, N), dtype=tdt, device=dev)
    eng.fill_uniform(x, 42, offset=start * N)
    det = torch.empty((J, Bg, N), dtype=tdt, device=dev)
    app = torch.empty((Bg, N), dtype=tdt, device=dev)
    y = torch.empty((Bg, N), dtype=tdt, device=dev)
    eng.bind_torch_stream()
    flags = 0 if args.exact else nat.FLAG_FMA
    lo_a, hi_a = nat.taps_array(lo), nat.taps_array(hi)
    fwd = lib.vw_modwt_forward_f32 if dtype == "f32" else lib.vw_modwt_forward_f64
    inv = lib.vw_modwt_inverse_f32 if dtype == "f32" else lib.vw_modwt_inverse_f64
    xp, dp, ap, yp = (c_void_p(t.data_ptr()) for t in (x, det, app, y))

    def check(st):
        if st != 0:
            raise RuntimeError(f"engine status {st}: {nat.last_error()}")

    if pipeline == "fwd+inv":
        def step(flags=flags):
            check(fwd(eng.ctx, xp, Bg, N, N, lo_a, hi_a, L, w.wavelet_id, nat.PERIODIC, J, flags, dp, ap))
            check(inv(eng.ctx, dp, ap, Bg, N, lo_a, hi_a, L, w.wavelet_id, nat.PERIODIC, J, 0xFFFFFFFF, 0, flags, yp))
        bytes_per_sample = {"forward": (J + 2) * esz, "inverse": (J + 2) * esz}
    else:  # SWT universal soft-threshold denoise (config 3)
        thr = torch.empty((Bg,), dtype=torch.float64, device=dev)
        tp = c_void_p(thr.data_ptr())

        def step(flags=flags):
            check(lib.vw_swt_denoise_f64(eng.ctx, xp, Bg, N, N, lo_a, hi_a, L, w.wavelet_id, nat.PERIODIC, J, -1.0, 1,
                                         flags, yp, tp))
        bytes_per_sample = {"forward": (J + 2) * esz, "inverse": (J + 2) * esz, "sigma": esz}

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    eng.reset_timing()
    eng.enable_timing(args.events == "inline")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    eng.enable_timing(False)
    elapsed = t1 - t0
    if args.events == "separate":
        # per-kernel HIP-event durations from an instrumented replay of the same K steps
        eng.enable_timing(True)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        eng.enable_timing(False)
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = tt.item()

    # per-kernel durations measured live with HIP events on the engine's stream
    fam = {}
    for k in ("forward", "inverse", "sigma", "forward_level", "inverse_level"):
        ms, n = eng.kernel_time(k)
        if n:
            fam[k] = (ms / n, n)
    dom = max(fam, key=lambda k: fam[k][0] * fam[k][1])
    dom_ms = fam[dom][0]
    units = Bg * N
    base_family = dom.replace("_level", "")
    per_launch_bytes = bytes_per_sample.get(base_family, (J + 2) * esz) * units
    if dom.endswith("_level"):
        per_launch_bytes /= J  # one launch per level
    achieved = per_launch_bytes / (dom_ms * 1e-3) / 1e9

    total_samples = units * world * args.steps
    value = total_samples / elapsed / 1e6

    traffic = None
    tfile = os.path.join(ROOT, "profiles", f"hbm_traffic_{args.config}.json")
    if os.path.exists(tfile):
        try:
            with open(tfile) as fh:
                tj = json.load(fh)
            traffic = tj.get(dom, {}).get("bytes_per_launch")
        except Exception:
            traffic = None

    # The other accumulation mode, same workload, timed the same way (reported beside the headline).
    alt = None
    if not args.no_alt:
        aflags = flags ^ nat.FLAG_FMA
        for _ in range(args.warmup):
            step(aflags)
        eng.reset_timing()
        eng.enable_timing(True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        a0 = time.perf_counter()
        for _ in range(args.steps):
            step(aflags)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        a1 = time.perf_counter()
        eng.enable_timing(False)
        aelapsed = a1 - a0
        if world > 1:
            tt = torch.tensor([aelapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            aelapsed = tt.item()
        akern = {}
        for k in ("forward", "inverse", "sigma", "forward_level", "inverse_level"):
            ms, n = eng.kernel_time(k)
            if n:
                akern[k] = round(ms / n, 5)
        alt = {"accumulation": ACC_NAME[bool(aflags & nat.FLAG_FMA)],
               "value": round(units * world * args.steps / aelapsed / 1e6, 2), "kernels_ms": akern}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(w, J, N, dtype, pipeline, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "Msamples/sec MODWT fwd+inv db4 L=6, batch 4096×4096 fp64 @ 1/2/4/8 GPU"
            if args.config == "db4" else f"Msamples/sec {args.config} ({pipeline})",
            "value": round(value, 2),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic: counter-based splitmix64 uniform[-1,1), seed 42, generated on device",
            "config": {
                "workload": f"{wname} MODWT J={J} {pipeline}, {Bg} signals x {N} samples per GPU, {dtype}, PERIODIC",
                "wavelet": wname, "levels": J, "batch_per_gpu": Bg, "signal_length": N, "boundary": "PERIODIC",
                "accumulation": ACC_NAME[bool(flags & nat.FLAG_FMA)],
                "parallelism": f"batch-shard x{world} (no collective)",
                "kernels_ms": {k: round(v[0], 5) for k, v in fam.items()},
                "kernel_timing": ("HIP events on the engine stream around each launch, "
                                  + ("inside the timed loop" if args.events == "inline" else
                                     "in a replay of the K timed steps right after the (uninstrumented) timed loop")),
                "kernel_ms_per_step": round(sum(v[0] * v[1] for v in fam.values()) / args.steps, 5),
                "other_accumulation": alt,
            },
            "roofline": {
                "bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "algorithmic_bytes_per_launch": per_launch_bytes,
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(w, J, N, dtype, pipeline, seconds):
    """vectorwave-core's scalar loops (C restatement, zero taps included) on this host's cores, bounded sample."""
    import numpy as np
    from oracle import oracle as O

    lo, hi = w.lowPassDecomposition(), w.highPassDecomposition()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    os.environ.setdefault("OMP_NUM_THREADS", str(threads))
    fn = (lambda xs: O.batch_fwd_inv(xs, lo, hi, O.PERIODIC, J, w.wavelet_id)) if pipeline == "fwd+inv" else \
         (lambda xs: O.batch_denoise(xs, lo, hi, O.PERIODIC, J, -1.0, True, w.wavelet_id))
    # calibrate with one round of `threads` signals, then size the sample to ~`seconds`
    probe = O.fill_uniform(threads * N, 42).reshape(threads, N)
    t0 = time.perf_counter()
    _, used = fn(probe)
    dt = time.perf_counter() - t0
    rounds = max(1, int(seconds / max(dt, 1e-6)))
    B = min(threads * rounds, 4096)
    xs = O.fill_uniform(B * N, 42).reshape(B, N)
    t0 = time.perf_counter()
    _, used = fn(xs)
    dt = time.perf_counter() - t0
    return {"value": round(B * N / dt / 1e6, 3), "unit": "Msamples/s", "cores": int(used), "kind": "port",
            "sample": f"{B} signals x {N} samples ({w.name()} J={J} {pipeline}, fp64, core semantics), "
                      f"{dt:.1f} s wall on {used} OpenMP threads"}


if __name__ == "__main__":
    main()
