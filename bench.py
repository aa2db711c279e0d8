#!/usr/bin/env python3
"""bench.py -- MODWT fwd+inv throughput on MI355X (BASELINE.json metric), one process per GPU.

Default workload (BASELINE.json configs[1]): db4, J=6, forward + inverse of a GLOBAL batch of
4096 x 4096 fp64 signals, split across the N GPUs by contiguous row blocks (shard_rows; strong
scaling) -- no collective on the data path.  With N > 1 the same per-GPU work as at
N = 1 (4096 rows per rank) is timed afterwards and reported as `weak_scaling`.

A "step" = one multi-level forward pass + one multi-level inverse pass over the rank's rows, inputs
already resident in HBM (generated on device by the counter-based generator).  The K timed steps are
recorded once through the C ABI into one HIP graph (vw_capture_begin / vw_graph_launch) and replayed
once: no host-side planning or kernel-argument packing inside the timed region -- at 8 GPUs a pass is
~30 us of GPU work.  Every kernel launch of those K steps is bracketed by HIP event nodes inside the
graph, so per-kernel durations come from the timed steps themselves (`--launch direct|graph-step`
and `--events none` for A/B).

Clock settle: an MI355X leaving idle runs the first ~50 ms of load below its steady clock (measured
per step, profiles/r02/trace_*.log).  Before the W warmup steps the step is replayed for
`--settle` seconds (default 1.0, untimed, reported as settle_s / settle_steps), then W warmup
steps, then exactly K timed steps between barrier + device synchronize on both sides; the elapsed
time is the max over ranks.

`--gpus N` without torchrun: the parent spawns N rank processes (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_*) before any GPU call and relays rank 0's line.  Under torchrun each process is one rank.

Prints ONE JSON line (rank 0) with value = Msamples/s of the whole job, a `roofline` object for the
dominant pass (algorithmic bytes per launch / its average HIP-event duration over the timed steps) and a `cpu_baseline` object (the C restatement of
vectorwave-core's scalar loops, timed on a bounded sample on this host's cores, N = 1 only).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config db4|sym8-denoise|db8-stream|coif5-f32]
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time
from ctypes import c_void_p

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ACC_NAME = {
    True: "fma (fused multiply-add per tap; max-abs error vs vectorwave-core < 1e-12 at this configuration, tests/test_gpu_headline.py)",
    False: "exact (separate multiply and add in the reference's tap order; bit-identical to vectorwave-core)",
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (/opt/skills/guides/MI355X_MICROARCH.md)
COPY_GBS = 6167.2      # measured plain-copy kernel ("copy 1->1 nt", profiles/r01/membench_v2.log)

LAUNCH_DESC = {
    "graph-k": "the K timed steps recorded once into one HIP graph (vw_capture_begin / vw_graph_launch), replayed once",
    "graph-step": "a one-step HIP graph replayed K times",
    "direct": "direct C-ABI calls",
}

# name: (wavelet, levels, GLOBAL batch, N, dtype, pipeline) -- BASELINE.json configs[1..4]
CONFIGS = {
    "db4": ("db4", 6, 4096, 4096, "f64", "fwd+inv"),
    "sym8-denoise": ("sym8", 8, 16384, 16384, "f64", "denoise"),
    "db8-stream": ("db8", 10, 256, 1 << 20, "f64", "fwd+inv"),       # 256 PERIODIC 2^20-sample blocks
    "coif5-f32": ("coif5", 6, 65536, 8192, "f32", "fwd+inv"),
}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--settle", type=float, default=1.0, help="seconds of untimed steps before warmup (clock settle)")
    p.add_argument("--config", default="db4", choices=sorted(CONFIGS))
    p.add_argument("--batch", type=int, default=0, help="override the GLOBAL batch")
    p.add_argument("--wavelet", default="", help="override the config's wavelet (experiments)")
    p.add_argument("--exact", action="store_true",
                   help="headline in EXACT accumulation (bit-identical to vectorwave-core) instead of FMA")
    p.add_argument("--no-alt", action="store_true", help="skip the timing of the other accumulation mode")
    p.add_argument("--no-weak", action="store_true", help="N > 1: skip the weak-scaling measurement")
    p.add_argument("--launch", default="graph-k", choices=sorted(LAUNCH_DESC),
                   help="how the timed steps are issued (see measure())")
    p.add_argument("--events", default="inline", choices=["inline", "none"],
                   help="HIP events around every kernel launch inside the timed steps (inline) or none")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=6.0, help="target wall time of the CPU baseline sample")
    p.add_argument("--dry-run", action="store_true",
                   help="CPU only: launch the ranks, shard, run the timing collectives (gloo), print the plan")
    p.add_argument("--ref-shapes", action="store_true",
                   help="the reference's own JMH shapes (MultiLevelBatchSIMDBenchmark) through the host-memory "
                        "(JNI-shaped) path: per-call us with H2D / kernel / D2H separated, beside the CPU "
                        "restatement on the same rows; one JSON line (and --out FILE)")
    p.add_argument("--out", default="", help="--ref-shapes: also write the JSON to this file")
    return p.parse_args(argv)


# ---------------------------------------------------------------------------------------------
# Launcher: one process per GPU, spawned before anything touches a GPU.
def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in live:  # a dead rank leaves the others waiting in a collective
                    q.terminate()
        time.sleep(0.05)
    return rc


# ---------------------------------------------------------------------------------------------
def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)
    if args.ref_shapes:
        return ref_shapes(args)
    run(args, world, rank, local)


# ---------------------------------------------------------------------------------------------
# The reference's measurement shapes (vectorwave-benchmarks/src/main/java/com/morphiqlabs/benchmark/
# MultiLevelBatchSIMDBenchmark.java:29-36): batch {8,16,32} x N {4096,8192} x {db4, haar} x J {3,5},
# multi-level forward, PERIODIC.  This is the regime of a BatchMODWT / MultiLevelMODWTTransform caller:
# small batches handed over as host arrays, where staging and launch latency dominate.
REF_SHAPES = [(B, n, wv, J) for B in (8, 16, 32) for n in (4096, 8192) for wv in ("db4", "haar") for J in (3, 5)]


def ref_shapes(args):
    import statistics

    import numpy as np
    import torch

    import vectorwave_amd as vw
    from vectorwave_amd import _native as nat

    eng = vw.Engine.get(0)
    lib = eng.lib
    reps = 30
    rows = []
    P = lambda a: c_void_p(a.ctypes.data)  # noqa: E731
    D = lambda t: c_void_p(t.data_ptr())   # noqa: E731

    def med_us(fn, n=reps):
        fn()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts) * 1e6

    for B, n, wname, J in REF_SHAPES:
        w = vw.get_wavelet(wname)
        lo, hi = nat.taps_array(w.lowPassDecomposition()), nat.taps_array(w.highPassDecomposition())
        L = len(w.lowPassDecomposition())
        J = min(J, vw.max_levels(n, L))   # the benchmark's own clamp (getMaximumLevels)
        rng = np.random.default_rng(42)
        x = rng.standard_normal((B, n))   # nextGaussian-shaped input
        det = np.empty((J, B, n))
        app = np.empty((B, n))
        fl_host = nat.FLAG_HOST_MEMORY | nat.FLAG_CORE_LEVELS

        def host_call():
            st = lib.vw_modwt_forward_f64(eng.ctx, P(x), B, n, n, lo, hi, L, w.wavelet_id, nat.PERIODIC, J, fl_host,
                                          P(det), P(app))
            if st:
                raise RuntimeError(nat.last_error())
        call_us = med_us(host_call)
        # the same call's parts: H2D of x, the device-resident forward, D2H of the J + 1 output planes
        xd = torch.empty((B, n), dtype=torch.float64, device="cuda")
        dd = torch.empty((J, B, n), dtype=torch.float64, device="cuda")
        ad = torch.empty((B, n), dtype=torch.float64, device="cuda")
        eng.bind_torch_stream()
        h2d_us = med_us(lambda: lib.vw_memcpy(eng.ctx, D(xd), P(x), x.nbytes, 0))
        d2h_us = med_us(lambda: (lib.vw_memcpy(eng.ctx, P(det), D(dd), det.nbytes, 1),
                                 lib.vw_memcpy(eng.ctx, P(app), D(ad), app.nbytes, 1)))
        lib.vw_memcpy(eng.ctx, D(xd), P(x), x.nbytes, 0)

        def dev_call():
            lib.vw_modwt_forward_f64(eng.ctx, D(xd), B, n, n, lo, hi, L, w.wavelet_id, nat.PERIODIC, J,
                                     nat.FLAG_CORE_LEVELS, D(dd), D(ad))
        dev_call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            dev_call()
        e1.record()
        torch.cuda.synchronize()
        kernel_us = e0.elapsed_time(e1) * 1e3 / reps
        host_call()   # det / app again from the host-memory call (the D2H timing copied other bytes there)
        cpu_us, same = ref_shapes_cpu(x, w, J, det, app)
        rows.append({"batch": B, "n": n, "wavelet": wname, "levels": J, "gpu_host_call_us": round(call_us, 1),
                     "h2d_us": round(h2d_us, 1), "device_forward_us": round(kernel_us, 2), "d2h_us": round(d2h_us, 1),
                     "h2d_GBps": round(x.nbytes / h2d_us / 1e3, 2),
                     "d2h_GBps": round((det.nbytes + app.nbytes) / d2h_us / 1e3, 2),
                     "cpu_scalar_us": round(cpu_us, 1), "cpu_over_gpu_call": round(cpu_us / call_us, 2),
                     "bit_exact_vs_restatement": same})
    out = {"mode": "ref-shapes", "source": "MultiLevelBatchSIMDBenchmark.java:29-36 (multi-level forward, PERIODIC)",
           "gpu_path": "vw_modwt_forward_f64 with VW_FLAG_HOST_MEMORY from pageable numpy arrays (the JNI shape): "
                       "H2D, fused forward kernel, D2H, synchronize; median of %d calls" % reps,
           "cpu_path": "C restatement of MultiLevelMODWTTransform.decompose per signal (zero taps included), "
                       "1 thread, as the JMH scalar_multiLevel benchmark (Scope.Thread)",
           "shapes": rows}
    line = json.dumps(out)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(line + "\n")
    print(line, flush=True)


def ref_shapes_cpu(x, w, J, det, app):
    """CPU leg of --ref-shapes (the checker / baseline, outside any GPU timing): the restatement of
    vectorwave-core's decompose per signal on one thread; also checks the GPU rows bit for bit."""
    import numpy as np
    from oracle import oracle as O

    lo, hi = w.lowPassDecomposition(), w.highPassDecomposition()
    same = True
    t0 = time.perf_counter()
    for b in range(x.shape[0]):
        d, a = O.decompose(x[b], lo, hi, O.PERIODIC, J)   # single-threaded at these N (vw_oracle.c)
        same = same and bool(np.array_equal(d, det[:, b, :]) and np.array_equal(a, app[b]))
    return (time.perf_counter() - t0) * 1e6, same


def dry_run(args, world, rank):
    """The N > 1 control path without a GPU: row blocks, barrier, max-over-ranks (gloo)."""
    import torch
    import torch.distributed as dist
    from vectorwave_amd.shard import shard_rows

    _, _, Bg, N, _, _ = CONFIGS[args.config]
    Bg = args.batch or Bg
    if world > 1:
        dist.init_process_group("gloo")
    start, rows = shard_rows(Bg, world, rank)
    elapsed = 0.001 * (rank + 1)
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
        blocks = [None] * world
        dist.all_gather_object(blocks, (rank, start, rows, os.environ.get("LOCAL_RANK")))
        dist.destroy_process_group()
    else:
        blocks = [(rank, start, rows, os.environ.get("LOCAL_RANK", "0"))]
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "global_batch": Bg, "blocks": blocks,
                          "max_elapsed": elapsed}), flush=True)


class Workload:
    """Device buffers + the two passes of one config over `rows` signals, as C-ABI calls."""

    def __init__(self, eng, w, J, rows, N, dtype, pipeline, row_offset, torch):
        from vectorwave_amd import _native as nat
        self.nat, self.eng, self.lib = nat, eng, eng.lib
        self.w, self.J, self.rows, self.N, self.pipeline = w, J, rows, N, pipeline
        self.f32 = dtype == "f32"
        tdt = torch.float32 if self.f32 else torch.float64
        dev = torch.device("cuda", eng.device)
        self.x = torch.empty((rows, N), dtype=tdt, device=dev)
        eng.fill_uniform(self.x, 42, offset=row_offset * N)
        self.y = torch.empty((rows, N), dtype=tdt, device=dev)
        if pipeline == "fwd+inv":
            self.det = torch.empty((J, rows, N), dtype=tdt, device=dev)
            self.app = torch.empty((rows, N), dtype=tdt, device=dev)
        else:
            self.thr = torch.empty((rows,), dtype=torch.float64, device=dev)
        eng.bind_torch_stream()
        lo, hi = w.lowPassDecomposition(), w.highPassDecomposition()
        self.L = len(lo)
        self.lo_a, self.hi_a = nat.taps_array(lo), nat.taps_array(hi)
        self.graphs = {}

    def _check(self, st):
        if st != 0:
            raise RuntimeError(f"engine status {st}: {self.nat.last_error()}")

    def passes(self, flags):
        """[(family, fn)] of one step."""
        nat, lib, w, J, N, B = self.nat, self.lib, self.w, self.J, self.N, self.rows
        p = lambda t: c_void_p(t.data_ptr())  # noqa: E731
        if self.pipeline == "fwd+inv":
            fwd = lib.vw_modwt_forward_f32 if self.f32 else lib.vw_modwt_forward_f64
            inv = lib.vw_modwt_inverse_f32 if self.f32 else lib.vw_modwt_inverse_f64
            xp, dp, ap, yp = p(self.x), p(self.det), p(self.app), p(self.y)
            return [
                ("forward", lambda: self._check(fwd(self.eng.ctx, xp, B, N, N, self.lo_a, self.hi_a, self.L,
                                                    w.wavelet_id, nat.PERIODIC, J, flags, dp, ap))),
                ("inverse", lambda: self._check(inv(self.eng.ctx, dp, ap, B, N, self.lo_a, self.hi_a, self.L,
                                                    w.wavelet_id, nat.PERIODIC, J, 0xFFFFFFFF, 0, flags, yp))),
            ]
        xp, yp, tp = p(self.x), p(self.y), p(self.thr)
        return [("denoise", lambda: self._check(lib.vw_swt_denoise_f64(
            self.eng.ctx, xp, B, N, N, self.lo_a, self.hi_a, self.L, w.wavelet_id, nat.PERIODIC, J, -1.0, 1, flags,
            yp, tp)))]

    def step_fn(self, flags):
        fns = [fn for _, fn in self.passes(flags)]

        def step():
            for fn in fns:
                fn()
        return step

    def close(self):
        for g in self.graphs.values():
            g.close()
        self.graphs.clear()


PASS_FAMILIES = {"forward": ("forward", "forward_level"), "inverse": ("inverse", "inverse_level"),
                 "sigma": ("sigma",)}


def measure(torch, dist, world, eng, wl, flags, mode, steps, warmup, settle_s, events):
    """Settle, warm up, then time exactly `steps` steps between barrier + synchronize.

    mode "graph-k" (default): the K timed steps are recorded once into ONE graph and replayed once --
    no host work inside the timed region; with `events`, every kernel launch is bracketed by HIP
    event nodes inside that graph (live per-kernel times of the timed steps).  "graph-step": a
    one-step graph replayed K times.  "direct": C-ABI calls (events via the engine's launch timer).
    Returns ((device_elapsed_s, host_elapsed_s), settle (s, steps), {family: (total_ms, launches)},
    timed steps sampled).
    """
    step = wl.step_fn(flags)
    step()  # outside any capture: LDS attributes, workspaces, occupancy queries
    torch.cuda.synchronize()
    if mode == "direct":
        run1 = step
    else:
        g1 = eng.capture(step)
        wl.graphs[("step", flags)] = g1
        run1 = lambda: g1.launch(1)  # noqa: E731
    st = settle(torch, run1, settle_s)
    for _ in range(warmup):
        run1()
    torch.cuda.synchronize()
    eng.reset_timing()
    sampled = 0
    if mode == "graph-k":
        # event nodes cost ~4 us each inside a graph: bracket the kernels of every `every`-th timed
        # step only (5 of 20, 50 of 200), the others run back to back as in production
        every = (4 if steps >= 8 else 1) if events else 0

        def record():
            nonlocal sampled
            for k in range(steps):
                on = events and k % every == 0
                sampled += on
                eng.enable_timing(on)
                step()
            eng.enable_timing(events)
        gk = eng.capture(record)
        wl.graphs[("k", flags)] = gk
        body = lambda: gk.launch(1)  # noqa: E731
    else:
        eng.enable_timing(events and mode == "direct")
        sampled = steps if events and mode == "direct" else 0
        body = lambda: [run1() for _ in range(steps)]  # noqa: E731
    # Timed region: barrier + synchronize, then the K steps bracketed by HIP events on the stream the
    # engine enqueues on (torch's current stream, bound by Workload), then synchronize.  No collective
    # lies inside [t0, t1]: the closing barrier of the contract comes after the clock is read.
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    body()
    ev1.record()
    torch.cuda.synchronize()
    host_elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    # device time of the K steps (first kernel start .. last kernel end on this rank's stream)
    elapsed = ev0.elapsed_time(ev1) * 1e-3
    fams = {}
    for k in ("forward", "inverse", "sigma", "forward_level", "inverse_level"):
        ms, n = eng.kernel_time(k)
        if n:
            fams[k] = (ms, n)
    eng.enable_timing(False)
    eng.reset_timing()
    return (elapsed, host_elapsed), st, fams, sampled


def max_over_ranks(torch, dist, world, v, dev):
    if world == 1:
        return v
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def settle(torch, run1, seconds):
    """Replay the step untimed until `seconds` have passed (GPU clock settle); returns (s, steps)."""
    if seconds <= 0:
        return 0.0, 0
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < seconds:
        for _ in range(10):
            run1()
        n += 10
        torch.cuda.synchronize()
    return time.perf_counter() - t0, n


def run(args, world, rank, local):
    import torch
    import torch.distributed as dist

    # VW_BENCH_DEVICE_MOD (rehearsal only): map ranks onto fewer GPUs (rank r -> r mod M)
    dmod = int(os.environ.get("VW_BENCH_DEVICE_MOD", "0"))
    local = local % dmod if dmod > 0 else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        # the only collectives are the timing barrier and the max over ranks of the elapsed time (host
        # scalars, after a device synchronize): gloo -- no data-path exchange exists, so no RCCL
        dist.init_process_group("gloo")

    import vectorwave_amd as vw
    from vectorwave_amd import _native as nat
    from vectorwave_amd.shard import shard_rows

    wname, J, Bg, N, dtype, pipeline = CONFIGS[args.config]
    Bg = args.batch or Bg
    wname = args.wavelet or wname
    w = vw.get_wavelet(wname)
    esz = 4 if dtype == "f32" else 8
    eng = vw.Engine.get(local)
    # all work on one dedicated (non-default, capturable) stream; the engine binds to it
    torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    flags = 0 if args.exact else nat.FLAG_FMA
    events = args.events == "inline"

    # ---- strong scaling (headline): rank r owns rows [start, start + rows) of the global batch
    start, rows = shard_rows(Bg, world, rank)
    wl = Workload(eng, w, J, rows, N, dtype, pipeline, start, torch)
    (elapsed, host_elapsed), (settle_s, settle_steps), fams, sampled = measure(
        torch, dist, world, eng, wl, flags, args.launch, args.steps, args.warmup, args.settle, events)
    elapsed = max_over_ranks(torch, dist, world, elapsed, dev)
    host_elapsed = max_over_ranks(torch, dist, world, host_elapsed, dev)
    value = Bg * N * args.steps / elapsed / 1e6
    # correctness guard on the timed buffers (outside the timed region): fails the run loudly
    check = verify(torch, wl, w, J, pipeline, flags, nat)
    checks = [None] * world
    if world > 1:
        dist.all_gather_object(checks, check)
    else:
        checks = [check]

    # algorithmic bytes per pass: forward reads x, writes J details + approx;
    # inverse reads J + 1 rows, writes y; the denoise sigma pass re-reads d_1
    units = rows * N
    pass_bytes = {"forward": (J + 2) * esz * units, "inverse": (J + 2) * esz * units, "sigma": esz * units}
    kernels = {k: {"launches_per_step": round(n / max(sampled, 1), 3), "ms_per_launch": round(ms / n, 5)}
               for k, (ms, n) in fams.items()}
    pass_ms = {}
    for p_, members in PASS_FAMILIES.items():
        tot = sum(fams[m][0] for m in members if m in fams)
        if tot > 0:
            pass_ms[p_] = tot / sampled
    roof = None
    if pass_ms:
        dom = max(pass_ms, key=lambda f: pass_ms[f])
        achieved = pass_bytes[dom] / (pass_ms[dom] * 1e-3) / 1e9
        traffic, tsrc = committed_traffic(args.config, dom, rows)
        members = [f"{m} x{kernels[m]['launches_per_step']:g}" for m in PASS_FAMILIES[dom] if m in kernels]
        roof = {"bound": "hbm", "kernel": f"{dom} pass ({', '.join(members)} launches per step)",
                "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
                "algorithmic_bytes_per_launch": pass_bytes[dom], "avg_launch_ms": round(pass_ms[dom], 5),
                # also the fraction of what a plain copy kernel reaches on this GPU
                "copy_ref_GBps": COPY_GBS, "copy_frac": round(achieved / COPY_GBS, 4),
                "copy_ref_source": "tools/membench.hip streaming copy, MI355X (profiles/r01/membench_v2.log)"}

    # ---- the other accumulation mode, same rows, timed the same way (beside the headline)
    alt = None
    if not args.no_alt:
        aflags = flags ^ nat.FLAG_FMA
        (ael, _), _, afams, asampled = measure(torch, dist, world, eng, wl, aflags, args.launch, args.steps,
                                               args.warmup, 0.0, events)
        ael = max_over_ranks(torch, dist, world, ael, dev)
        alt = {"accumulation": ACC_NAME[bool(aflags & nat.FLAG_FMA)],
               "value": round(Bg * N * args.steps / ael / 1e6, 2),
               "kernels_ms": {k: round(ms / n, 5) for k, (ms, n) in afams.items()}}
    wl.close()
    del wl

    # ---- weak scaling (N > 1): every rank owns a full per-GPU batch of Bg rows (the N = 1 workload)
    weak = None
    if world > 1 and not args.no_weak:
        wk = Workload(eng, w, J, Bg, N, dtype, pipeline, rank * Bg, torch)
        (wel, _), _, _, _ = measure(torch, dist, world, eng, wk, flags, args.launch, args.steps, args.warmup,
                                    min(args.settle, 0.3), False)
        wel = max_over_ranks(torch, dist, world, wel, dev)
        weak = {"value": round(world * Bg * N * args.steps / wel / 1e6, 2), "batch_per_gpu": Bg,
                "ms_per_step": round(wel / args.steps * 1e3, 4), "global_batch": world * Bg}
        wk.close()

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
            "settle_s": round(settle_s, 3),
            "settle_steps": settle_steps,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "timing": {"value_from": "HIP events around the K timed steps on each rank's stream, max over ranks",
                       "device_s": round(elapsed, 7), "host_wall_s": round(host_elapsed, 7),
                       "host_wall_value": round(Bg * N * args.steps / host_elapsed / 1e6, 2),
                       "collective_inside_timed_region": False},
            "check": checks,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic: counter-based splitmix64 uniform[-1,1), seed 42, generated on device",
            "config": {
                "workload": f"{wname} MODWT J={J} {pipeline}, global batch {Bg} x {N} samples, {dtype}, PERIODIC",
                "wavelet": wname, "levels": J, "global_batch": Bg, "batch_per_gpu": rows, "signal_length": N,
                "boundary": "PERIODIC", "accumulation": ACC_NAME[bool(flags & nat.FLAG_FMA)],
                "parallelism": f"batch-shard x{world} (contiguous row blocks, no collective)",
                "launch": LAUNCH_DESC[args.launch],
                "passes_ms": {f: round(v, 5) for f, v in pass_ms.items()},
                "kernel_timing": (f"HIP events around every kernel launch of {sampled} of the {args.steps} timed "
                                  "steps (event nodes inside the replayed graph)" if args.launch == "graph-k" else
                                  "HIP events around every launch (engine timer)" if args.launch == "direct"
                                  else "none") if events else "none",
                "kernels": kernels,
                "other_accumulation": alt,
            },
            "weak_scaling": weak,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def committed_traffic(config, fam, rows=0):
    """HBM bytes per pass from the committed rocprofv3 PMC capture (FETCH_SIZE x2 + WRITE_SIZE, gfx950
    correction), with the commit it was captured at -- PMC needs its own rocprofv3 pass."""
    path = os.path.join(ROOT, "profiles", f"hbm_traffic_{config}.json")
    if not os.path.exists(path):
        return None, None
    try:
        with open(path) as fh:
            tj = json.load(fh)
        ent = tj.get(fam) or {}
        b = ent.get("bytes_per_launch")
        if b is not None and tj.get("rows") and rows:
            b = round(b * rows / tj["rows"])  # captured on the full batch; this rank's share
        src = f"profiles/hbm_traffic_{config}.json (rocprofv3 PMC, captured at {tj.get('captured_at', '?')})"
        return b, (src if b is not None else None)
    except Exception:
        return None, None


def verify(torch, wl, w, J, pipeline, flags, nat):
    """Post-timing correctness guard (the checker, outside the timed region): the first and last of this
    rank's rows of the timed buffers against the C restatement of vectorwave-core (oracle/, test
    infrastructure), plus perfect reconstruction over every row.  Raises -- no number is printed for a
    kernel that writes wrong values.  Bars as tests/test_gpu_headline.py: FMA <= 1e-12, EXACT bit-exact
    (fp64); fp32 1e-5 * max|x| * J."""
    from oracle import oracle as O

    lo, hi = w.lowPassDecomposition(), w.highPassDecomposition()
    rl, rh = w.lowPassReconstruction(), w.highPassReconstruction()
    torch.cuda.synchronize()
    fma = bool(flags & nat.FLAG_FMA)
    rows = sorted({0, wl.rows - 1})
    worst = 0.0
    tol = 0.0
    for r in rows:
        xr = wl.x[r].double().cpu().numpy()
        if wl.f32:
            tol = 1e-5 * float(abs(xr).max()) * J
        elif fma:
            tol = 1e-12
        if pipeline == "fwd+inv":
            d, a = O.decompose(xr, lo, hi, O.PERIODIC, J, core=False)
            y_ref = O.reconstruct(d, a, rl, rh, O.PERIODIC, w.wavelet_id)
            got = [(wl.det[:, r, :], d), (wl.app[r], a), (wl.y[r], y_ref)]
        else:
            y_ref, t_ref = O.swt_denoise(xr, lo, hi, O.PERIODIC, J, -1.0, True, w.wavelet_id)
            got = [(wl.y[r], y_ref)]
        for g, ref in got:
            e = float(abs(g.double().cpu().numpy() - ref).max())
            worst = max(worst, e)
    pr = None
    if pipeline == "fwd+inv":
        pr = float((wl.y.double() - wl.x.double()).abs().max().item())
    pr_bar = 1e-3 if wl.f32 else 1e-8   # truncated published taps (db8 J=10: ~1e-9; SURVEY.md key fact 5)
    ok = worst <= tol and (pr is None or pr < pr_bar)
    res = {"rows": rows, "max_abs_vs_oracle": worst, "tol": tol, "pr_max_abs": pr, "pr_bar": pr_bar, "ok": ok}
    if not ok:
        raise RuntimeError(f"bench correctness guard failed: {res}")
    return res


def cpu_baseline(w, J, N, dtype, pipeline, seconds):
    """vectorwave-core's scalar loops (C restatement, zero taps included) on this host's cores, bounded sample."""
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
