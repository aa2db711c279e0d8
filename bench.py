#!/usr/bin/env python3
"""bench.py -- MODWT fwd+inv throughput on MI355X (BASELINE.json metric), one process per GPU.

Default workload (BASELINE.json configs[1]): db4, J=6, forward + inverse of a GLOBAL batch of
4096 x 4096 fp64 signals, split across the N GPUs by contiguous row blocks (shard_rows; strong
scaling) -- no collective on the data path.  With N > 1 the same per-GPU work as at
N = 1 (4096 rows per rank) is timed afterwards and reported as `weak_scaling`.

A "step" = one multi-level forward pass + one multi-level inverse pass over the rank's rows, inputs
already resident in HBM (generated on device by the counter-based generator).  Each pass is
recorded once into a HIP graph through the C ABI (vw_capture_begin / vw_graph_launch): the timed
loop replays the graphs, so host-side planning and kernel-argument packing are not on the clock --
at 8 GPUs a pass is ~30 us of GPU work.

Clock settle: an MI355X leaving idle runs the first ~50 ms of load below its steady clock (measured
per step, profiles/r02/trace_*.log).  Before the W warmup steps the step is replayed for
`--settle` seconds (default 1.0, untimed, reported as settle_s / settle_steps), then W warmup
steps, then exactly K timed steps between barrier + device synchronize on both sides; the elapsed
time is the max over ranks.

`--gpus N` without torchrun: the parent spawns N rank processes (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_*) before any GPU call and relays rank 0's line.  Under torchrun each process is one rank.

Prints ONE JSON line (rank 0) with value = Msamples/s of the whole job, a `roofline` object for the
dominant pass (algorithmic bytes per launch / its average HIP-event duration, events recorded around
every graph replay inside the timed loop) and a `cpu_baseline` object (the C restatement of
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
    True: "fma (fused multiply-add per tap; max-abs error vs vectorwave-core < 1e-12, tests/test_gpu_parity.py)",
    False: "exact (separate multiply and add in the reference's tap order; bit-identical to vectorwave-core)",
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (/opt/skills/guides/MI355X_MICROARCH.md)

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
    p.add_argument("--no-graph", action="store_true", help="direct C-ABI calls in the timed loop instead of graphs")
    p.add_argument("--events", default="inline", choices=["inline", "none"],
                   help="HIP events around every pass inside the timed loop (inline) or none")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=6.0, help="target wall time of the CPU baseline sample")
    p.add_argument("--dry-run", action="store_true",
                   help="CPU only: launch the ranks, shard, run the timing collectives (gloo), print the plan")
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
    run(args, world, rank, local)


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

    def runners(self, flags, graph):
        """[(family, run())]: graph replays (recorded once) or direct calls."""
        out = []
        for fam, fn in self.passes(flags):
            if graph:
                key = (fam, flags)
                if key not in self.graphs:
                    fn()  # first call outside capture: LDS attributes, workspaces, occupancy queries
                    self.graphs[key] = self.eng.capture(fn)
                g = self.graphs[key]
                out.append((fam, lambda g=g: g.launch(1)))
            else:
                out.append((fam, fn))
        return out

    def close(self):
        for g in self.graphs.values():
            g.close()
        self.graphs.clear()


def timed(torch, dist, world, runs, steps, events):
    """K steps between barrier + synchronize; per-pass HIP events inside the loop. -> (elapsed, {fam: [ms]})."""
    evs = []
    if events:
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(len(runs) + 1)] for _ in range(steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        if events:
            evs[k][0].record()
        for i, (_, run) in enumerate(runs):
            run()
            if events:
                evs[k][i + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    per = {fam: [] for fam, _ in runs}
    for e in evs:
        for i, (fam, _) in enumerate(runs):
            per[fam].append(e[i].elapsed_time(e[i + 1]))
    return elapsed, per


def max_over_ranks(torch, dist, world, v, dev):
    if world == 1:
        return v
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def settle(torch, runs, seconds):
    """Replay the step untimed until `seconds` have passed (GPU clock settle); returns (s, steps)."""
    if seconds <= 0:
        return 0.0, 0
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < seconds:
        for _ in range(10):
            for _, run in runs:
                run()
        n += 10
        torch.cuda.synchronize()
    return time.perf_counter() - t0, n


def launch_breakdown(eng, wl, flags, steps):
    """Kernel launches per pass and per-family HIP-event times from the engine's own launch timer
    (a short direct-call replay after the timed region; every kernel launch bracketed)."""
    eng.reset_timing()
    eng.enable_timing(True)
    for _ in range(steps):
        for _, fn in wl.passes(flags):
            fn()
    import torch
    torch.cuda.synchronize()
    eng.enable_timing(False)
    out = {}
    for k in ("forward", "inverse", "sigma", "forward_level", "inverse_level"):
        ms, n = eng.kernel_time(k)
        if n:
            out[k] = {"launches_per_step": n / steps, "ms_per_launch": round(ms / n, 5)}
    return out


def run(args, world, rank, local):
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

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
    graph = not args.no_graph
    events = args.events == "inline"

    # ---- strong scaling (headline): rank r owns rows [start, start + rows) of the global batch
    start, rows = shard_rows(Bg, world, rank)
    wl = Workload(eng, w, J, rows, N, dtype, pipeline, start, torch)
    runs = wl.runners(flags, graph)
    settle_s, settle_steps = settle(torch, runs, args.settle)
    for _ in range(args.warmup):
        for _, run_ in runs:
            run_()
    torch.cuda.synchronize()
    elapsed, per = timed(torch, dist, world, runs, args.steps, events)
    elapsed = max_over_ranks(torch, dist, world, elapsed, dev)
    value = Bg * N * args.steps / elapsed / 1e6

    # algorithmic bytes per pass: forward reads x, writes J details + approx;
    # inverse reads J + 1 rows, writes y; denoise = forward + the d_1 median re-read + inverse
    units = rows * N
    pass_bytes = {"forward": (J + 2) * esz * units, "inverse": (J + 2) * esz * units,
                  "denoise": (2 * (J + 2) + 1) * esz * units}
    fam_ms = {f: sum(v) / len(v) for f, v in per.items() if v}
    breakdown = launch_breakdown(eng, wl, flags, min(args.steps, 20))
    roof = None
    if fam_ms:
        dom = max(fam_ms, key=lambda f: fam_ms[f])
        achieved = pass_bytes[dom] / (fam_ms[dom] * 1e-3) / 1e9
        traffic, tsrc = committed_traffic(args.config, dom)
        kern = {"forward": "forward pass", "inverse": "inverse pass", "denoise": "denoise step"}[dom]
        roof = {"bound": "hbm", "kernel": f"{kern} ({launches_desc(breakdown, dom)})", "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic, "traffic_source": tsrc,
                "algorithmic_bytes_per_launch": pass_bytes[dom], "avg_launch_ms": round(fam_ms[dom], 5)}

    # ---- the other accumulation mode, same rows, timed the same way (beside the headline)
    alt = None
    if not args.no_alt:
        aflags = flags ^ nat.FLAG_FMA
        aruns = wl.runners(aflags, graph)
        for _ in range(args.warmup):
            for _, run_ in aruns:
                run_()
        torch.cuda.synchronize()
        ael, aper = timed(torch, dist, world, aruns, args.steps, events)
        ael = max_over_ranks(torch, dist, world, ael, dev)
        alt = {"accumulation": ACC_NAME[bool(aflags & nat.FLAG_FMA)],
               "value": round(Bg * N * args.steps / ael / 1e6, 2),
               "passes_ms": {f: round(sum(v) / len(v), 5) for f, v in aper.items() if v}}
    wl.close()
    del wl

    # ---- weak scaling (N > 1): every rank owns a full per-GPU batch of Bg rows (the N = 1 workload)
    weak = None
    if world > 1 and not args.no_weak:
        wk = Workload(eng, w, J, Bg, N, dtype, pipeline, rank * Bg, torch)
        wruns = wk.runners(flags, graph)
        settle(torch, wruns, min(args.settle, 0.3))
        for _ in range(args.warmup):
            for _, run_ in wruns:
                run_()
        torch.cuda.synchronize()
        wel, _ = timed(torch, dist, world, wruns, args.steps, False)
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
                "launch": "HIP graph per pass (vw_capture_begin / vw_graph_launch)" if graph else "direct C-ABI calls",
                "passes_ms": {f: round(v, 5) for f, v in fam_ms.items()},
                "pass_timing": "HIP events on the engine stream around every pass, inside the timed loop"
                if events else "none",
                "kernels": breakdown,
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


def launches_desc(breakdown, fam):
    keys = [fam, fam + "_level"] if fam != "denoise" else ["forward", "sigma", "inverse", "forward_level",
                                                           "inverse_level"]
    parts = [f"{k} x{v['launches_per_step']:g}" for k, v in breakdown.items() if k in keys]
    return ", ".join(parts) or fam


def committed_traffic(config, fam):
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
        src = f"profiles/hbm_traffic_{config}.json (rocprofv3 PMC, captured at {tj.get('captured_at', '?')})"
        return b, (src if b is not None else None)
    except Exception:
        return None, None


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
