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
from ctypes import byref, c_void_p

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# The accumulation claim of each config's line, naming the test and the tolerance that cover it.
ACC_FMA = {
    "db4": "fma (fused multiply-add per tap; max-abs error vs vectorwave-core <= 1e-12 at this configuration, "
           "4096 x 4096 in the bench's own kernel policy: tests/test_gpu_headline.py)",
    "sym8-denoise": "fma (fused multiply-add per tap; output within 1e-12 * max|x| and thresholds within 1e-12 "
                    "relative of vectorwave-core at the config-3 shape sym8 J=8 N=16384: "
                    "tests/test_gpu_configs.py::test_config3_sym8_swt_j8_denoise_16384)",
    "db8-stream": "fma (fused multiply-add per tap; every level, approximation and inverse within 1e-12 of "
                  "vectorwave-extensions' BatchMODWT on a db8 J=10 2^20 block: "
                  "tests/test_gpu_configs.py::test_config4_db8_j10_block_2p20)",
    "coif5-f32": "fma fp32 (fused multiply-add per tap in fp32; within 1e-5 * max|x| * J of the fp64 "
                 "restatement, SURVEY.md §8d: tests/test_gpu_configs.py::test_config5_coif5_f32_j6_8192)",
}
ACC_EXACT = {
    "db4": "exact (separate multiply and add in the reference's tap order; bit-identical to vectorwave-core: "
           "tests/test_gpu_headline.py, tests/test_gpu_parity.py)",
    "sym8-denoise": "exact (bit-identical output and thresholds: tests/test_gpu_configs.py)",
    "db8-stream": "exact (bit-identical in all 10 levels and the inverse: tests/test_gpu_configs.py)",
    "coif5-f32": "exact fp32 (separate multiply and add in fp32; within 1e-5 * max|x| * J of the fp64 "
                 "restatement: tests/test_gpu_configs.py)",
}


def acc_name(config, fma):
    return (ACC_FMA if fma else ACC_EXACT).get(config, "fma" if fma else "exact")
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (/opt/skills/guides/MI355X_MICROARCH.md)
# Vector-ALU peaks for the FMA work of the taps: fp32 from the microarchitecture guide (157.3 TFLOP/s
# vector), fp64 the MI355X spec sheet's 78.6 (the guide lists no fp64 figure); beside them the issue
# rates tools/valubench.hip measured on this GPU (profiles/r03/valubench.log)
VALU_PEAK_TFLOPS = {"f32": 157.3, "f64": 78.6}
VALU_MEASURED_TFLOPS = {"f32": {"v_fma_f32": 95.3, "v_pk_fma_f32": 117.4}, "f64": {"v_fma_f64": 61.6}}
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
    p.add_argument("--ref-nonfinite", default="off", choices=["on", "off"],
                   help="VW_FLAG_REF_NONFINITE (the unvalidated batch facade's NaN/Inf spread, vw_ref.hip) on the "
                        "timed calls: identical results for finite data; db4's kernels probe their rows in-line "
                        "and each pass adds one fix-up launch (-0.9 %% on db4, profiles/r06/ab_db4_ref_nonfinite_on_off_final_probe.log)")
    p.add_argument("--no-weak", action="store_true", help="N > 1: skip the weak-scaling measurement")
    p.add_argument("--launch", default="graph-k", choices=sorted(LAUNCH_DESC),
                   help="how the timed steps are issued (see measure())")
    p.add_argument("--events", default="inline", choices=["inline", "none"],
                   help="HIP events around every kernel launch inside the timed steps (inline) or none")
    p.add_argument("--contexts", type=int, default=0,
                   help="contexts (each on its own stream) sharing a GPU's rows; 0 = policy (see run())")
    p.add_argument("--rotate", type=int, default=0,
                   help="R buffer sets, step i working on set i mod R, so no step re-reads an input an earlier step "
                        "left in the 256 MiB Infinity Cache; 0 = auto (R * input bytes >= 512 MiB, R >= 2, "
                        "outputs rotated too); 1 = one set (the round-1..3 method)")
    p.add_argument("--rotate-outputs", action="store_true", help="explicit --rotate R: rotate the outputs too")
    p.add_argument("--no-isolated", action="store_true",
                   help="skip the isolated per-pass kernel timing reported in roofline.isolated")
    p.add_argument("--overlap-steps", action="store_true",
                   help="pipeline step i+1's forward with step i's inverse on two contexts (rotated buffer sets); "
                        "default when the rank has <= 2 signals per CU and --contexts is not given")
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


class Part:
    """One context's share of a rank's rows: its own vw_ctx, torch stream and buffers.

    `rotate` R > 1 keeps R input buffers (and, with `rotate_outputs`, R output sets) and step i uses set
    i mod R, so a buffer is re-read only after R steps of other traffic: with R * rows * N * size beyond
    the 256 MiB Infinity Cache no step can be served from what an earlier step left on die
    (`--rotate`).  Every set holds the same input values (same generator offset)."""

    def __init__(self, eng, stream, w, J, rows, N, dtype, pipeline, row_offset, torch, rotate=1,
                 rotate_outputs=False):
        from vectorwave_amd import _native as nat
        self.nat, self.eng, self.lib, self.stream = nat, eng, eng.lib, stream
        self.w, self.J, self.rows, self.N, self.pipeline = w, J, rows, N, pipeline
        self.f32 = dtype == "f32"
        tdt = torch.float32 if self.f32 else torch.float64
        dev = torch.device("cuda", eng.device)
        self.rotate = max(1, rotate)
        nout = self.rotate if rotate_outputs else 1
        self.sets = []
        with torch.cuda.stream(stream):
            for r in range(self.rotate):
                st = {"x": torch.empty((rows, N), dtype=tdt, device=dev)}
                eng.fill_uniform(st["x"], 42, offset=row_offset * N)
                if r < nout:
                    st["y"] = torch.empty((rows, N), dtype=tdt, device=dev)
                    if pipeline == "fwd+inv":
                        st["det"] = torch.empty((J, rows, N), dtype=tdt, device=dev)
                        st["app"] = torch.empty((rows, N), dtype=tdt, device=dev)
                    else:
                        st["thr"] = torch.empty((rows,), dtype=torch.float64, device=dev)
                else:
                    st.update({k: v for k, v in self.sets[0].items() if k != "x"})
                self.sets.append(st)
            eng.bind_torch_stream()
        self.last = 0   # the set the most recent step used (verify() checks that one)
        lo, hi = w.lowPassDecomposition(), w.highPassDecomposition()
        self.L = len(lo)
        self.lo_a, self.hi_a = nat.taps_array(lo), nat.taps_array(hi)

    def __getattr__(self, k):  # x / y / det / app / thr of the most recently used set
        if k in ("x", "y", "det", "app", "thr"):
            return self.__dict__["sets"][self.__dict__["last"]][k]
        raise AttributeError(k)

    def footprint(self):
        seen, tot = set(), 0
        for st in self.sets:
            for t in st.values():
                if t.data_ptr() not in seen:
                    seen.add(t.data_ptr())
                    tot += t.numel() * t.element_size()
        return tot

    def _check(self, st):
        if st != 0:
            raise RuntimeError(f"engine status {st}: {self.nat.last_error()}")

    def step_fn(self, flags, only=None):
        """One step of this part: the config's passes over its rows, as C-ABI calls on its context.
        Returns step(i): step i works on buffer set i mod R.  only="forward" / "inverse" (fwd+inv, for the
        isolated kernel timing): that pass alone (the inverse reads the coefficients a full step left)."""
        nat, lib, w, J, N, B = self.nat, self.lib, self.w, self.J, self.N, self.rows
        p = lambda t: c_void_p(t.data_ptr())  # noqa: E731
        ctx = self.eng.ctx
        if self.pipeline == "fwd+inv":
            fwd = lib.vw_modwt_forward_f32 if self.f32 else lib.vw_modwt_forward_f64
            inv = lib.vw_modwt_inverse_f32 if self.f32 else lib.vw_modwt_inverse_f64
            ptrs = [(p(s["x"]), p(s["det"]), p(s["app"]), p(s["y"])) for s in self.sets]

            def step(i=0):
                r = i % self.rotate
                self.last = r
                xp, dp, ap, yp = ptrs[r]
                if only != "inverse":
                    self._check(fwd(ctx, xp, B, N, N, self.lo_a, self.hi_a, self.L, w.wavelet_id, nat.PERIODIC, J,
                                    flags, dp, ap))
                if only != "forward":
                    self._check(inv(ctx, dp, ap, B, N, self.lo_a, self.hi_a, self.L, w.wavelet_id, nat.PERIODIC, J,
                                    0xFFFFFFFF, 0, flags, yp))
            return step
        ptrs = [(p(s["x"]), p(s["y"]), p(s["thr"])) for s in self.sets]

        def step(i=0):
            r = i % self.rotate
            self.last = r
            xp, yp, tp = ptrs[r]
            self._check(lib.vw_swt_denoise_f64(ctx, xp, B, N, N, self.lo_a, self.hi_a, self.L, w.wavelet_id,
                                               nat.PERIODIC, J, -1.0, 1, flags, yp, tp))
        return step


def measure_overlap(torch, dist, world, pt, eng_i, stream_i, flags, steps, warmup, settle_s):
    """Step schedule `overlap-steps`: consecutive steps pipelined over two contexts on two streams --
    every forward on the part's context / stream F, every inverse on context I / stream I, step i's
    inverse after its forward (event), step i's forward after step i - R's inverse (the buffer set it
    overwrites), R >= 2 rotated output sets.  So step i + 1's forward overlaps step i's inverse; each
    step still runs its full forward and inverse.  The steps are issued by the engine itself
    (vw_pipeline_run: one C call for all K steps) -- not a Python call per pass, whose
    ~50 us per step at 512 rows was as long as the GPU step.  Graph capture is no substitute: the same
    steps recorded into one graph lost the overlap (35.6K vs 42.3K Msamples/s at 512 rows,
    profiles/r04/ab_overlap_graph.log).  Returns (device s of the K timed steps -- events on stream F
    around them, stream I joined back --, host wall s of the same interval, host s spent issuing them)."""
    nat, lib = pt.nat, pt.lib
    R = pt.rotate
    assert R >= 2 and pt.pipeline == "fwd+inv", "overlapped steps need >= 2 buffer sets (outputs too) and fwd+inv"
    sF, sI = pt.stream, stream_i
    eF, eI = pt.eng, eng_i
    with torch.cuda.stream(sI):
        eI.bind_torch_stream()
    with torch.cuda.stream(sF):
        eF.bind_torch_stream()
    arr = lambda key: (c_void_p * R)(*[st[key].data_ptr() for st in pt.sets])  # noqa: E731
    pipe = c_void_p()
    pt._check(lib.vw_pipeline_create(eF.ctx, eI.ctx, 4 if pt.f32 else 8, R, arr("x"), arr("det"), arr("app"),
                                     arr("y"), pt.rows, pt.N, pt.lo_a, pt.hi_a, pt.L, pt.w.wavelet_id, nat.PERIODIC,
                                     pt.J, flags, byref(pipe)))
    try:
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < settle_s or n < warmup:
            k = 20 if n >= warmup else max(1, min(20, warmup - n))
            pt._check(lib.vw_pipeline_run(pipe, k))
            n += k
            torch.cuda.synchronize()
        pt._check(lib.vw_pipeline_join(pipe))
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        h0 = time.perf_counter()
        ev0.record(sF)
        pt._check(lib.vw_pipeline_run(pipe, steps))
        h1 = time.perf_counter()
        pt._check(lib.vw_pipeline_join(pipe))
        ev1.record(sF)
        torch.cuda.synchronize()
        h2 = time.perf_counter()
        pt.last = int(lib.vw_pipeline_last_set(pipe))
        if world > 1:
            dist.barrier()
    finally:
        lib.vw_pipeline_destroy(pipe)
    return ev0.elapsed_time(ev1) * 1e-3, h2 - h0, h1 - h0


class Workload:
    """A rank's rows split over K contexts of its GPU (contiguous blocks, shard_rows), each on its own
    stream: with K = 2 one part's inverse overlaps the other's forward tail (and the two parts' first
    row loads) -- the in-process form of DeviceGroup on one device (tools/concurrency_probe.py:
    4096 x 4096 db4 0.383 -> 0.369 ms per step at K = 2)."""

    def __init__(self, engines, streams, w, J, rows, N, dtype, pipeline, row_offset, torch, rotate=1,
                 rotate_outputs=False):
        from vectorwave_amd.shard import shard_rows
        K = min(len(engines), rows)
        self.parts = []
        for k in range(K):
            s0, r = shard_rows(rows, K, k)
            self.parts.append(Part(engines[k], streams[k], w, J, r, N, dtype, pipeline, row_offset + s0, torch,
                                   rotate, rotate_outputs))
        self.rows, self.N, self.J, self.pipeline = rows, N, J, pipeline
        self.f32 = dtype == "f32"
        self.graphs = []
        self.overlap = None        # (inverse engine, stream) of the overlapped-steps schedule
        self.host_issue_s = None   # overlapped steps: host seconds spent issuing the K timed steps

    def close(self):
        for g in self.graphs:
            g.close()
        self.graphs.clear()


PASS_FAMILIES = {"forward": ("forward", "forward_level"), "inverse": ("inverse", "inverse_level"),
                 "sigma": ("sigma",)}
FAMILIES = ("forward", "inverse", "sigma", "forward_level", "inverse_level")


def measure(torch, dist, world, wl, flags, mode, steps, warmup, settle_s, events, only=None):
    """Settle, warm up, then time exactly `steps` steps between barrier + synchronize.

    Every part records its steps into HIP graphs on its own context and stream; the main stream forks
    to the parts' streams and joins them (events), so the timed region is ONE event pair on the main
    stream.  mode "graph-k" (default): the K timed steps recorded once per part and replayed once --
    no host work inside the timed region; with `events`, every kernel launch is bracketed by HIP event
    nodes inside the graphs.  "graph-step": a one-step graph replayed K times.  "direct": C-ABI calls.
    Returns ((device_elapsed_s, host_elapsed_s), settle (s, steps), {family: (total_ms, launches)},
    timed steps sampled, {pass: wall ms per sampled step across parts}).
    """
    if getattr(wl, "overlap", None):
        eng_i, stream_i = wl.overlap
        el, host_el, issue = measure_overlap(torch, dist, world, wl.parts[0], eng_i, stream_i, flags, steps, warmup,
                                             settle_s)
        wl.host_issue_s = issue
        return (el, host_el), (settle_s, 0), {}, 0, {}
    parts = wl.parts
    main = torch.cuda.current_stream()
    fns = [pt.step_fn(flags, only) for pt in parts]

    def fork_join(fn):
        # the part on the main stream itself needs no fork / join (no cross-stream latency at K = 1)
        others = [k for k, pt in enumerate(parts) if pt.stream != main]
        ev = None
        if others:
            ev = torch.cuda.Event()
            ev.record(main)
        ends = []
        for k, pt in enumerate(parts):
            if k in others:
                pt.stream.wait_event(ev)
            with torch.cuda.stream(pt.stream):
                fn(k)
                if k in others:
                    e = torch.cuda.Event()
                    e.record(pt.stream)
                    ends.append(e)
        for e in ends:
            main.wait_event(e)

    fork_join(lambda k: fns[k]())  # outside any capture: LDS attributes, workspaces, occupancy queries
    torch.cuda.synchronize()

    def capture_all(fn_of):
        gs = []
        for k, pt in enumerate(parts):
            with torch.cuda.stream(pt.stream):
                gs.append(pt.eng.capture(fn_of(k)))
        wl.graphs.extend(gs)
        return gs

    R = max(pt.rotate for pt in parts)
    ctr = [0]

    def next_i():
        ctr[0] += 1
        return ctr[0] - 1

    if mode == "direct":
        def run1():
            i = next_i()
            fork_join(lambda k: fns[k](i))
    else:
        # one single-step graph per buffer set, cycled (settle / warmup / graph-step mode)
        g1s = [capture_all(lambda k, r=r: (lambda: fns[k](r))) for r in range(R)]

        def run1():
            g = g1s[next_i() % R]
            fork_join(lambda k: g[k].launch(1))
    # The timed body is prepared BEFORE the settle / warmup, so the timed replay follows the warmup with
    # no host-side capture gap in between (a GPU idle for milliseconds drops its clock again).
    sampled = 0
    if mode == "graph-k":
        # event nodes cost ~4 us each inside a graph: bracket the kernels of every `every`-th timed
        # step only (5 of 20, 50 of 200), the others run back to back as in production
        every = (4 if steps >= 8 else 1) if events else 0
        sampled = sum(1 for k in range(steps) if events and k % every == 0)

        def record_of(k):
            eng = parts[k].eng

            def record():
                for i in range(steps):
                    eng.enable_timing(events and i % every == 0)
                    fns[k](i)
                eng.enable_timing(False)
            return record
        gk = capture_all(record_of)
        body = lambda: fork_join(lambda k: gk[k].launch(1))  # noqa: E731
    else:
        sampled = steps if events and mode == "direct" else 0
        body = lambda: [run1() for _ in range(steps)]  # noqa: E731
    st = settle(torch, run1, settle_s)
    for _ in range(warmup):
        run1()
    torch.cuda.synchronize()
    for pt in parts:
        pt.eng.reset_timing()
        # graph replays report their event nodes only while timing is on; direct calls are timed by it
        pt.eng.enable_timing(events and mode in ("graph-k", "direct"))
    # Timed region: barrier + synchronize, then the K steps of every part between two HIP events on
    # the main stream (fork / join), then synchronize.  No collective lies inside [t0, t1]: the closing
    # barrier of the contract comes after the clock is read.
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(main)
    body()
    ev1.record(main)
    torch.cuda.synchronize()
    host_elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    elapsed = ev0.elapsed_time(ev1) * 1e-3  # device time of the K steps of all parts
    # per family: launch durations; per pass: the wall window of its launches across the parts, per
    # sampled step (parts overlap, so a pass's window is what its bytes moved in)
    fams, spans = {}, {}
    for f in FAMILIES:
        sp = [pt.eng.kernel_spans(f, ev0) if events and sampled else [] for pt in parts]
        n = sum(len(x) for x in sp)
        if n:
            fams[f] = (sum(e - s for x in sp for s, e in x), n)
            spans[f] = sp
    pass_ms = {}
    for p_, members in PASS_FAMILIES.items():
        wins = []
        for i in range(sampled):
            lo_, hi_ = None, None
            for m in members:
                for x in spans.get(m, []):
                    per = len(x) // sampled if sampled else 0
                    for s_, e_ in x[i * per:(i + 1) * per]:
                        lo_ = s_ if lo_ is None else min(lo_, s_)
                        hi_ = e_ if hi_ is None else max(hi_, e_)
            if lo_ is not None:
                wins.append(hi_ - lo_)
        if wins:
            pass_ms[p_] = sum(wins) / len(wins)
    for pt in parts:
        pt.eng.enable_timing(False)
        pt.eng.reset_timing()
    return (elapsed, host_elapsed), st, fams, sampled, pass_ms


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


def plan_schedule(args, rows, N, esz, cus, pipeline):
    """(contexts K, overlapped steps?, (buffer sets R, outputs rotated?)) for `rows` signals on one GPU.

    Contexts per GPU: K parts of the rows, each on its own context + stream (--contexts; 0 = policy: 2
    above 2 signals per CU -- measured on MI355X, db4 4096 x 4096: 43.6-44.0K -> 44.7-45.7K; 1024 rows:
    39.4K -> 44.1K; 512 rows: 37.0K -> 36.1K, profiles/r03/ab_contexts.log; 4 at >= 16 signals per CU of
    <= 4096 samples -- round 5, same box, three alternations, db4 4096 x 4096: 2 contexts 45.2-45.6K, 3
    45.1-46.5K, 4 46.0-46.5K, 8 45.3-45.5K, profiles/r05/ab_contexts_4096.log).

    Buffer sets: with one set the same 128 MiB input was re-read every step and stayed in
    the Infinity Cache (the persistent forward's LDS-DMA allocates there, the streaming loads and stores
    around it are non-temporal): same box, db4 4096 x 4096, forward 0.163-0.164 ms with one set vs
    0.187-0.197 ms with three (profiles/r04/ab_rotate_4096.log).  So every step reads a fresh input:
    R * input >= 512 MiB, R >= 2.

    Step schedule: `overlap` pipelines consecutive steps over two contexts (step i+1's forward beside step
    i's inverse, measure_overlap); otherwise the K contexts split the rows.  Policy (measured on MI355X,
    db4 J=6, rotated sets; profiles/r04/ab_overlap_direct_512.log, ab_overlap_direct_4096.log,
    ab_overlap_graph.log): at <= 2 signals per CU (the 8-GPU shard of the headline: 512 rows) the passes
    are short and each leaves the GPU half idle at its ends, so overlapping consecutive steps wins
    (37.7-38.0K -> 42.1-42.4K) while splitting the rows over two contexts loses (34.9-35.2K); from 1024
    rows on two contexts win (42.3K vs 37.3-37.5K at 1024, 42.2-44.2K vs 40.0-40.6K at 4096).  Only for
    signals the one-workgroup-per-signal kernels hold (N <= 16384): the long-signal kernels tile every
    signal over many workgroups, and db8-stream (256 x 2^20) runs 15.1-15.3K sequentially vs 14.7-14.8K
    overlapped (profiles/r04/ab_schedule_db8.log)."""
    K = args.contexts or (4 if rows >= 16 * cus and N <= 4096 else 2 if rows > 2 * cus else 1)
    R = args.rotate or max(2, -(-(512 << 20) // max(rows * N * esz, 1)))
    rot = (R, bool(args.rotate_outputs or not args.rotate))
    overlap = pipeline == "fwd+inv" and (args.overlap_steps or (not args.contexts and rows <= 2 * cus and N <= 16384))
    if overlap:
        K = 1
        rot = (max(rot[0], 2), True)
    return K, overlap, rot


def make_engines(vw, torch, dev, local, main, K, overlap):
    """K contexts (the process-wide one first) with their streams (main first), plus the inverse context
    and stream of the overlapped-steps schedule.  Extra contexts are closed by close_engines."""
    engines = [vw.Engine.get(local)] + [vw.Engine(local) for _ in range(K - 1)]
    streams = [main] + [torch.cuda.Stream(device=dev) for _ in range(K - 1)]
    ov = (vw.Engine(local), torch.cuda.Stream(device=dev)) if overlap else None
    return engines, streams, ov


def close_engines(engines, ov):
    for e in engines[1:] + ([ov[0]] if ov else []):
        e.close()


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
    # the main stream (fork / join and the timing events; context 0 runs on it) and one capturable stream
    # per further context
    main = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(main)
    flags = 0 if args.exact else nat.FLAG_FMA
    ref_nf = args.ref_nonfinite == "on"
    if ref_nf:
        flags |= nat.FLAG_REF_NONFINITE
    events = args.events == "inline"

    # ---- strong scaling (headline): rank r owns rows [start, start + rows) of the global batch
    start, rows = shard_rows(Bg, world, rank)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    K, overlap, rot = plan_schedule(args, rows, N, esz, cus, pipeline)
    engines, streams, ov = make_engines(vw, torch, dev, local, main, K, overlap)
    wl = Workload(engines, streams, w, J, rows, N, dtype, pipeline, start, torch, *rot)
    wl.overlap = ov
    footprint = sum(pt.footprint() for pt in wl.parts)
    # With overlapping launches (K > 1 contexts, overlapped steps) a launch's duration says nothing about the
    # kernel's own rate: the roofline takes it from a one-context timing after the timed region (below), so the
    # timed region itself carries no per-kernel event nodes (~4 us each inside a graph; db4 4096 x 4096, same
    # box: 44.2-44.4K with them, 44.6-44.8K without, profiles/r06/ab_db4_launch_modes.log)
    events_timed = events and not (K > 1 or overlap)
    (elapsed, host_elapsed), (settle_s, settle_steps), fams, sampled, pass_ms = measure(
        torch, dist, world, wl, flags, args.launch, args.steps, args.warmup, args.settle, events_timed)
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
    # Kernel roofline (the dominant pass): with K > 1 contexts the passes of the parts
    # overlap, so a launch's duration says nothing about the kernel's own rate; the kernels are then
    # timed once more by ONE context over the same rows (after the headline's timed region, same
    # graph method).  With K = 1 the headline's own launches are used.
    kfams, ksampled, kpass_ms = fams, sampled, pass_ms
    if (K > 1 or overlap) and events:
        wk1 = Workload(engines[:1], streams[:1], w, J, rows, N, dtype, pipeline, start, torch, *rot)
        _, _, kfams, ksampled, kpass_ms = measure(torch, dist, world, wk1, flags, args.launch, args.steps,
                                                  args.warmup, min(args.settle, 0.5), events)
        wk1.close()
        del wk1
    # Isolated pass timing (fwd+inv): each pass alone, its launches back to back over the rotated buffer sets,
    # so a launch's duration holds its own traffic only -- in the step, the inverse also absorbs the write-back
    # of the forward's coefficient rows (sc1 stores) that drains while it runs.  Reported beside the roofline,
    # not in place of it.
    iso = None
    if events and pipeline == "fwd+inv" and not args.no_isolated:
        wki = Workload(engines[:1], streams[:1], w, J, rows, N, dtype, pipeline, start, torch, *rot)
        prime = wki.parts[0].step_fn(flags)
        with torch.cuda.stream(wki.parts[0].stream):
            for r in range(wki.parts[0].rotate):
                prime(r)   # every set holds the coefficients of its input
        torch.cuda.synchronize()
        iso = {}
        for fam in ("forward", "inverse"):
            _, _, _, _, ipass = measure(torch, dist, world, wki, flags, args.launch, args.steps, args.warmup,
                                        min(args.settle, 0.3), events, only=fam)
            if fam in ipass:
                iso[fam] = ipass[fam]
        wki.close()
        del wki
    kkernels = {k: {"launches_per_step": round(n / max(ksampled, 1), 3), "ms_per_launch": round(ms / n, 5)}
                for k, (ms, n) in kfams.items()}
    # algorithmic flops per pass: every level applies both filters, L taps each, one FMA (2 flop) per
    # tap and sample (ScalarOps.java:700-723, MultiLevelMODWTTransform.java:576-589)
    L = len(w.lowPassDecomposition())
    pass_flop = {"forward": 4 * L * J * units, "inverse": 4 * L * J * units, "sigma": 0}
    roof = None
    if kpass_ms:
        dom = max(kpass_ms, key=lambda f: kpass_ms[f])
        achieved = pass_bytes[dom] / (kpass_ms[dom] * 1e-3) / 1e9
        traffic, tsrc = committed_traffic(args.config, dom, rows)
        members = [f"{m} x{kkernels[m]['launches_per_step']:g}" for m in PASS_FAMILIES[dom] if m in kkernels]
        step_bytes = sum(pass_bytes[f] for f in kpass_ms)
        roof = {"bound": "hbm", "kernel": f"{dom} pass ({', '.join(members)} launches per step, one context)",
                "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
                "algorithmic_bytes_per_launch": pass_bytes[dom], "avg_launch_ms": round(kpass_ms[dom], 5),
                "duration_from": ("HIP event nodes around every launch of the sampled timed steps"
                                  + (f" of a one-context timing of the same {rows} rows (the headline's "
                                     f"{'overlapped steps' if overlap else f'{K} contexts'} overlap their "
                                     f"launches)" if (K > 1 or overlap) else "")),
                "kernels": kkernels,
                # also the fraction of what a plain copy kernel reaches on this GPU
                "copy_ref_GBps": COPY_GBS, "copy_frac": round(achieved / COPY_GBS, 4),
                "copy_ref_source": "tools/membench.hip streaming copy, MI355X (profiles/r01/membench_v2.log)",
                # the headline step as a whole: every pass's algorithmic bytes over the timed wall time
                "step": {"bytes": step_bytes, "ms": round(elapsed / args.steps * 1e3, 5),
                         "achieved": round(step_bytes / (elapsed / args.steps) / 1e9, 1),
                         "frac": round(step_bytes / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4)}}
        # the compute roof of the same pass: which floor (bytes at the HBM peak, flops at the VALU peak)
        # is higher decides the bound; long filters (coif5, L = 30) are VALU-bound, db4 is HBM-bound
        tflops = pass_flop[dom] / (kpass_ms[dom] * 1e-3) / 1e12
        vpk = VALU_PEAK_TFLOPS[dtype]
        hbm_floor = pass_bytes[dom] / (HBM_PEAK_GBS * 1e9) * 1e3
        valu_floor = pass_flop[dom] / (vpk * 1e12) * 1e3
        compute = {"flop_per_launch": pass_flop[dom], "achieved": round(tflops, 2), "peak": vpk, "unit": "TFLOP/s",
                   "frac": round(tflops / vpk, 4), "measured_issue_TFLOPs": VALU_MEASURED_TFLOPS[dtype],
                   "floor_ms": {"hbm": round(hbm_floor, 5), "valu": round(valu_floor, 5)}}
        roof["compute"] = compute
        if iso:
            roof["isolated"] = {
                "method": "each pass timed alone (its launches back to back over the rotated buffer sets, HIP event "
                          "nodes, one context); in the step the inverse also carries the drain of the forward's "
                          "write-back coefficient rows",
                "ms_per_launch": {f: round(v, 5) for f, v in iso.items()},
                "achieved_GBps": {f: round(pass_bytes[f] / (v * 1e-3) / 1e9, 1) for f, v in iso.items()},
                "frac": {f: round(pass_bytes[f] / (v * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) for f, v in iso.items()}}
        if valu_floor > hbm_floor:
            # VALU-bound pass: the headline roofline fields carry the compute roof; the HBM figures stay
            # beside them
            roof["hbm"] = {k: roof[k] for k in ("achieved", "peak", "unit", "frac")}
            roof.update({"bound": "valu", "achieved": compute["achieved"], "peak": vpk, "unit": "TFLOP/s",
                         "frac": compute["frac"]})

    # ---- the other accumulation mode, same rows, timed the same way (beside the headline)
    alt = None
    if not args.no_alt:
        aflags = flags ^ nat.FLAG_FMA
        (ael, _), _, afams, asampled, _ = measure(torch, dist, world, wl, aflags, args.launch, args.steps,
                                                  args.warmup, min(args.settle, 0.3), events)
        ael = max_over_ranks(torch, dist, world, ael, dev)
        alt = {"accumulation": acc_name(args.config, bool(aflags & nat.FLAG_FMA)),
               "value": round(Bg * N * args.steps / ael / 1e6, 2),
               "kernels_ms": {k: round(ms / n, 5) for k, (ms, n) in afams.items()}}
    host_issue = wl.host_issue_s
    wl.close()
    del wl

    # ---- weak scaling (N > 1): every rank owns a full per-GPU batch of Bg rows (the N = 1 workload)
    weak = None
    if world > 1 and not args.no_weak:
        # the full per-GPU batch gets its own schedule, buffer sets and contexts (reusing the
        # shard's R and overlap decision allocated 32 rotated 4096 x 4096 sets and overlapped 4096 rows)
        Kw, overlap_w, rot_w = plan_schedule(args, Bg, N, esz, cus, pipeline)
        engines_w, streams_w, ov_w = make_engines(vw, torch, dev, local, main, Kw, overlap_w)
        wk = Workload(engines_w, streams_w, w, J, Bg, N, dtype, pipeline, rank * Bg, torch, *rot_w)
        wk.overlap = ov_w
        (wel, _), _, _, _, _ = measure(torch, dist, world, wk, flags, args.launch, args.steps, args.warmup,
                                       min(args.settle, 0.3), False)
        wel = max_over_ranks(torch, dist, world, wel, dev)
        weak = {"value": round(world * Bg * N * args.steps / wel / 1e6, 2), "batch_per_gpu": Bg,
                "ms_per_step": round(wel / args.steps * 1e3, 4), "global_batch": world * Bg}
        wk.close()
        del wk
        close_engines(engines_w, ov_w)

    close_engines(engines, ov)

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
                       "host_issue_us_per_step": (round(host_issue / args.steps * 1e6, 2) if host_issue is not None
                                                  else None),
                       "host_issue_from": ("host clock around the one vw_pipeline_run call that enqueues the K "
                                           "timed steps (overlapped steps)" if host_issue is not None else
                                           "graph replay: one launch per context for all K steps"),
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
                "boundary": "PERIODIC", "accumulation": acc_name(args.config, bool(flags & nat.FLAG_FMA)),
                "nonfinite": ("VW_FLAG_REF_NONFINITE: the batch facade's NaN/Inf spread reproduced (rows probed "
                              "in-line by the kernels, a fix-up launch per pass)" if ref_nf else
                              "not emulated in the timed calls (VW_FLAG_REF_NONFINITE off)"),
                "parallelism": f"batch-shard x{world} (contiguous row blocks, no collective)"
                               + (f", {K} contexts per GPU (own stream each, row blocks)" if K > 1 else "")
                               + (", consecutive steps pipelined over two contexts (step i+1's forward beside "
                                  "step i's inverse, one buffer set per step in flight)" if overlap else ""),
                "schedule": "overlap-steps" if overlap else ("contexts" if K > 1 else "sequential"),
                "contexts_per_gpu": K,
                "launch": ("vw_pipeline_run: the engine issues the K steps from C++ on two streams, event edges "
                           "between them (overlapped steps)"
                           if overlap else LAUNCH_DESC[args.launch]),
                "buffer_sets": {"sets": rot[0], "outputs_rotated": rot[1], "device_bytes_per_rank": footprint,
                                "why": "step i works on set i mod R: no step re-reads an input an earlier step left "
                                       "in the 256 MiB Infinity Cache"},
                "passes_ms": {f: round(v, 5) for f, v in kpass_ms.items()},
                "kernel_timing": ((f"HIP events around every kernel launch of {sampled} of the {args.steps} timed "
                                   "steps (event nodes inside the replayed graph)" if args.launch == "graph-k" else
                                   "HIP events around every launch (engine timer)" if args.launch == "direct"
                                   else "none") if events_timed else
                                  "none inside the timed region (overlapping launches): the kernels are timed by the "
                                  "one-context pass of roofline.duration_from" if events else "none"),
                "kernels": kernels if events_timed else kkernels if roof else {},
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
    # the first row of the first context's block and the last row of the last context's block
    picks = [(wl.parts[0], 0), (wl.parts[-1], wl.parts[-1].rows - 1)]
    worst = 0.0
    tol = 0.0
    for pt, r in picks:
        xr = pt.x[r].double().cpu().numpy()
        if wl.f32:
            tol = 1e-5 * float(abs(xr).max()) * J
        elif fma:
            tol = 1e-12
        if pipeline == "fwd+inv":
            d, a = O.decompose(xr, lo, hi, O.PERIODIC, J, core=False)
            y_ref = O.reconstruct(d, a, rl, rh, O.PERIODIC, w.wavelet_id)
            got = [(pt.det[:, r, :], d), (pt.app[r], a), (pt.y[r], y_ref)]
        else:
            y_ref, t_ref = O.swt_denoise(xr, lo, hi, O.PERIODIC, J, -1.0, True, w.wavelet_id)
            got = [(pt.y[r], y_ref)]
        for g, ref in got:
            e = float(abs(g.double().cpu().numpy() - ref).max())
            worst = max(worst, e)
    rows = [0, wl.rows - 1]
    pr = None
    if pipeline == "fwd+inv":
        pr = max(float((pt.y.double() - pt.x.double()).abs().max().item()) for pt in wl.parts)
    pr_bar = 1e-3 if wl.f32 else 1e-8   # truncated published taps (db8 J=10: ~1e-9; SURVEY.md key fact 5)
    ok = worst <= tol and (pr is None or pr < pr_bar)
    res = {"rows": rows, "max_abs_vs_oracle": worst, "tol": tol, "pr_max_abs": pr, "pr_bar": pr_bar, "ok": ok}
    if not ok:
        if os.environ.get("VW_BENCH_UNGUARDED") != "1":
            raise RuntimeError(f"bench correctness guard failed: {res}")
        # timing-only experiments (variant builds that skip work by design, tools/ab.sh): the line is printed
        # with ok false and marked, never as a result
        res["unguarded_experiment"] = True
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
