"""bench.py's multi-GPU control path on CPU: `--gpus N` spawns N rank processes (RANK / LOCAL_RANK /
WORLD_SIZE set, no GPU touched by the parent), each owns its shard_rows() block of the GLOBAL batch
(strong scaling), and the timing collectives (barrier, max over ranks) run over gloo."""
import json
import os
import subprocess
import sys

import pytest

from vectorwave_amd.shard import gather_order

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=180, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # only rank 0 prints
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2, 3])
def test_launcher_starts_n_ranks_with_row_blocks(n):
    out = _run("--gpus", str(n), "--dry-run")
    assert out["n_gpus"] == n and out["global_batch"] == 4096
    blocks = sorted(out["blocks"])
    assert [b[0] for b in blocks] == list(range(n))
    assert [(b[1], b[2]) for b in blocks] == gather_order(4096, n)
    assert [str(b[3]) for b in blocks] == [str(r) for r in range(n)]  # LOCAL_RANK = rank on one node
    assert out["max_elapsed"] == pytest.approx(0.001 * n)  # max over ranks, not rank 0's


def test_launcher_uneven_batch():
    out = _run("--gpus", "2", "--dry-run", "--batch", "4097")
    assert sorted((b[1], b[2]) for b in out["blocks"]) == [(0, 2049), (2049, 2048)]


def test_no_collective_inside_timed_interval():
    """bench.measure() on fakes that log every call: between the start of the clock (perf_counter + the
    opening HIP event on the main stream) and its end (closing event + synchronize + perf_counter) only
    the fork to the contexts' streams, their graph replays and the join run -- the barriers of the
    contract lie outside."""
    import contextlib
    sys.path.insert(0, ROOT)
    import bench

    log = []

    class Ev:
        def __init__(self, **kw):
            pass

        def record(self, stream=None):
            log.append("event")

        def elapsed_time(self, other):
            return 1.0

    class Stream:
        def wait_event(self, e):
            log.append("wait")

    class FakeCuda:
        Event = Ev

        @staticmethod
        def synchronize():
            log.append("sync")

        @staticmethod
        def current_stream():
            return Stream()

        @staticmethod
        def stream(s):
            return contextlib.nullcontext()

    class FakeTorch:
        cuda = FakeCuda

    class FakeDist:
        @staticmethod
        def barrier():
            log.append("barrier")

    class G:
        def launch(self, n):
            log.append("replay")

        def close(self):
            pass

    class Eng:
        def capture(self, fn):
            fn()
            return G()

        def reset_timing(self):
            pass

        def enable_timing(self, on):
            pass

        def kernel_spans(self, f, ev):
            return []

    class Part:
        rotate = 2   # two buffer sets: the timed steps alternate, still one replay per context

        def __init__(self):
            self.eng, self.stream = Eng(), Stream()

        def step_fn(self, flags, only=None):
            return lambda i=0: log.append("step")

    class Wl:
        def __init__(self):
            self.parts = [Part(), Part()]
            self.graphs = []

    real = bench.time.perf_counter

    def pc():
        log.append("clock")
        return real()

    bench.time.perf_counter = pc
    try:
        (dev_s, host_s), _, _, _, _ = bench.measure(FakeTorch, FakeDist, 2, Wl(), 0, "graph-k", 4, 1, 0.0, False)
    finally:
        bench.time.perf_counter = real
    # the timed window: from the clock read followed by the opening event to the closing clock read
    i0 = max(i for i in range(len(log) - 1) if log[i] == "clock" and log[i + 1] == "event")
    i1 = max(i for i, v in enumerate(log) if v == "clock")
    window = log[i0:i1 + 1]
    assert "barrier" not in window, window
    assert window[:2] == ["clock", "event"] and window[-3:] == ["event", "sync", "clock"], window
    assert window.count("replay") == 2   # one K-step graph per context
    assert "barrier" in log[:i0] and "barrier" in log[i1:]   # contract barriers, both outside
    assert dev_s == pytest.approx(1e-3)


def test_schedule_policy_per_shape():
    # bench.plan_schedule (round 5): the 8-GPU shard of the headline (512 rows) pipelines consecutive steps,
    # the full 4096-row batch splits over 4 contexts, long signals keep sequential steps / 2 contexts; the
    # weak-scaling pass plans its own -- rows and N decide, not the strong-scaling shard
    import argparse
    import bench
    a = argparse.Namespace(contexts=0, rotate=0, rotate_outputs=False, overlap_steps=False)
    cus = 256
    K, ov, rot = bench.plan_schedule(a, 512, 4096, 8, cus, "fwd+inv")
    assert ov and K == 1 and rot[0] >= 2 and rot[1]
    K, ov, rot = bench.plan_schedule(a, 4096, 4096, 8, cus, "fwd+inv")
    assert not ov and K == 4 and rot[0] * 4096 * 4096 * 8 >= 512 << 20
    K, ov, _ = bench.plan_schedule(a, 256, 1 << 20, 8, cus, "fwd+inv")          # db8-stream
    assert not ov and K == 1
    K, ov, _ = bench.plan_schedule(a, 16384, 16384, 8, cus, "denoise")         # sym8-denoise
    assert not ov and K == 2
    K, ov, _ = bench.plan_schedule(a, 65536, 8192, 4, cus, "fwd+inv")          # coif5-f32
    assert not ov and K == 2
    K, ov, _ = bench.plan_schedule(a, 1024, 4096, 8, cus, "fwd+inv")
    assert not ov and K == 2
    a.contexts = 3
    K, ov, _ = bench.plan_schedule(a, 512, 4096, 8, cus, "fwd+inv")
    assert not ov and K == 3
