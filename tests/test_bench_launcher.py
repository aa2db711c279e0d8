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
