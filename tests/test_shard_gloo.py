"""Multi-process batch sharding on CPU (gloo, world size 2): the N>1 path of bench.py.

Each rank transforms its shard_rows() block of a global batch (the oracle stands in for the device:
this tests the host-side partitioning), the per-rank results are gathered, and they must equal the
single-process transform of the whole batch bit for bit -- no row lost, duplicated or reordered, and
the per-rank generator offsets reproduce the global input.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from vectorwave_amd.shard import gather_order, shard_rows

N, J = 64, 3


def test_shard_rows_partition():
    for total in (0, 1, 7, 4096, 4097):
        for world in (1, 2, 3, 8):
            blocks = gather_order(total, world)
            assert sum(c for _, c in blocks) == total
            pos = 0
            for s, c in blocks:
                assert s == pos
                pos += c
            counts = [c for _, c in blocks]
            assert max(counts) - min(counts) <= 1
    with pytest.raises(ValueError):
        shard_rows(10, 2, 2)


def _transform_rows(x):
    from oracle import oracle as O
    from vectorwave_amd import get_wavelet

    w = get_wavelet("db4")
    lo, hi = w.lowPassDecomposition(), w.highPassDecomposition()
    out = []
    for row in x:
        det, app = O.decompose(row, lo, hi, O.PERIODIC, J)
        y = O.reconstruct(det, app, lo, hi, O.PERIODIC, w.wavelet_id)
        out.append(np.concatenate([det.reshape(-1), app, y]))
    return np.stack(out) if out else np.zeros((0, (J + 2) * N))


def _worker(rank, world, port, total, out_path):
    import torch
    import torch.distributed as dist
    from oracle import oracle as O

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    start, count = shard_rows(total, world, rank)
    # the same counter-based input the device generator produces for these global rows
    x = O.fill_uniform(count * N, 42, offset=start * N).reshape(count, N)
    local = torch.from_numpy(_transform_rows(x).reshape(-1).copy())
    parts = [None] * world
    dist.all_gather_object(parts, local)
    if rank == 0:
        np.save(out_path, torch.cat(parts).numpy())
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("total", [6, 7])
def test_gloo_world2_matches_single_process(tmp_path, total):
    from oracle import oracle as O

    world = 2
    out = str(tmp_path / "gathered.npy")
    mp.spawn(_worker, args=(world, _free_port(), total, out), nprocs=world, join=True)
    got = np.load(out)
    xg = O.fill_uniform(total * N, 42).reshape(total, N)
    np.testing.assert_array_equal(got, _transform_rows(xg).reshape(-1))
    parts = [O.fill_uniform(c * N, 42, offset=s * N).reshape(c, N) for s, c in gather_order(total, world)]
    np.testing.assert_array_equal(np.concatenate(parts), xg)
