"""Row sharding of a signal batch across GPUs (one process per GPU).

MODWT/SWT signals are independent, so a batch splits into contiguous row blocks with
no exchange on the data path: rank r of `world` transforms rows [start, start + count) of the global
batch on its own device.  Used by bench.py (strong scaling, the headline: the GLOBAL batch split into
contiguous blocks; its weak-scaling line gives every rank a full batch) and by DeviceGroup, whose C
entry points (vw_modwt_forward_multi_f64) split the same way in one process.
"""


def shard_rows(total, world, rank):
    """(start, count) of rank's contiguous block; the first total % world ranks get one extra row."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    if total < 0:
        raise ValueError("negative batch")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def gather_order(total, world):
    """Row blocks of every rank, in rank order (their concatenation is the global batch)."""
    return [shard_rows(total, world, r) for r in range(world)]
