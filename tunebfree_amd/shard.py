"""Instance sharding across ranks (one process per GPU).

The hot path partitions: every organ instance is independent, so
N GPUs render disjoint contiguous instance ranges with no data-path collective.
bench.py uses a fixed per-GPU batch (weak scaling): n_total = batch * world.
"""


def shard(n_total: int, rank: int, world: int):
    """(first, count) of the contiguous instance range owned by `rank`."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, rem = divmod(int(n_total), world)
    first = rank * base + min(rank, rem)
    return first, base + (1 if rank < rem else 0)
