"""Round-robin partition of a block stream across ranks (one process per GPU).

Block g of the global stream belongs to rank g % world; a rank
holds its blocks in stream order, so local block i is global block
i * world + rank.  Blocks are independent, so there is no data-path
collective: ranks only meet at the timing barrier and the max-over-ranks
reduction of elapsed time (bench.py).
"""
from __future__ import annotations

from .corpus import Corpus, fillseq


def owner(g: int, world: int) -> int:
    return g % world


def global_index(i: int, rank: int, world: int) -> int:
    return i * world + rank


def local_count(total: int, rank: int, world: int) -> int:
    """Blocks rank holds when `total` blocks are dealt round-robin."""
    return total // world + (1 if rank < total % world else 0)


def fillseq_shard(per_rank: int, rank: int, world: int, block_size: int = 4096) -> Corpus:
    """This rank's `per_rank` blocks of one fillseq stream (weak scaling:
    the stream is per_rank * world blocks long)."""
    return fillseq(per_rank, block_size=block_size, stride=world, phase=rank)


def fillseq_total(total: int, rank: int, world: int, block_size: int = 4096) -> Corpus:
    """This rank's share of a `total`-block fillseq stream dealt round-robin
    (strong scaling: config C4 is total = 1 048 576 over 8 ranks)."""
    return fillseq(local_count(total, rank, world), block_size=block_size, stride=world,
                   phase=rank)


def interleave(per_rank: list, total: int):
    """Put per-rank arrays (local order, first axis = block) back in global
    stream order: global block g = local i of rank g % world, i = g // world."""
    import numpy as np
    world = len(per_rank)
    first = per_rank[0]
    out = np.empty((total,) + tuple(first.shape[1:]), dtype=first.dtype)
    for r, a in enumerate(per_rank):
        assert a.shape[0] == local_count(total, r, world)
        out[r::world] = a
    return out


def max_over_ranks(value: float, dist, device=None) -> float:
    """Max of a per-rank float (elapsed time) over all ranks; identity if
    torch.distributed is not initialised."""
    if dist is None or not dist.is_available() or not dist.is_initialized():
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)   # gloo: a CPU tensor
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
