"""Multi-GPU sharding of the table grid and of minimizer query batches.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  Rays and queries
are independent, so the only communication is assembling the result:

* table: contiguous blocks of TxHeight rows per rank (the row-major TxH-descending /
  angle-ascending order the reference's lookup expects, MultiRayAirIceRefraction.cc:1035-1039),
  padded to an equal slab so one ``gather`` (RCCL) moves every slab to the root;
* queries: equal index ranges, gathered the same way.

``compute`` callables make the sharding logic testable without a GPU (tests/test_distributed.py
runs it with world_size 2 over gloo).
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist


def shard_rows(total_rows: int, world: int, rank: int) -> tuple[int, int, int]:
    """(row_begin, row_count, rows_per_rank): contiguous blocks, last rank may be short."""
    per = -(-total_rows // world)
    begin = min(rank * per, total_rows)
    count = max(0, min(per, total_rows - begin))
    return begin, count, per


def shard_range(n: int, world: int, rank: int) -> tuple[int, int, int]:
    return shard_rows(n, world, rank)


def gather_slabs(slab: torch.Tensor, per_items: int, counts: list[int], root: int = 0,
                 group=None) -> torch.Tensor | None:
    """slab: (cols, per_items) padded local block.  Returns (cols, sum(counts)) on root."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if rank == root:
        bufs = [torch.empty_like(slab) for _ in range(world)]
        dist.gather(slab, gather_list=bufs, dst=root, group=group)
        return torch.cat([b[:, :c] for b, c in zip(bufs, counts)], dim=1)
    dist.gather(slab, dst=root, group=group)
    return None


def table_sharded(grid, compute: Callable[[int, int, torch.Tensor], None], cols: int = 11,
                  dtype=torch.float32, device=None, root: int = 0, group=None):
    """Build the full grid across ranks.  compute(row_begin, row_count, out) fills
    out[:, :row_count*angle_steps].  Returns the assembled table on root, else None."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    asteps = int(grid.angle_steps)
    begin, count, per = shard_rows(int(grid.height_steps), world, rank)
    slab = torch.zeros((cols, per * asteps), dtype=dtype, device=device)
    if count:
        compute(begin, count, slab)
    counts = [shard_rows(int(grid.height_steps), world, r)[1] * asteps for r in range(world)]
    return gather_slabs(slab, per * asteps, counts, root, group)


def queries_sharded(n: int, compute: Callable[[int, int, torch.Tensor], None], cols: int,
                    dtype=torch.float64, device=None, root: int = 0, group=None):
    """compute(begin, count, out) fills out[:, :count] for queries [begin, begin+count)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    begin, count, per = shard_range(n, world, rank)
    slab = torch.zeros((cols, per), dtype=dtype, device=device)
    if count:
        compute(begin, count, slab)
    counts = [shard_range(n, world, r)[1] for r in range(world)]
    return gather_slabs(slab, per, counts, root, group)


def gpu_table_compute(solver, grid, stream=None):
    """compute() for table_sharded backed by the HIP table kernel (slab stride = per*angles)."""
    def compute(begin: int, count: int, out: torch.Tensor) -> None:
        solver.table_device(grid, out, None, row_begin=begin, row_count=count,
                            ld=out.shape[1], stream=stream)
    return compute
