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
    begin, count, per = shard_rows(int(grid.table_rows), world, rank)
    slab = torch.zeros((cols, per * asteps), dtype=dtype, device=device)
    if count:
        compute(begin, count, slab)
    counts = [shard_rows(int(grid.table_rows), world, r)[1] * asteps for r in range(world)]
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


def sharded_step_grid_step(base_step: float, world: int) -> float:
    """TxH step of the N-GPU weak-scaling table: the base grid refined N-fold in TxH, so each
    of the N contiguous row slabs holds about as many rows as the base grid."""
    return base_step / world


def run_sharded_table(grid, compute: Callable[[int, int, torch.Tensor], None], steps: int,
                      warmup: int, device=None, coll_device=None, sync: Callable[[], None] = None,
                      gather_reps: int = 3, cols: int = 11, dtype=torch.float32, root: int = 0,
                      group=None) -> dict:
    """The north_star's multi-GPU table: rank r builds its contiguous slab of TxH rows
    (shard_rows; the TxH-descending / angle-ascending order the lookup expects,
    MultiRayAirIceRefraction.cc:1035-1039) ``steps`` times between barriers, then the slabs
    are assembled on ``root`` by one gather (RCCL over xGMI for backend "nccl"), timed in its
    own barrier bracket ``gather_reps`` times.  The reference assembles one table the same way
    in its row loop (.cc:2079-2136).  ``compute(row_begin, row_count, slab)`` fills the slab
    (stride = rows_per_rank x angle_steps); ``sync`` waits for the device (torch.cuda.synchronize
    on a GPU).  Returns the per-rank timings reduced by max over ranks and, on root, the
    assembled (cols, n_rays) table."""
    import time
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sync = sync or (lambda: None)
    coll_device = coll_device if coll_device is not None else device
    asteps = int(grid.angle_steps)
    begin, count, per = shard_rows(int(grid.table_rows), world, rank)
    slab = torch.zeros((cols, per * asteps), dtype=dtype, device=device)

    def step():
        if count:
            compute(begin, count, slab)

    for _ in range(warmup):
        step()
    sync()
    dist.barrier(group)
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    elapsed = time.perf_counter() - t0
    dist.barrier(group)
    counts = [shard_rows(int(grid.table_rows), world, r)[1] * asteps for r in range(world)]
    send = slab if coll_device is None or slab.device == torch.device(coll_device) \
        else slab.to(coll_device)
    assembled = None
    gather_s = []
    for _ in range(max(1, gather_reps)):
        sync()
        dist.barrier(group)
        g0 = time.perf_counter()
        assembled = gather_slabs(send, per * asteps, counts, root, group)
        sync()
        gather_s.append(time.perf_counter() - g0)
    red = torch.tensor([elapsed, min(gather_s)], dtype=torch.float64, device=coll_device)
    dist.all_reduce(red, op=dist.ReduceOp.MAX, group=group)
    return {"elapsed_s": float(red[0]), "gather_s": float(red[1]), "row_begin": begin,
            "row_count": count, "rows_per_rank": per, "rays_this_rank": count * asteps,
            "bytes_to_root": sum(counts[r] for r in range(world) if r != root) * cols
            * slab.element_size(),
            "slab": slab, "assembled": assembled}
