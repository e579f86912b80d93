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
    """slab: (cols, per_items) padded local block.  Returns (cols, sum(counts)) on root.

    One gather per column, each rank's column segment received straight into its place in the
    root's single (cols, world x per_items) buffer: the root holds the table once (plus at most
    one slab of padding), never a list of world slabs to concatenate.  shard_rows fills the ranks
    in order, so the gathered segments are the table's prefix."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    cols = slab.shape[0]
    assert slab.shape[1] == per_items and slab.is_contiguous()
    total = sum(counts)
    k = 0
    while k < world and counts[k] == per_items:
        k += 1
    assert k == world or (counts[k] <= per_items and not any(counts[k + 1:])), \
        "slabs must fill the ranks in order (shard_rows)"
    if rank == root:
        buf = torch.empty((cols, world * per_items), dtype=slab.dtype, device=slab.device)
        for c in range(cols):
            dist.gather(slab[c], gather_list=[buf[c, r * per_items:(r + 1) * per_items]
                                              for r in range(world)], dst=root, group=group)
        return buf[:, :total]
    for c in range(cols):
        dist.gather(slab[c], dst=root, group=group)
    return None


class SharedHostTable:
    """A (cols, n) float32 table in host memory that every rank on the node maps (a file under
    /dev/shm): the destination of the per-rank D2H copies that assemble a sharded table in host
    memory, where the reference keeps it (AllTableAllAntData, MultiRayAirIceRefraction.cc:2101-2136),
    without routing the slabs through the root's HBM.  The creator reserves the
    pages up front (posix_fallocate: a full /dev/shm fails here, not as a SIGBUS mid-copy) and
    unlinks the file once every rank has mapped it, so it disappears with the last process."""

    def __init__(self, path: str, cols: int, n: int, create: bool):
        import mmap
        import os
        self.cols, self.n, self.path = cols, n, path
        nbytes = cols * n * 4
        if create:
            fd = os.open(path, os.O_CREAT | os.O_RDWR | os.O_TRUNC, 0o600)
            try:
                os.posix_fallocate(fd, 0, max(nbytes, 1))
            except OSError:
                os.close(fd)
                os.unlink(path)
                raise
        else:
            fd = os.open(path, os.O_RDWR)
        try:
            self._mm = mmap.mmap(fd, max(nbytes, 1))
        finally:
            os.close(fd)
        self.tensor = torch.frombuffer(self._mm, dtype=torch.float32, count=cols * n).view(cols, n)
        self._registered = []

    def register_columns(self, first: int, count: int, register) -> None:
        """Page-lock the part of every column this rank writes ([first, first+count)) with
        ``register(ptr, nbytes)`` (airice_host_register): DMA targets for its D2H copies."""
        base = self.tensor.data_ptr()
        page = 4096
        spans = []
        for c in range(self.cols):
            a = base + (c * self.n + first) * 4
            b = a + count * 4
            a0, b0 = a & ~(page - 1), (b + page - 1) & ~(page - 1)
            if spans and a0 <= spans[-1][1]:
                spans[-1] = (spans[-1][0], max(spans[-1][1], b0))
            else:
                spans.append((a0, b0))
        for a0, b0 in spans:
            if b0 > a0:
                register(a0, b0 - a0)
                self._registered.append(a0)

    def unregister(self, unregister) -> None:
        for a0 in self._registered:
            unregister(a0)
        self._registered = []

    def close(self) -> None:
        self.tensor = None
        try:
            self._mm.close()
        except BufferError:  # a view is still alive: the mapping goes with the process
            pass


def assemble_to_host(slab: torch.Tensor, count_items: int, first_item: int, host: torch.Tensor,
                     copy=None) -> None:
    """This rank's part of the host-assembled table: host[:, first:first+count] = slab[:, :count].
    ``copy(slab, count, host, first)`` performs it (the GPU path: airice_table_to_host, one D2H
    copy per column into this rank's page-locked rows); default: a torch copy (CPU ranks)."""
    if count_items == 0:
        return
    if copy is not None:
        copy(slab, count_items, host, first_item)
    else:
        host[:, first_item:first_item + count_items].copy_(slab[:, :count_items])


def _try(make):
    """(make(), None), or (None, the error's text) when it raises: any exception (a RuntimeError
    from torch.from_file as well as an OSError), so that every failure reaches the agreement
    all-reduce (_all_ok) instead of leaving the other ranks waiting in it."""
    try:
        return make(), None
    except Exception as e:  # noqa: BLE001 -- reported to every rank, never swallowed
        return None, f"{type(e).__name__}: {e}"


def _all_ok(ok: bool, group=None, device=None) -> bool:
    """True on every rank iff ``ok`` is true on every rank (one all-reduce)."""
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


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
                      group=None, assemble: str = "rccl", host_path: str | None = None,
                      host_copy=None, host_register=None, host_unregister=None) -> dict:
    """The north_star's multi-GPU table: rank r builds its contiguous slab of TxH rows
    (shard_rows; the TxH-descending / angle-ascending order the lookup expects,
    MultiRayAirIceRefraction.cc:1035-1039) ``steps`` times between barriers, then the slabs
    are assembled, timed in their own barrier bracket ``gather_reps`` times:

    * ``assemble="rccl"``: on ``root``'s device by one gather per column (RCCL over xGMI for
      backend "nccl"; gather_slabs), the root holding the table once;
    * ``assemble="host"``: in host memory, where the reference keeps the table (its row loop
      appends to AllTableAllAntData, .cc:2079-2136): every rank copies its slab into its rows of a
      SharedHostTable at ``host_path`` (``host_copy``: the GPU path's strided D2H copy per
      column, airice_table_to_host, into page-locked pages, ``host_register``), all ranks' copies
      in parallel over their own PCIe links; no collective moves table data.

    ``compute(row_begin, row_count, slab)`` fills the slab (stride = rows_per_rank x
    angle_steps); ``sync`` waits for the device (torch.cuda.synchronize on a GPU).  Returns the
    per-rank timings reduced by max over ranks and, on root, the assembled (cols, n_rays) table."""
    import time
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sync = sync or (lambda: None)
    coll_device = coll_device if coll_device is not None else device
    asteps = int(grid.angle_steps)
    n_rays = int(grid.table_rows) * asteps
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
    assembled = None
    gather_s = []
    host = None
    host_error = None
    if assemble == "host":
        if host_path is None:
            raise ValueError("assemble='host' needs host_path")
        # the root creates the shared table, then the others map it; a failure on any rank (a full
        # /dev/shm, permissions) is agreed on by every rank, which then all take the RCCL gather,
        # instead of the failing rank raising while the others wait in a barrier
        if rank == root:
            host, host_error = _try(lambda: SharedHostTable(host_path, cols, n_rays, create=True))
        if not _all_ok(host_error is None, group, coll_device):
            host_error = host_error or "the root could not create the shared host table"
        else:
            if rank != root:
                host, host_error = _try(
                    lambda: SharedHostTable(host_path, cols, n_rays, create=False))
            if not _all_ok(host_error is None, group, coll_device):
                host_error = host_error or "a rank could not map the shared host table"
        if rank == root and host is not None:
            import os
            os.unlink(host_path)  # every rank has it mapped (or failed); it goes with the last process
        if host_error is not None:
            if host is not None:
                host.close()
                host = None
            assemble = "rccl"
    if assemble == "host":
        if host_register is not None and count:
            host.register_columns(begin * asteps, count * asteps, host_register)
        for _ in range(max(1, gather_reps)):
            sync()
            dist.barrier(group)
            g0 = time.perf_counter()
            assemble_to_host(slab, count * asteps, begin * asteps, host.tensor, host_copy)
            sync()
            gather_s.append(time.perf_counter() - g0)
        dist.barrier(group)  # every rank's rows are in place before the root reads the table
        if rank == root:
            assembled = host.tensor
        moved = n_rays * cols * slab.element_size()
    elif assemble == "rccl":
        send = slab if coll_device is None or slab.device == torch.device(coll_device) \
            else slab.to(coll_device)
        for _ in range(max(1, gather_reps)):
            sync()
            dist.barrier(group)
            g0 = time.perf_counter()
            assembled = gather_slabs(send, per * asteps, counts, root, group)
            sync()
            gather_s.append(time.perf_counter() - g0)
        moved = sum(counts[r] for r in range(world) if r != root) * cols * slab.element_size()
    else:
        raise ValueError(f"unknown assemble mode {assemble!r}")
    red = torch.tensor([elapsed, min(gather_s)], dtype=torch.float64, device=coll_device)
    dist.all_reduce(red, op=dist.ReduceOp.MAX, group=group)
    return {"elapsed_s": float(red[0]), "gather_s": float(red[1]), "row_begin": begin,
            "row_count": count, "rows_per_rank": per, "rays_this_rank": count * asteps,
            "bytes_to_root": moved if assemble == "rccl" else 0,
            "bytes_assembled": moved, "assemble": assemble, "host_assembly_error": host_error,
            "slab": slab, "assembled": assembled, "host": host,
            "host_unregister": host_unregister}
