"""CPU rehearsal of bench.py's multi-rank table flow (test infrastructure only).

bench.py runs its table path through a backend object (bench.HipBackend: libairice.so's kernels on
the process's GPU).  CpuRehearsalBackend stands in for it on a CPU rank: the slab a rank builds is
the oracle's table rows for the same grid rows, events are wall clocks, and host copies are tensor
copies.  Everything else -- the TxH-row sharding, the barriers and max-over-ranks timing, the
per-column gathers (gloo here, RCCL on the GPU node), the node-shared host table and its fallback,
the single-GPU bitwise check and the JSON line -- is bench.py's own code.  Used by
tests/test_distributed.py to drive bench.main() at world size 8 without GPUs."""
import os
import time

import torch

import oracle
from tests.conftest import ATMOSPHERE_GZ


class _WallEvent:
    def __init__(self):
        self.t = None

    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other) -> float:
        return (other.t - self.t) * 1e3


class CpuRehearsalBackend:
    is_gpu = False

    def __init__(self, local_rank: int):
        self.dev = torch.device("cpu")
        self.stream = None
        self.solver = None
        self.m = oracle.load_atmosphere(ATMOSPHERE_GZ)
        self.builds = 0

    def event(self):
        return _WallEvent()

    def sync(self) -> None:
        pass

    def release(self) -> None:
        pass

    def table(self, grid, out, row_begin: int = 0, row_count=None, ld=None) -> None:
        og = oracle.grid_init(grid.depth_m * 100, grid.ice_m * 100, grid.height_step,
                              grid.start_angle, grid.stop_angle, grid.angle_step)
        if row_count is None:
            row_count = int(grid.table_rows)
        t = oracle.table_rows(self.m, og, row_begin, row_begin + row_count, nthreads=1)
        out[:, :t.shape[1]] = torch.from_numpy(t)
        self.builds += 1

    def table_to_host(self, slab, cnt: int, host, first: int) -> None:
        host[:, first:first + cnt].copy_(slab[:, :cnt])

    def host_register(self, ptr: int, nbytes: int) -> None:
        pass

    def host_unregister(self, ptr: int) -> None:
        pass


def rank_main(rank: int, world: int, port: int, argv, json_path: str) -> None:
    """One rank of a bench.py run (torch.distributed.run's environment, gloo)."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      AIRICE_DIST_BACKEND="gloo")
    import bench
    bench.main(argv, make_backend=CpuRehearsalBackend, json_path=json_path)
