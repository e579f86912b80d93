"""BASELINE cfg4: the fine table (TxH 100000 -> 3000 m @ 1 m x launch angle 90.1 -> 180 deg @
0.01 deg, antenna 200 m below the ice: 97,001 x 8,991 = 872,135,991 rays, 38.4 GB of float
columns) built on the GPU(s), timed, spot-checked against the CPU oracle.

    python tools/fine_table.py [--to-host]                         # one GPU: the whole table
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        tools/fine_table.py [--to-host]                            # N GPUs: row slabs + gather

With N ranks every rank builds its contiguous slab of TxH rows; one RCCL gather assembles the
table on rank 0 (airiceraytracing_amd.distributed.table_sharded), and --to-host copies it into
pinned host memory (AllTableAllAntData lives in host memory).  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CFG4 = dict(depth_cm=-20000.0, ice_cm=300000.0, height_step=1.0, start_angle=90.1,
            stop_angle=180.0, angle_step=0.01)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--to-host", action="store_true")
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--check-rows", type=int, default=12)
    a = p.parse_args()
    import torch
    import torch.distributed as dist
    from airiceraytracing_amd import AirIceSolver, make_grid
    from airiceraytracing_amd.distributed import gpu_table_compute, shard_rows, table_sharded

    distributed = "RANK" in os.environ
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dev = torch.device(f"cuda:{int(os.environ.get('LOCAL_RANK', '0'))}")
    torch.cuda.set_device(dev)
    if distributed:
        dist.init_process_group(backend="nccl", device_id=dev)
    s = AirIceSolver()
    g = make_grid(CFG4["depth_cm"], CFG4["ice_cm"], CFG4["height_step"], CFG4["start_angle"],
                  CFG4["stop_angle"], CFG4["angle_step"])
    n = g.n_rays
    asteps = g.angle_steps
    begin, count, per = shard_rows(g.height_steps, world, rank)
    slab = torch.empty((11, per * asteps), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream()

    def build():
        s.table_device(g, slab, None, row_begin=begin, row_count=count, ld=per * asteps,
                       stream=stream)

    build()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if distributed:
        dist.barrier()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(a.reps):
        build()
    e1.record(stream)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    wall = (time.perf_counter() - t0) / a.reps
    kms = e0.elapsed_time(e1) / a.reps
    w = torch.tensor([wall], dtype=torch.float64, device=dev)
    if distributed:
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
    wall = float(w.item())
    res = {"metric": "cfg4 fine table rays/s", "rays": n, "rows": g.height_steps,
           "angles": asteps, "n_gpus": world, "build_ms_max_over_ranks": wall * 1e3,
           "kernel_ms_rank0": kms, "value": n / wall, "unit": "rays/s",
           "table_bytes": 44 * n}
    # gather to rank 0 (RCCL) and optionally to pinned host memory
    full = slab
    if distributed:
        del slab
        torch.cuda.empty_cache()
        t1 = time.perf_counter()
        full = table_sharded(g, gpu_table_compute(s, g, stream), device=dev)
        torch.cuda.synchronize()
        dist.barrier()
        res["build_and_gather_s"] = time.perf_counter() - t1
    if rank == 0:
        if a.to_host:
            host = torch.empty(full.shape, dtype=torch.float32, pin_memory=True)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            host.copy_(full, non_blocking=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t2
            res["d2h_s"] = dt
            res["d2h_GBps"] = full.numel() * 4 / dt / 1e9
            del host
        # spot check: evenly spaced rows (the first and last included) against the oracle
        import oracle
        om = oracle.load_atmosphere(os.path.join(ROOT, "airiceraytracing_amd", "data",
                                                 "Atmosphere.dat.gz"))
        og = oracle.grid_init(CFG4["depth_cm"], CFG4["ice_cm"], CFG4["height_step"],
                              CFG4["start_angle"], CFG4["stop_angle"], CFG4["angle_step"])
        rows = np.unique(np.linspace(0, g.height_steps - 1, a.check_rows).astype(int))
        worst = 0
        nan_ok = True
        from tests import parity
        ld = full.shape[1]
        for r in rows:
            got = full[:, r * asteps:(r + 1) * asteps].cpu().numpy()
            ref = oracle.table_rows(om, og, int(r), int(r) + 1, nthreads=16)
            worst = max(worst, parity.float_ulp_diff(got, ref))
            nan_ok &= bool(np.array_equal(np.isnan(got), np.isnan(ref)))
        res["check"] = {"rows": rows.tolist(), "max_float_ulps": int(worst),
                        "nan_pattern_equal": nan_ok, "ld": ld}
        print(json.dumps(res), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
