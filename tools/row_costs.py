"""Per-ray cost of the table kernel by the number of air layers a row's rays cross (GPU box;
tools only): the cfg4 grid's rows (8,991 rays each) in blocks of 200 rows of one layer count,
each timed with HIP events over 20 launches.  Gives the cost model of the multi-GPU row
sharding (airiceraytracing_amd.distributed.row_cost_weights)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from airiceraytracing_amd import AirIceSolver, make_grid
    s = AirIceSolver()
    g = make_grid(-20000.0, 300000.0, 1.0, 90.1, 180.0, 0.01)
    dev = torch.device("cuda:0")
    rows = 200
    out = torch.empty((11, rows * g.angle_steps), dtype=torch.float32, device=dev)
    # first row of each layer class: Tx heights 100000 - row (m); layer bounds 23141.75, 8363.54,
    # 3217.48 m above the 3000 m ice
    starts = {4: 1000, 3: 80000, 2: 93000, 1: 96790}
    res = {}
    st = torch.cuda.current_stream()
    for segs, r0 in starts.items():
        n = min(rows, g.table_rows - r0)
        for _ in range(3):
            s.table_device(g, out, row_begin=r0, row_count=n, ld=out.shape[1], stream=st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(20):
            s.table_device(g, out, row_begin=r0, row_count=n, ld=out.shape[1], stream=st)
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        res[segs] = {"rows": n, "first_row_txh": 100000.0 - r0, "ms": ms,
                     "ps_per_ray": ms * 1e9 / (n * g.angle_steps)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
