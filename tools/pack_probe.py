"""Debug probe (GPU box): airice_lookup_pack timing (host wall clock and HIP events) on the cfg2
table."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from airiceraytracing_amd import AirIceSolver, _lib, make_grid
    from airiceraytracing_amd.solver import _stream_handle
    s = AirIceSolver()
    g = make_grid(-20000.0, 300000.0, 20.0, 92.0, 180.0, 0.5)
    t = torch.empty((11, g.n_rays), dtype=torch.float32, device="cuda:0")
    s.table_device(g, t)
    lt = s.lookup_table(t, g)
    s.lookup_pack(lt)
    torch.cuda.synchronize()
    for st in (None, torch.cuda.Stream()):
        h = _stream_handle(st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st if st is not None else torch.cuda.current_stream())
        w0 = time.perf_counter()
        for _ in range(10):
            _lib.check(_lib.lib().airice_lookup_pack(ctypes.byref(lt), _lib.ptr(lt._packed), h), "pack")
        w1 = time.perf_counter()
        e1.record(st if st is not None else torch.cuda.current_stream())
        torch.cuda.synchronize()
        w2 = time.perf_counter()
        print(f"stream={st}: host enqueue {(w1 - w0) / 10 * 1e6:.1f} us/call, wall {(w2 - w0) / 10 * 1e6:.1f} us/call, events {e0.elapsed_time(e1) / 10 * 1e3:.1f} us/call")


if __name__ == "__main__":
    main()
