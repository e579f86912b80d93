"""Wave-level executions of the grouped root finder's blocks (debug, GPU box): how many times a
wave of roots_sorted_kernel runs its loop, the lean (evaluation-free) bisection run, an evaluation
and each phase's update -- the instruction streams the VALU issue counts (pmc_summary.json) are
made of.

    tools/build_variant.sh airiceraytracing_amd/csrc /tmp/stats.so -DAIRICE_SORTED_STATS=1
    AIRICE_GROUP_MIN=1 AB_LIB=/tmp/stats.so python tools/solve_blocks.py [n]

(AIRICE_GROUP_MIN=1: the batch-wide grouping, since round 4 the default of the trace source only.)
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NAMES = ["loop_trip", "bisect_top", "lean_run", "lean_inner_trip", "evaluation", "upd_probe",
         "upd_flo", "upd_fhi", "upd_est", "upd_guard", "upd_bisect", "x_est", "lanes", "lean_closed"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
    import torch
    from airiceraytracing_amd import _lib
    _lib.LIB_PATH = os.path.abspath(os.environ["AB_LIB"])
    from airiceraytracing_amd import AirIceSolver
    from tests.parity import cfg3_queries
    L = _lib.lib()
    fn = L.airice_debug_exec_counters
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 16)()
    s = AirIceSolver()
    dev = torch.device("cuda:0")
    txh, dst, dep = cfg3_queries(n, seed=12345)
    t = [torch.from_numpy(a).to(dev) for a in (txh, dst, dep)]
    out = torch.empty((17, n), dtype=torch.float64, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    s.solve_device(t[0], t[1], t[2], 3000.0, out, st)
    torch.cuda.synchronize()
    fn(buf, 16, 1)
    s.solve_device(t[0], t[1], t[2], 3000.0, out, st)
    torch.cuda.synchronize()
    fn(buf, 16, 1)
    waves = buf[12]
    res = {"queries": n, "waves": waves,
           "per_wave": {k: buf[i] / waves for i, k in enumerate(NAMES) if k != "lanes"}}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
