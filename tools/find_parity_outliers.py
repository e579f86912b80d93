"""Diagnostic (GPU box): the cfg3 1e6 device batch against the oracle on every query; prints each
query whose outputs exceed the 1e-9 rule, with both sides' launch angle, status and the column
errors, so a difference can be traced to its bisection path (tools only)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from tests import parity  # noqa: E402


def main():
    import torch
    from airiceraytracing_amd import AirIceSolver
    s = AirIceSolver()
    om = oracle.load_atmosphere(os.path.join(ROOT, "airiceraytracing_amd", "data", "Atmosphere.dat.gz"))
    n = 1_000_000
    txh, dist, depth = parity.cfg3_queries(n)
    dev = torch.device("cuda:0")
    t = [torch.from_numpy(a).to(dev) for a in (txh, dist, depth)]
    out = torch.empty((17, n), dtype=torch.float64, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    s.solve_device(t[0], t[1], t[2], 3000.0, out, st)
    torch.cuda.synchronize()
    out, st = out.cpu().numpy(), st.cpu().numpy()
    ref, rst = oracle.solve_batch(om, txh, dist, depth, 3000.0, nthreads=16)
    mask = (rst & oracle.SOLVE_UNPINNED) == 0
    scale = np.maximum(np.abs(ref), parity.SOLVE_FLOORS[:, None])
    err = np.abs(out - ref) / scale
    err[:, ~mask] = 0
    err = np.nan_to_num(err)
    bad = np.flatnonzero((err > 1e-9).any(axis=0))
    print(f"pinned {mask.sum()} bad {bad.size}; max rel per col "
          + " ".join(f"{c}:{err[c].max():.2e}" for c in range(17)))
    for i in bad[:20]:
        print(f"q {i}: txh {txh[i]!r} dist {dist[i]!r} depth {depth[i]!r} st gpu {st[i]} ref {rst[i]}")
        print(f"   launch gpu {out[10, i]!r} ref {ref[10, i]!r} (rel {abs(out[10,i]-ref[10,i])/ref[10,i]:.2e})")
        print("   cols " + " ".join(f"{c}:{err[c, i]:.2e}" for c in range(17) if err[c, i] > 1e-11))
        print("   gpu " + " ".join(f"{v:.17g}" for v in out[:, i]))
        print("   ref " + " ".join(f"{v:.17g}" for v in ref[:, i]))
    # the launch-angle differences over the whole batch, in units of the GSL tolerance
    dl = np.abs(out[10] - ref[10]) / np.abs(ref[10])
    dl = dl[mask & np.isfinite(dl)]
    print("launch angle rel diff: zero", int((dl == 0).sum()), "of", dl.size, "; max", dl.max(),
          "; > 1e-12:", int((dl > 1e-12).sum()))


def trace():
    """The same for the cfg5 1e7 pythonwrapper batch (Py_TraceIceToAir rows)."""
    import torch
    from airiceraytracing_amd import AirIceSolver, VARIANT_PYWRAPPER
    s = AirIceSolver(variant=VARIANT_PYWRAPPER)
    om = oracle.load_atmosphere(os.path.join(ROOT, "airiceraytracing_amd", "data", "Atmosphere.dat.gz"),
                                pi=oracle.PI_EXACT)
    n = 10_000_000
    q = parity.cfg5_queries(n)
    dev = torch.device("cuda:0")
    t = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in q]
    out = torch.empty((n, 10), dtype=torch.float64, device=dev)
    s.trace_ice_to_air_device(*t, out)
    torch.cuda.synchronize()
    out = out.cpu().numpy()
    ref = oracle.py_trace_batch(om, *q, nthreads=16)
    scale = np.maximum(np.abs(ref), parity.TRACE_FLOORS[None, :])
    err = np.nan_to_num(np.abs(out - ref) / scale)
    bad = np.flatnonzero((err > 1e-9).any(axis=1))
    print(f"trace: bad {bad.size}; max rel per col "
          + " ".join(f"{c}:{err[:, c].max():.2e}" for c in range(10)))
    for i in bad[:20]:
        print(f"q {i}: depth {q[0][i]!r} ice {q[1][i]!r} txh {q[2][i]!r} dist {q[3][i]!r}")
        print("   cols " + " ".join(f"{c}:{err[i, c]:.2e}" for c in range(10) if err[i, c] > 1e-11))
        print("   gpu " + " ".join(f"{v:.17g}" for v in out[i]))
        print("   ref " + " ".join(f"{v:.17g}" for v in ref[i]))


if __name__ == "__main__":
    if sys.argv[1:] == ["trace"]:
        trace()
    else:
        main()
