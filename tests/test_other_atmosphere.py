"""A second GDAS atmosphere (arbitrary Atmosphere.dat files, AirIceRayTracing.cc:860).

The shipped file is transformed deterministically into another valid GDAS-format file: interior
layer bounds moved, the fit's C row scaled, and the refractivity n-1 of every (height, n) point
scaled (a "wetter" profile).  The library's host parse must equal the oracle's parse of the same
text (CPU), and the GPU table and minimizer must match the oracle on it (-m gpu).  Parity vs the
reference itself is unpinned for this file (no recorded reference output exists for it)."""
import os

import numpy as np
import pytest

import oracle
from tests import parity

NTHREADS = min(16, os.cpu_count() or 1)


def synthetic_gdas(text: bytes) -> bytes:
    lines = text.decode().splitlines()
    out = [lines[0]]
    atm = [float(v) for v in lines[1].split()]
    # interior layer bounds (cm): 3.2 km -> 3.5 km, 8.4 km -> 9.0 km (the top bound stays at the
    # profile's last height: GDAS files end their (h, n) data there, .cc:73-147)
    atm[1], atm[2] = 3.5e5, 9.0e5
    out.append(" " + "  ".join(f"{v:.8E}" for v in atm))
    out.append(lines[2])
    out.append(lines[3])
    c = [float(v) for v in lines[4].split()]
    c = [v * 0.97 for v in c[:4]] + [c[4]]
    out.append(" " + "  ".join(f"{v:.8E}" for v in c))
    out.append(lines[5])
    for ln in lines[6:]:
        parts = ln.split()
        if len(parts) != 2:
            out.append(ln)
            continue
        h, n = float(parts[0]), float(parts[1])
        out.append(f"{h: .8E} {1 + (n - 1) * 1.06: .8E}")
    return ("\n".join(out) + "\n").encode()


@pytest.fixture(scope="module")
def synth(atmosphere_text, tmp_path_factory):
    text = synthetic_gdas(atmosphere_text)
    path = tmp_path_factory.mktemp("atm") / "Atmosphere.dat"
    path.write_bytes(text)
    return text, str(path)


def test_synthetic_file_differs(atmosphere_text, synth):
    a = oracle.parse_atmosphere(atmosphere_text)
    b = oracle.parse_atmosphere(synth[0])
    assert list(a.atmlay) != list(b.atmlay)
    assert a.N0 != b.N0
    assert list(a.C_air) != list(b.C_air)


def test_host_parse_matches_oracle(synth):
    from airiceraytracing_amd import _lib
    text, path = synth
    m = _lib.load_medium(path)
    o = oracle.parse_atmosphere(text)
    assert list(m.atmlay_cm) == list(o.atmlay)
    assert m.N0 == o.N0
    assert list(m.B_air) == list(o.B_air)
    assert list(m.C_air) == list(o.C_air)
    assert m.max_layers == o.max_layers


@pytest.mark.gpu
def test_gpu_table_and_solves(synth):
    from airiceraytracing_amd import AirIceSolver, make_grid
    text, path = synth
    s = AirIceSolver(atmosphere=path)
    om = oracle.parse_atmosphere(text)
    g = make_grid(-20000.0, 300000.0, 40.0, 92.0, 180.0, 0.5)
    og = oracle.grid_init(-20000.0, 300000.0, 40.0, 92.0, 180.0, 0.5)
    table, full = s.table_host(g, full=True)
    ot, of = oracle.table_rows(om, og, 0, og.height_steps, full=True, nthreads=NTHREADS)
    rep = parity.compare_columns(full, of, parity.RAY_FLOORS)
    assert rep["ok"], rep
    assert parity.float_ulp_diff(table, ot) <= 1
    txh, dist, depth = parity.cfg3_queries(5000, seed=8)
    out, st = s.solve_host(txh, dist, depth, 3000.0)
    ref, rst = oracle.solve_batch(om, txh, dist, depth, 3000.0)
    mask = (rst & oracle.SOLVE_UNPINNED) == 0
    assert np.array_equal(st.astype(np.int64)[mask], rst[mask].astype(np.int64))
    rep = parity.compare_columns(out, ref, parity.SOLVE_FLOORS, mask=mask)
    assert rep["ok"], rep
