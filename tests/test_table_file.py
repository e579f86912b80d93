"""Table persistence: airice_table_save / _file_read_info / _load through the
library's host code (no GPU).  The reference keeps AllTableAllAntData in memory only
(MultiRayAirIceRefraction.cc:2101-2136), so there is no reference file format to match: the
checks are an exact round trip of an oracle-built antenna table, the header's grid and medium,
and refusal of damaged files and of a table traced in another medium."""
import ctypes
import os

import numpy as np
import pytest

import oracle
from airiceraytracing_amd import _lib
from airiceraytracing_amd.solver import AirIceSolver, make_grid
from tests.conftest import ATMOSPHERE_GZ


@pytest.fixture(scope="module")
def solver(tmp_path_factory):
    import gzip
    d = tmp_path_factory.mktemp("atm")
    p = d / "Atmosphere.dat"
    p.write_bytes(gzip.decompress(open(ATMOSPHERE_GZ, "rb").read()))
    return AirIceSolver(str(p))


@pytest.fixture(scope="module")
def antenna(oracle_medium):
    # a coarse cfg2-kind antenna table (200 m x 1 deg) from the oracle
    g = make_grid(-20000.0, 300000.0, 200.0, 92.0, 180.0, 1.0)
    og = oracle.grid_init(-20000.0, 300000.0, 200.0, 92.0, 180.0, 1.0)
    t = np.ascontiguousarray(oracle.table_rows(oracle_medium, og, 0, og.height_steps),
                             dtype=np.float32)
    assert t.shape == (11, g.table_rows * g.angle_steps)
    return g, t


def test_round_trip_exact(solver, antenna, tmp_path):
    g, t = antenna
    path = tmp_path / "ant0.airtbl"
    solver.save_table(str(path), g, t)
    assert not os.path.exists(str(path) + ".part")
    assert os.path.getsize(path) == _lib.TABLE_FILE_HEADER + t.nbytes
    info = solver.table_file_info(str(path))
    assert info.n_rays == t.shape[1]
    assert info.checksum == _lib.lib().airice_table_checksum(_lib.ptr(t), t.shape[1], t.shape[1])
    g2, t2 = solver.load_table(str(path))
    assert t2.tobytes() == t.tobytes()  # NaN patterns included
    for f, _ in _lib.Grid._fields_:
        assert getattr(g2, f) == getattr(g, f), f
    for f, _ in _lib.Medium._fields_:
        if f != "reserved_":
            assert np.array_equal(np.asarray(getattr(info.medium, f)),
                                  np.asarray(getattr(solver.medium, f))), f


def test_strided_source_and_empty_table(solver, antenna, tmp_path):
    g, t = antenna
    n = t.shape[1]
    wide = np.full((11, n + 13), 7.0, dtype=np.float32)
    wide[:, :n] = t
    view = wide[:, :n]  # column stride n + 13
    solver.save_table(str(tmp_path / "v.airtbl"), g, view)
    _, back = solver.load_table(str(tmp_path / "v.airtbl"))
    assert back.tobytes() == t.tobytes()
    empty = np.empty((11, 0), dtype=np.float32)
    solver.save_table(str(tmp_path / "e.airtbl"), g, empty)
    _, back = solver.load_table(str(tmp_path / "e.airtbl"))
    assert back.shape == (11, 0)


def test_refuses_damaged_files_and_other_media(solver, antenna, tmp_path):
    g, t = antenna
    path = tmp_path / "a.airtbl"
    solver.save_table(str(path), g, t)
    img = path.read_bytes()
    bad = tmp_path / "bad.airtbl"
    cases = [img[:0], img[:100], img[:_lib.TABLE_FILE_HEADER], img[:-4], img + b"\0",
             b"NOTATABL" + img[8:]]
    flipped = bytearray(img)
    flipped[_lib.TABLE_FILE_HEADER + 4 * 1000 + 1] ^= 0x40
    cases.append(bytes(flipped))
    for c in cases:
        bad.write_bytes(c)
        with pytest.raises(_lib.AirIceLibraryError):
            solver.load_table(str(bad))
    # a table traced with the pythonwrapper's medium (exact pi) is refused unless asked not to check
    py = AirIceSolver(None, _lib.VARIANT_PYWRAPPER)
    with pytest.raises(_lib.AirIceLibraryError, match="another medium"):
        py.load_table(str(path))
    _, back = py.load_table(str(path), check_medium=False)
    assert back.tobytes() == t.tobytes()
    with pytest.raises(ValueError):
        solver.save_table(str(tmp_path / "x.airtbl"), g, t.astype(np.float64))
    with pytest.raises(_lib.AirIceLibraryError):
        solver.table_file_info(str(tmp_path / "missing.airtbl"))


def test_header_layout_is_fixed(solver, antenna, tmp_path):
    """The header is little-endian at fixed offsets (airice_host.cpp): magic, version 1, header
    bytes 512, 11 columns, n_rays at 32, checksum at 40, the medium from 48, the grid from 368."""
    g, t = antenna
    path = tmp_path / "h.airtbl"
    solver.save_table(str(path), g, t)
    h = path.read_bytes()[:512]
    assert h[:8] == b"AIRTBL01"
    assert np.frombuffer(h[8:20], "<u4").tolist() == [1, 512, 11]
    assert int(np.frombuffer(h[32:40], "<u8")[0]) == t.shape[1]
    assert np.frombuffer(h[48:88], "<f8").tolist() == list(solver.medium.atmlay_cm)
    assert float(np.frombuffer(h[368:376], "<f8")[0]) == g.start_height
    assert int(np.frombuffer(h[424:428], "<i4")[0]) == g.angle_steps
    assert int(np.frombuffer(h[452:456], "<i4")[0]) == g.table_rows
    assert h[456:] == bytes(56)
    assert ctypes.sizeof(_lib.TableFileInfo) >= 320 + 88 + 16
