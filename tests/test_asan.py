"""Sanitizer build: the host code of libairice.so -- GDAS parse, grid
set-up, the namespace readers, the host table lookup (column and packed-record paths) -- and
the oracle, built with -fsanitize=address,undefined -fno-sanitize-recover=all
(tests/cpp/asan_harness.cpp, `make -C airiceraytracing_amd/csrc asan`) and run on the real
atmosphere, hostile atmosphere texts, edge grid arguments and edge lookups (NaN, H <= 0, heights
outside the table, D = 0, D beyond every THD).  Any ASan/UBSan report aborts the harness."""
import gzip
import json
import os
import struct
import subprocess

import numpy as np

import oracle
from tests.conftest import ATMOSPHERE_GZ, ROOT

HARNESS = os.path.join(ROOT, "tests", "cpp", "asan_harness")


def test_host_code_and_oracle_run_clean_under_asan_ubsan(tmp_path):
    # incremental: rebuilds the harness when a source or header it compiles has changed
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "airiceraytracing_amd", "csrc"),
                    "asan"], check=True)
    text = gzip.decompress(open(ATMOSPHERE_GZ, "rb").read())
    (tmp_path / "Atmosphere.dat").write_bytes(text)
    m = oracle.parse_atmosphere(text)
    # an antenna table of the cfg2 kind on a coarse grid (200 m x 1 deg), from the oracle
    g = oracle.grid_init(-20000.0, 300000.0, 200.0, 92.0, 180.0, 1.0)
    t = oracle.table_rows(m, g, 0, g.height_steps)
    with open(tmp_path / "table.bin", "wb") as f:
        f.write(struct.pack("<qddii", t.shape[1], g.stop_height, g.height_step, g.height_steps,
                            g.angle_steps))
        f.write(np.ascontiguousarray(t, dtype=np.float32).tobytes())
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    out = subprocess.run([HARNESS, str(tmp_path / "Atmosphere.dat"), str(tmp_path / "table.bin")],
                         capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-4000:]
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr, out.stderr
    r = json.loads(out.stdout)
    assert r["real"] == [0, 0, m.max_layers]          # library, oracle, namespace reader
    n_hostile, lib_ok, oracle_ok = r["hostile"]
    assert n_hostile > 200 and 0 < lib_ok < n_hostile and lib_ok == oracle_ok
    # grid: the default, then zero / negative / NaN / too-fine steps and reversed angles rejected,
    # Tx rows <= 0 skipped, an empty grid rejected
    grid = r["grid"]
    assert grid[0] == [0, 9701, 900, 9701]
    assert [x[0] for x in grid[1:7]] == [-1] * 6
    assert grid[7][0] == 0 and grid[7][3] < grid[7][1]
    assert grid[8][0] == -1
    lk = r["lookup"]
    assert lk["checked"] > 2500 and lk["col_vs_packed_mismatch"] == 0
    assert lk["vs_oracle_mismatch"] == 0
    # table files: the round trip is exact, another medium and every damaged copy are refused
    same, other_refused, n_bad, n_rejected = r["table_file"]
    assert same == 1 and other_refused == 1 and n_bad == n_rejected == 12
    assert r["oracle_paths"] == 1
