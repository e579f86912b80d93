"""Accuracy of the device math primitives the ray kernels are built from
(airiceraytracing_amd/csrc/airice_device.hpp), run on the GPU over random and edge inputs
(tests/cpp/prims_gpu.hip) and checked on the host:

- fast_sqrt / sqrt_rsqrt: one v_rsq_f64 seed (24.2 bits, tools/rcp_rsq_accuracy.hip), one
  Goldschmidt step and one Newton correction -> within 1 ulp of numpy's correctly rounded sqrt;
  the reciprocal (a multiplicative factor of every segment's closed forms) within 16 ulp of
  1/sqrt in long double (10 measured over 2^-40..2^40);
- div_pos: v_rcp_f64 (24.4 bits), one Newton step, Markstein residual -> within 1 ulp of a / b;
- asin_fast: the degree-12 polynomial / half-angle form -> within 3 ulp of mpmath (sampled) and
  NaN exactly where asin() is NaN;
- log_ratio (log(a/b) with the lean table log): absolute error within 4 * 2^-53 of the exact
  log(a/b) for a/b in the kernels' range.
These bound the rewrites DESIGN.md §4 lists; end-to-end parity is tests/test_gpu_parity.py."""
import os
import subprocess

import numpy as np
import pytest

from tests.conftest import ROOT

EXE = os.path.join(ROOT, "tests", "cpp", "prims_gpu")


def _ulps(got, ref):
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    return np.abs(got - ref) / np.spacing(np.abs(ref))


def _inputs(n, seed=2024):
    rng = np.random.default_rng(seed)
    q = np.concatenate([rng.uniform(0, 4, n // 2), np.exp2(rng.uniform(-40, 40, n // 2))])
    q[:4] = [0.0, 1.0, 4.0, 0.25]
    a = rng.uniform(-2, 2, n)
    b = np.exp2(rng.uniform(-12, 12, n))
    # rare branches of div_pos / log_ratio: b or a/b outside 2^+-1000, zeros, infinities, NaN
    # (quotients stay finite: log_ratio takes log of the IEEE quotient)
    a[4:16] = [1.0, 1.0, 0.0, 1.0, 2.0**-1050, 2.0**1020, 1.0, -1.0, np.inf, np.nan, 1.0,
               2.0**-60]
    b[4:16] = [2.0**-1010, 2.0**1010, 1.0, 0.0, 1.0, 2.0**10, np.inf, 0.0, 1.0, 1.0, np.nan,
               2.0**-1074]
    x = np.concatenate([rng.uniform(-1, 1, n - 16),
                        [0.5, -0.5, np.nextafter(0.5, 0), np.nextafter(0.5, 1), 1.0, -1.0, 0.0,
                         -0.0, 1.0 + 2**-52, -1.5, np.nan, 0.74, 1e-300, 0.25, 0.999999, 0.7]])
    return q, a, b, x


@pytest.mark.gpu
def test_device_primitives(tmp_path):
    assert os.path.exists(EXE), "build with __graft_entry__.build()"
    n = 1 << 20
    q, a, b, x = _inputs(n)
    np.stack([q, a, b, x], axis=1).astype(np.float64).tofile(tmp_path / "in.bin")
    r = subprocess.run([EXE, str(tmp_path / "in.bin"), str(tmp_path / "out.bin"), str(n)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    o = np.fromfile(tmp_path / "out.bin", dtype=np.float64).reshape(n, 6)
    sq = np.sqrt(q)
    nz = q > 0
    assert np.array_equal(o[~nz, 0], sq[~nz]) and np.array_equal(o[~nz, 1], sq[~nz])
    assert _ulps(o[nz, 0], sq[nz]).max() <= 1.0
    assert _ulps(o[nz, 1], sq[nz]).max() <= 1.0
    rs = (np.longdouble(1) / np.sqrt(q[nz].astype(np.longdouble))).astype(np.float64)
    ur = _ulps(o[nz, 2], rs)
    assert ur.max() <= 16.0, (ur.max(), q[nz][np.argmax(ur)])
    with np.errstate(all="ignore"):
        q_ref = a / b
    fq = np.isfinite(q_ref) & (q_ref != 0)
    assert _ulps(o[fq, 3], q_ref[fq]).max() <= 1.0
    assert np.array_equal(o[~fq, 3], q_ref[~fq], equal_nan=True)
    ref_asin = np.arcsin(x)
    fin = np.isfinite(ref_asin)
    assert np.array_equal(np.isnan(o[:, 4]), np.isnan(ref_asin))
    z = fin & (ref_asin != 0)
    assert _ulps(o[z, 4], ref_asin[z]).max() <= 3.0
    assert np.array_equal(o[fin & (ref_asin == 0), 4], ref_asin[fin & (ref_asin == 0)])
    # log(a / b): log(a) - log(b) in long double (special values: -inf, +inf, NaN as the
    # IEEE log of the quotient)
    with np.errstate(all="ignore"):
        lr = (np.log(a.astype(np.longdouble)) - np.log(b.astype(np.longdouble))).astype(np.float64)
    fin = np.isfinite(lr)
    err = np.abs(o[fin, 5] - lr[fin]) / np.maximum(np.spacing(np.abs(lr[fin])), 2.0**-53)
    # absolute error of the degree-5 lean log (<= 2.9 x 2^-52, tests/test_tlog.py) plus the
    # quotient's rounding: 6 units of 2^-53 measured (degree 7: 4)
    assert err.max() <= 8.0, err.max()
    assert np.array_equal(o[~fin, 5], lr[~fin], equal_nan=True), (a[~fin], b[~fin], o[~fin, 5])
    # mpmath sample for asin
    mpmath = pytest.importorskip("mpmath")
    mpmath.mp.prec = 100
    worst = 0.0
    for i in range(0, n, 997):
        if not fin[i] or x[i] == 0:
            continue
        ref = mpmath.asin(mpmath.mpf(float(x[i])))
        worst = max(worst, float(abs(mpmath.mpf(float(o[i, 4])) - ref)) / np.spacing(abs(float(ref))))
    assert worst <= 3.0, worst
