"""CPU checks of tools/table_vs_minimizer.py, the restatement of RunMultiRayCode_loop.C's grid
(:40-95) and comparison (:116-187); the GPU run against the oracle is
tests/test_gpu_loop_validation.py."""
import numpy as np

from tools import table_vs_minimizer as tvm


def test_harness_grid():
    hR, D, thR, shape = tvm.harness_queries()
    assert shape == (789, 390) and hR.size == 307710
    assert hR[0] == 300100.0 and thR[0] == 90.2 and thR[389] == 90.2 + 389 * 0.23
    assert hR[390] == 300100.0 + 12300.0          # loop order: heights outer, angles inner
    # the straight line from Tx hits the antenna 200 m below the surface (:89-95)
    i = 390 * 100 + 150
    exp = (hR[i] - 300000.0 + 20000.0) * np.tan((180 - thR[i]) * (3.1415927 / 180))
    assert D[i] == exp and np.all(D > 0)


def test_harness_values_and_counts():
    ok = np.array([1, 1, 0, 1, 1], np.uint8)
    tok = np.array([1, 0, 1, 1, 1], np.uint8)
    hd = np.array([100.0, 200.0, 300.0, np.nan, 500.0]) * 100
    td = np.array([101.0, 0.0, 300.0, 400.0, 0.0]) * 100
    rt, it = tvm.harness_values(hd, ok, td, tok)
    assert rt.tolist() == [100.0, 200.0, -1000.0, -1000.0, 500.0]
    assert it.tolist() == [101.0, -1000.0, 300.0, 400.0, -1000.0]   # table 0 -> no result
    s = tvm.summarize(rt, it)
    assert (s["count1_minimizer_solved"], s["count2_table_solved"], s["count3_both"],
            s["count4_table_only"], s["minimizer_only"]) == (3, 3, 1, 2, 2)
    assert np.isclose(s["percent_error"]["max"], 1.0) and s["h1error_dRR_counts"][2] == 1
