"""Regenerate tests/golden/table_cfg2_rows.npz from the oracle (regression fixture)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle  # noqa: E402

m = oracle.load_atmosphere(os.path.join(HERE, "..", "..", "airiceraytracing_amd", "data",
                                        "Atmosphere.dat.gz"))
g = oracle.grid_init(-20000.0, 300000.0, 20.0, 92.0, 180.0, 0.5)
rows = np.array([0, 1, 1000, 2500, 4000, 4800, 4849, 4850])
full = np.stack([oracle.table_rows(m, g, int(r), int(r) + 1, full=True)[1] for r in rows])
np.savez_compressed(os.path.join(HERE, "table_cfg2_rows.npz"), rows=rows, full=full)
print(full.shape)
