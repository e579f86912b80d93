"""Per-kernel durations from a rocprofv3 SQLite result (rocpd), split by grid size:
    python tools/prof_db.py gpurun_out/<dir>/run_results.db [min_grid]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
min_grid = int(sys.argv[2]) if len(sys.argv) > 2 else 0
rows = c.execute("select name, grid_x, count(*), avg(duration), min(duration) from kernels "
                 "where grid_x >= ? group by name, grid_x order by sum(duration) desc", (min_grid,))
for name, grid, n, avg, mn in rows:
    print(f"{avg / 1e3:10.2f} us avg {mn / 1e3:10.2f} min  x{n:<5d} grid {grid:<10d} {name[:80]}")
