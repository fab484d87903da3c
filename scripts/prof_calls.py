"""Per-dispatch durations of the kernels matching a pattern in the last steady-state
step of a rocprofv3 rocpd database (grid size identifies the layer).

    python scripts/prof_calls.py gpurun_out/prof "gemm_nt_kernel<128, 128, 4, 2, false>"
"""
import glob
import os
import sqlite3
import sys

d, pat = sys.argv[1], sys.argv[2]
marker = sys.argv[3] if len(sys.argv) > 3 else "ApplyF<true>"
db = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0]
c = sqlite3.connect(db)
rows = c.execute("select start, end, name, grid_x, grid_y, workgroup_x from kernels order by start").fetchall()
marks = [r[0] for r in rows if marker in r[2]]
lo, hi = marks[-2], marks[-1]
tot = 0
for s, e, n, gx, gy, wx in rows:
    if lo <= s < hi and pat in n:
        tot += e - s
        print(f"{(e - s) / 1e3:8.1f} us  grid={gx // max(wx, 1)}x{gy}  {n[:90]}")
print(f"total {tot / 1e3:.1f} us")
