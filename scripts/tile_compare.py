"""Call-by-call comparison of the gemm_nt kernels of two kernel traces of the same training
step (e.g. default 128-row tiles vs MPIT_GEMM_TILE=256), aligned by their order within the
last steady step (the Downpour apply kernel marks step boundaries).

    python scripts/tile_compare.py <trace dir A> <trace dir B> <out.md>
"""
import csv
import glob
import os
import re
import sys


def load(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(f)):
        blocks = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], blocks))
    rows.sort()
    marks = [s for s, e, n, b in rows if "ApplyF<true>" in n]
    lo, hi = marks[-2], marks[-1]
    step = [x for x in rows if lo <= x[0] < hi]
    nt = [x for x in step if "gemm_nt_kernel" in x[2]]
    return (hi - lo) / 1e6, step, nt


def tile(name):
    m = re.search(r"gemm_nt_kernel<[^,]+, (\d+), (\d+),", name)
    return f"{m.group(1)}x{m.group(2)}" if m else "?"


def main():
    a, b, out = sys.argv[1:4]
    wa, sa, na = load(a)
    wb, sb, nb = load(b)
    lines = [f"# gemm_nt call by call: {os.path.basename(a)} vs {os.path.basename(b)}", "",
             f"step wall: {wa:.2f} ms vs {wb:.2f} ms; gemm_nt summed: {sum(e - s for s, e, _, _ in na) / 1e6:.2f} ms vs "
             f"{sum(e - s for s, e, _, _ in nb) / 1e6:.2f} ms ({len(na)} vs {len(nb)} calls)", "",
             "| # | tile A | blocks A | us A | tile B | blocks B | us B | B/A |", "|---|---|---|---|---|---|---|---|"]
    for i, (x, y) in enumerate(zip(na, nb)):
        ua, ub = (x[1] - x[0]) / 1e3, (y[1] - y[0]) / 1e3
        if tile(x[2]) == tile(y[2]):
            continue  # same tile in both runs
        lines.append(f"| {i} | {tile(x[2])} | {x[3]} | {ua:.1f} | {tile(y[2])} | {y[3]} | {ub:.1f} | {ub / ua:.2f} |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
