"""Summarise a rocprofv3 ``--kernel-trace --stats`` CSV directory into a small markdown
file (the raw trace is too large to keep).

Steady state only: the per-step marker kernel (default: the Downpour push kernel, one per
training step) delimits steps; kernels between the marker of step ``-(k+1)`` and of the
last step are aggregated per name and divided by ``k``. This excludes MIOpen's
first-call algorithm search, which otherwise dominates the whole-run totals.
"""
import argparse
import csv
import glob
import os
import re


def _short(n, w=100):
    n = re.sub(r"\s+", " ", n)
    return n if len(n) <= w else n[: w - 3] + "..."


def _traces(d):
    """(path, [(start, end, name)]) per trace: rocprofv3 CSV or rocpd SQLite output."""
    for t in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        yield t, [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", ""))
                  for r in csv.DictReader(open(t))]
    for t in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        import sqlite3

        c = sqlite3.connect(t)
        yield t, [(int(a), int(b), n) for a, b, n in c.execute("select start, end, name from kernels")]


def summarise(d, out, marker="ApplyF<true>", k=3, top=30):
    lines = []
    for t, rows in _traces(d):
        rows.sort()
        marks = [s for (s, e, n) in rows if marker in n]
        if len(marks) < k + 1:
            lines.append(f"trace {t}: only {len(marks)} marker kernels, cannot window")
            continue
        lo, hi = marks[-(k + 1)], marks[-1]
        agg, busy = {}, 0
        for s, e, n in rows:
            if lo <= s < hi:
                a = agg.setdefault(_short(n), [0, 0])
                a[0] += 1
                a[1] += e - s
                busy += e - s
        wall = hi - lo
        lines.append(f"## steady state: {k} steps, {wall / k / 1e6:.2f} ms/step wall, "
                     f"{busy / k / 1e6:.2f} ms/step summed kernel time\n")
        lines.append("| kernel | calls/step | us/step | % of kernel time |")
        lines.append("|---|---|---|---|")
        for n, (c, s) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
            lines.append(f"| `{n}` | {c / k:.1f} | {s / k / 1e3:.1f} | {100 * s / max(busy, 1):.2f} |")
        lines.append("")
        mp = {n: v for n, v in agg.items() if "mpit" in n}
        if mp:
            lines.append("### mpit kernels (per step)\n")
            lines.append("| kernel | calls/step | us/call |")
            lines.append("|---|---|---|")
            for n, (c, s) in sorted(mp.items(), key=lambda kv: -kv[1][1]):
                lines.append(f"| `{n}` | {c / k:.1f} | {s / c / 1e3:.1f} |")
            lines.append("")
    open(out, "w").write("\n".join(lines) + "\n")
    return "\n".join(lines)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("out")
    ap.add_argument("--marker", default="ApplyF<true>")
    ap.add_argument("-k", type=int, default=3)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    print(summarise(a.dir, a.out, a.marker, a.k, a.top))
