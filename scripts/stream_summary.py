"""Per-stream view of a rocprofv3 kernel trace of the training step.

    python scripts/stream_summary.py <trace dir> <out.md> [marker] [steps]

Steps are delimited by the marker kernel (default ``cast_batch_kernel``: the per-step
weight plan, the first kernel of every step); the last ``steps`` complete steps (default 2)
are aggregated. Per stream: busy time (union of kernel intervals), and the kernels ranked by
summed time. The critical path of a step is the compute stream's busy time; the side
stream's kernels overlap it.
"""
import collections
import csv
import glob
import os
import re
import sys


def _short(n, w=70):
    n = n.replace("void ", "").replace("mpit::(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    return n[:w]


def _union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if cs is None:
            cs, ce = s, e
        elif s <= ce:
            ce = max(ce, e)
        else:
            tot += ce - cs
            cs, ce = s, e
    return tot + (ce - cs if cs is not None else 0)


def main():
    d, out = sys.argv[1], sys.argv[2]
    marker = sys.argv[3] if len(sys.argv) > 3 else "cast_batch_kernel"
    nsteps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    rows = []
    for t in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(t)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [int(r["Start_Timestamp"]) for r in rows if marker in r["Kernel_Name"]]
    if len(starts) < nsteps + 1:
        raise SystemExit(f"only {len(starts)} markers")
    a, b = starts[-(nsteps + 1)], starts[-1]
    sel = [r for r in rows if a <= int(r["Start_Timestamp"]) < b]
    by = collections.defaultdict(list)
    for r in sel:
        by[r["Stream_Id"]].append(r)
    lines = [f"# Per-stream kernel time, {nsteps} steady steps (`{d}`)", "",
             f"step wall (marker to marker): {(b - a) / 1e6 / nsteps:.2f} ms; any-stream busy "
             f"{_union([(int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in sel]) / 1e6 / nsteps:.2f} ms/step", ""]
    for sid, rs in sorted(by.items(), key=lambda kv: -len(kv[1])):
        busy = _union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rs]) / 1e6 / nsteps
        lines += [f"## stream {sid}: {len(rs) / nsteps:.0f} kernels/step, busy {busy:.2f} ms/step", "",
                  "| kernel | calls/step | us/step |", "|---|---|---|"]
        c = collections.defaultdict(lambda: [0, 0.0])
        for r in rs:
            k = _short(r["Kernel_Name"])
            c[k][0] += 1
            c[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        for k, (n, t) in sorted(c.items(), key=lambda kv: -kv[1][1])[:25]:
            lines.append(f"| `{k}` | {n / nsteps:.0f} | {t / nsteps:.1f} |")
        lines.append("")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:4]))


if __name__ == "__main__":
    main()
