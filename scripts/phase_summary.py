"""Phase breakdown of a training run from a rocprofv3 ``--marker-trace`` (roctx ranges
emitted by mpit_amd with MPIT_TRACE=1: step / fwd / bwd / gather_shard<k> / ps_wait on the
worker, ps_update / ps_copy_* in the native server) plus the kernel trace.

    python scripts/phase_summary.py <rocprofv3 out dir> <out.md> [--skip N]

Per process (pid) and range name: calls, mean and total host-side duration, skipping the
first ``--skip`` occurrences of every name (warmup). Kernel time per step is read from the
kernel trace between the first and the last kept ``step`` range of each pid.
"""
import argparse
import collections
import csv
import glob
import os


def _rows(d, pattern):
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        yield from csv.DictReader(open(f))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("out")
    ap.add_argument("--skip", type=int, default=2)
    a = ap.parse_args()
    ranges = collections.defaultdict(list)  # (pid, name) -> [(start, end)]
    for r in _rows(a.dir, "*marker_api_trace.csv"):
        name = r.get("Function") or r.get("Name") or r.get("Operation") or ""
        pid = r.get("Process_Id") or r.get("Pid") or "?"
        try:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        except (KeyError, ValueError):
            continue
        ranges[(pid, name)].append((s, e))
    kern = collections.defaultdict(list)
    for r in _rows(a.dir, "*kernel_trace.csv"):
        # rocprofv3's kernel trace has no process column: one traced process per output
        # file name (-o name_%pid%) or all kernels of the single traced process
        pid = r.get("Process_Id") or r.get("Pid") or "*"
        kern[pid].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "")))
    lines = ["# Phase breakdown (roctx ranges, host time)", "",
             f"Source: rocprofv3 --marker-trace --kernel-trace; first {a.skip} occurrences of each range skipped.", "",
             "| pid | range | calls | mean ms | total ms |", "|---|---|---|---|---|"]
    for (pid, name), v in sorted(ranges.items()):
        v = sorted(v)[a.skip:]
        if not v:
            continue
        d = [(e - s) / 1e6 for s, e in v]
        lines.append(f"| {pid} | `{name}` | {len(d)} | {sum(d) / len(d):.3f} | {sum(d):.2f} |")
    lines += ["", "## Device time inside the kept steps", "", "| pid | steps | ms/step wall | kernel ms/step (summed) | top kernels (ms/step) |",
              "|---|---|---|---|---|"]
    for (pid, name), v in sorted(ranges.items()):
        if name != "step":
            continue
        v = sorted(v)[a.skip:]
        if len(v) < 2:
            continue
        lo, hi = v[0][0], v[-1][1]
        ks = [k for k in kern.get(pid, kern.get("*", [])) if lo <= k[0] < hi]
        agg = collections.Counter()
        for s, e, n in ks:
            base = n.replace("void ", "").replace("mpit::(anonymous namespace)::", "").replace("at::native::", "")
            agg[base.split("<")[0].split("(")[0][:40]] += (e - s) / 1e6
        n = len(v)
        top = ", ".join(f"{k} {t / n:.2f}" for k, t in agg.most_common(5))
        lines.append(f"| {pid} | {n} | {(hi - lo) / 1e6 / n:.2f} | {sum(agg.values()) / n:.2f} | {top} |")
    open(a.out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
