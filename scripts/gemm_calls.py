"""Per-call GEMM table of one training step: joins the MPIT_GEMM_LOG=1 launch log (shapes,
issue order) with a rocprofv3 kernel trace of the same process (times), family by family
(gemm_nt / gemm_tn dispatches keep their issue order), over the last steady step (the
Downpour apply kernel marks step boundaries). TFLOP/s are of the GEMM's own M x N x K
(real fp32 or bf16 work, not the 6 split products of the fp32 path).

    python scripts/gemm_calls.py <stderr log> <trace dir> <out.md> [title]
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main():
    logf, tdir, out = sys.argv[1:4]
    title = sys.argv[4] if len(sys.argv) > 4 else "GEMM calls of one steady step"
    calls = {"nt": [], "tn": []}
    for line in open(logf, errors="replace"):
        m = re.search(r"MPIT_GEMM (nt|tn) (\d+) (\d+) (\d+) conv=(\d) (\w+)=(\d+)", line)
        if m:
            calls[m.group(1)].append((int(m.group(2)), int(m.group(3)), int(m.group(4)), int(m.group(5)),
                                      f"{m.group(6)}={m.group(7)}"))
    f = glob.glob(os.path.join(tdir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(f)):
        blocks = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], blocks))
    rows.sort()
    fam = {"nt": [x for x in rows if "gemm_nt_kernel" in x[2]], "tn": [x for x in rows if "gemm_tn_kernel" in x[2]]}
    for k in fam:
        if len(fam[k]) != len(calls[k]):
            sys.exit(f"{k}: {len(fam[k])} dispatches in the trace vs {len(calls[k])} logged launches")
    marks = [s for s, e, n, b in rows if "ApplyF<true>" in n]
    lo, hi = marks[-2], marks[-1]
    lines = [f"# {title}", "", f"step wall (apply to apply): {(hi - lo) / 1e6:.2f} ms", ""]
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    tot = {}
    for k in ("nt", "tn"):
        idx = [i for i, x in enumerate(fam[k]) if lo <= x[0] < hi]
        t_us, fl = 0.0, 0.0
        lines += [f"## gemm_{k}: {len(idx)} calls", "", "| # | M | N | K | conv | mode | blocks | us | TFLOP/s |",
                  "|---|---|---|---|---|---|---|---|---|"]
        for j, i in enumerate(idx):
            s, e, name, blocks = fam[k][i]
            M, N, K, conv, mode = calls[k][i]
            us = (e - s) / 1e3
            flop = 2.0 * M * N * K
            t_us += us
            fl += flop
            a = agg[(k, M, N, K, conv)]
            a[0] += 1
            a[1] += us
            a[2] += flop
            lines.append(f"| {j} | {M} | {N} | {K} | {conv} | {mode} | {blocks} | {us:.1f} | {flop / us / 1e6:.1f} |")
        tot[k] = (t_us, fl)
        lines += ["", f"gemm_{k} total {t_us / 1e3:.2f} ms, {fl / 1e12:.3f} TFLOP, {fl / max(t_us, 1e-9) / 1e6:.1f} TFLOP/s",
                  ""]
    lines += ["## by shape (sorted by time)", "", "| kind | M | N | K | conv | calls | us total | TFLOP/s |",
              "|---|---|---|---|---|---|---|---|"]
    for (k, M, N, K, conv), (n, us, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"| {k} | {M} | {N} | {K} | {conv} | {n} | {us:.0f} | {fl / us / 1e6:.1f} |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:4]))
    for k, (t, fl) in tot.items():
        print(f"gemm_{k}: {t / 1e3:.2f} ms  {fl / max(t, 1e-9) / 1e6:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
