"""Step-boundary latency chain of a parameter-server step from one rocprofv3
``--marker-trace --kernel-trace`` run (MPIT_TRACE=1, one process): for every steady step,
server apply kernel end -> host wakes from ps_wait -> next step range starts -> weight-cast
range starts -> weight-cast kernel starts -> next kernel starts (medians, us).

    python scripts/boundary_summary.py <rocprofv3 out dir>
"""
import csv
import glob
import os
import statistics
import sys


def rows(d, pat):
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        yield from csv.DictReader(open(f))


def main():
    d = sys.argv[1]
    rng = {}
    for r in rows(d, "*marker_api_trace.csv"):
        n = r.get("Function") or r.get("Name") or r.get("Operation") or ""
        try:
            rng.setdefault(n, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        except (KeyError, ValueError):
            pass
    for v in rng.values():
        v.sort()
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows(d, "*kernel_trace.csv"))
    applies = [(s, e) for s, e, n in ks if "ApplyF<true>" in n]
    chains = []
    for s_a, e_a in applies[2:-1]:
        wait_end = min((e for s, e in rng.get("ps_wait", []) if e >= e_a - 5_000_000), default=None)
        step_s = min((s for s, e in rng.get("step", []) if s >= e_a), default=None)
        wc_s = min((s for s, e in rng.get("wcast", []) if s >= e_a), default=None)
        cast = next(((s, e) for s, e, n in ks if s >= e_a and "cast_batch" in n), None)
        nxt = next((s for s, e, n in ks if cast and s >= cast[1]), None)
        if None in (wait_end, step_s, wc_s, cast, nxt):
            continue
        chains.append((wait_end - e_a, step_s - wait_end, wc_s - step_s, cast[0] - wc_s, nxt - cast[1],
                       cast[0] - e_a))
    if not chains:
        sys.exit("no complete step boundaries found")
    names = ["apply end -> ps_wait returns", "ps_wait -> next step range", "step start -> weight-cast range",
             "weight-cast range -> cast kernel", "cast kernel end -> next kernel", "apply end -> cast kernel (total)"]
    print(f"{len(chains)} step boundaries, medians in us:")
    for i, n in enumerate(names):
        print(f"  {n:34s} {statistics.median(c[i] for c in chains) / 1e3:8.1f}")


if __name__ == "__main__":
    main()
