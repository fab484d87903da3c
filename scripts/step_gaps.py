"""GPU idle time inside the steady steps of a kernel trace (union of all streams' kernel
intervals vs step wall; the Downpour apply kernel marks step boundaries) and the largest
gaps with the kernels on either side.

    python scripts/step_gaps.py <trace dir> [steps]
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f)))
    marks = [s for s, e, n in rows if "ApplyF<true>" in n]
    for k in range(max(0, len(marks) - 1 - nsteps), len(marks) - 1):
        lo, hi = marks[k], marks[k + 1]
        busy, cur_s, cur_e, prev, gaps = 0, None, None, None, []
        for s, e, n in (x for x in rows if lo <= x[0] < hi):
            n = n.replace("mpit::(anonymous namespace)::", "").replace("void ", "")[:50]
            if cur_e is None:
                cur_s, cur_e, prev = s, e, n
            elif s > cur_e:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, prev, n))
                cur_s, cur_e, prev = s, e, n
            elif e > cur_e:
                cur_e, prev = e, n
        busy += cur_e - cur_s
        gaps.sort(reverse=True)
        print(f"step wall {(hi - lo) / 1e6:.2f} ms, GPU busy {busy / 1e6:.2f} ms, idle {(hi - lo - busy) / 1e6:.2f} ms "
              f"in {len(gaps)} gaps")
        for g in gaps[:4]:
            print(f"    {g[0] / 1e3:7.1f} us  {g[1]}  ->  {g[2]}")


if __name__ == "__main__":
    main()
