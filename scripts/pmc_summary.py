"""Per-kernel MFMA utilisation from a rocprofv3 --pmc CSV (see scripts/pmc_bench.sh).

util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs).
"""
import collections
import csv
import re
import sys


def main(path: str, top: int = 25) -> None:
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].replace("mpit::(anonymous namespace)::", "").replace("void ", "")
        k = re.sub(r"\(.*", "", k)[:70]
        d[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVES":
            n[k] += 1
    rows = []
    for k, c in d.items():
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        rows.append((cyc, k, n[k], c["SQ_INSTS_MFMA"], c["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024) if cyc else 0.0))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    mf = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"] for c in d.values())
    print(f"Whole run: MFMA util {mf / (tot * 1024):.1%} of busy GPU cycles.\n")
    print("| kernel | dispatches | share of GPU cycles | MFMA instrs (M) | MFMA util |\n|---|---|---|---|---|")
    for cyc, k, cnt, mi, u in rows[:top]:
        print(f"| `{k}` | {cnt} | {cyc / tot:.1%} | {mi / 1e6:.1f} | {u:.1%} |")


if __name__ == "__main__":
    main(sys.argv[1])
