"""Summarise a rocprofv3 kernel-trace database of benchmarks/bn_apply_bw_probe.py: median
kernel time and bandwidth per shape for the backward apply (with / without the ReLU mask),
the forward apply and PyTorch's addcmul (same bytes), from the GPU's own timestamps.

    python benchmarks/bn_probe_summary.py <rocprof dir> <fp32|bf16>
"""
import glob
import json
import re
import sqlite3
import statistics
import sys

SH = [(112 * 112, 64), (56 * 56, 64), (56 * 56, 256), (28 * 28, 128), (28 * 28, 512), (14 * 14, 256),
      (14 * 14, 1024), (7 * 7, 512), (7 * 7, 2048)]
IT, WARM = 23, 3  # calls per kind and shape in the probe (timeit: 3 warm-up + 20)


def kind(n):
    if "bn_bwd_apply_kernel" in n:
        return "bwd" if re.search(r"bn_bwd_apply_kernel<[^,]+, true", n) else "bwd_nomask"
    if "bn_apply_kernel" in n:
        return "fwd"
    if "addcmul" in n:
        return "ref"
    return None


def main():
    d, dt = sys.argv[1], sys.argv[2]
    es = 2 if dt == "bf16" else 4
    c = sqlite3.connect(glob.glob(f"{d}/**/*.db", recursive=True)[0])
    seq = {}
    for n, dur in c.execute("select name, duration from kernels order by start"):
        k = kind(n)
        if k:
            seq.setdefault(k, []).append(dur)
    tot = {}
    for si, (hw, C) in enumerate(SH):
        M = 256 * hw
        row = {"M": M, "C": C}
        for k, v in seq.items():
            med = statistics.median(v[si * IT + WARM:(si + 1) * IT]) / 1e3  # us
            by = M * C * 3 * es + (M * C // 8 if k == "bwd" else 0)
            row[k + "_us"] = round(med, 1)
            row[k + "_TBs"] = round(by / med / 1e6, 2)
            tot[k] = tot.get(k, 0.0) + med
        print(json.dumps(row))
    print(json.dumps({"total_us": {k: round(v, 1) for k, v in tot.items()}}))


if __name__ == "__main__":
    main()
