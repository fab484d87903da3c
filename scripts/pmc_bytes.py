#!/usr/bin/env python3
"""HBM bytes per kernel of the bench step from PMC counters: two `rocprofv3 --pmc` passes over a
short `bench.py` run (FETCH_SIZE, then WRITE_SIZE: together they exceed the 4 TCC counters of
one pass), counters only with the kernel trace. Bytes per call are averaged per kernel name and
written to <outdir>/bytes.json; `scripts/pmc_bytes.py --table <outdir> <streams.md>` joins them
with a stream table's per-step time (scripts/stream_summary.py) into TB/s per kernel.

    gpurun -- python3 scripts/pmc_bytes.py <outdir> [bench args...]
"""
import collections
import csv
import glob
import json
import os
import re
import subprocess
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = {"fetch": "FETCH_SIZE", "write": "WRITE_SIZE"}  # KB per dispatch (summed over TCC channels)


def short(name: str) -> str:
    name = re.sub(r"^void ", "", name).replace("mpit::(anonymous namespace)::", "")
    return name.split("(")[0]


def collect(outdir: str, bench_args) -> int:
    out = os.path.join(ROOT, "gpurun_out", outdir)
    os.makedirs(out, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    per = collections.defaultdict(lambda: {"calls": 0})
    for ps, ctr in PASSES.items():
        d = os.path.join(out, ps)
        cmd = (["timeout", "-s", "KILL", "300", "rocprofv3", "--pmc", ctr, "--kernel-trace", "-d", d, "-o", "t",
                "--output-format", "csv", "--", sys.executable, "-u", os.path.join(ROOT, "bench.py")] + bench_args)
        with open(os.path.join(out, f"{ps}.log"), "w") as f:
            r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=f, stderr=subprocess.STDOUT)
        print(f"[pmc_bytes] pass {ps}: rc={r.returncode}", flush=True)
        if r.returncode:
            return r.returncode
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            print(f"[pmc_bytes] pass {ps}: no counter_collection.csv", flush=True)
            return 1
        seen = collections.Counter()
        for row in csv.DictReader(open(files[0])):
            k = short(row["Kernel_Name"])
            per[k][ps] = per[k].get(ps, 0.0) + float(row["Counter_Value"]) * 1024.0
            seen[k] += 1
        for k, n in seen.items():
            per[k]["calls_" + ps] = n
        for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
            if os.path.getsize(f) > 20 << 20:
                os.remove(f)
    res = {k: {"fetch_bytes_per_call": v.get("fetch", 0.0) / max(1, v.get("calls_fetch", 1)),
               "write_bytes_per_call": v.get("write", 0.0) / max(1, v.get("calls_write", 1)),
               "calls": v.get("calls_fetch", 0)} for k, v in per.items()}
    with open(os.path.join(out, "bytes.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(f"[pmc_bytes] {len(res)} kernels -> {out}/bytes.json", flush=True)
    return 0


def table(outdir: str, streams_md: str) -> None:
    res = json.load(open(os.path.join(outdir, "bytes.json")))
    rows = []
    for line in open(streams_md):
        m = re.match(r"\| `(.+?)` \| (\d+) \| ([\d.]+) \|", line)
        if not m:
            continue
        name, calls, us = m.group(1), int(m.group(2)), float(m.group(3))
        hit = [k for k in res if k.startswith(name.rstrip("…"))]
        if len(hit) != 1:
            continue
        b = res[hit[0]]
        byt = calls * (b["fetch_bytes_per_call"] + b["write_bytes_per_call"])
        rows.append((us, name, calls, b["fetch_bytes_per_call"] * calls / 1e6, b["write_bytes_per_call"] * calls / 1e6,
                     byt / (us * 1e-6) / 1e12 if us else 0.0))
    print("| kernel | calls/step | us/step | read MB/step | write MB/step | TB/s |")
    print("|---|---|---|---|---|---|")
    for us, name, calls, rd, wr, tbs in sorted(rows, reverse=True):
        print(f"| `{name}` | {calls} | {us:.1f} | {rd:.1f} | {wr:.1f} | {tbs:.2f} |")


if __name__ == "__main__":
    if sys.argv[1] == "--table":
        table(sys.argv[2], sys.argv[3])
    else:
        sys.exit(collect(sys.argv[1], sys.argv[2:]))
