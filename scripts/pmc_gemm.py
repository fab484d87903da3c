#!/usr/bin/env python3
"""Wave-cycle breakdown of the fp16x3 GEMM kernels on a few shapes from PMC counters: two
`rocprofv3 --pmc` passes per shape (each its own run, counters only with the kernel trace),
the GEMM kernels' counters summed, wait / active fractions of SQ_WAVE_CYCLES, MFMA util =
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024) (the round-3 recipe,
profiles/gemm_fp16x3_cycles_r03.md).

    gpurun -- python3 scripts/pmc_gemm.py <outdir> ["conv 256 14 14 256 256 3 1" ...]

PMC_PROBE_FLAGS="--planes": the operands as fp16 planes (gemm.hip FM 13).
"""
import collections
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = {
    "a": "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA "
         "SQ_INSTS_VALU GRBM_GUI_ACTIVE",
    "b": "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT "
         "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE",
}
SHAPES = ["conv 256 14 14 256 256 3 1", "nt 50176 1024 512", "tn 50176 1024 256"]


def main():
    out = os.path.join(ROOT, "gpurun_out", sys.argv[1])
    shapes = sys.argv[2:] or SHAPES
    os.makedirs(out, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    res = []
    for i, shape in enumerate(shapes):
        row = {"shape": shape}
        for ps, ctrs in PASSES.items():
            d = os.path.join(out, f"{ps}{i}")
            cmd = (["timeout", "-s", "KILL", "90", "rocprofv3", "--pmc"] + ctrs.split() +
                   ["--kernel-trace", "-d", d, "-o", ps, "--output-format", "csv", "--", sys.executable,
                    "benchmarks/gemm_probe.py", "--f32", "--f16x3"] + os.environ.get("PMC_PROBE_FLAGS", "").split()
                   + shape.split() + ["5"])
            with open(os.path.join(out, f"{ps}{i}.log"), "w") as f:
                rc = subprocess.call(cmd, stdout=f, stderr=subprocess.STDOUT, cwd=ROOT, env=env)
            if rc != 0:
                print(f"[pmc_gemm] {shape} pass {ps}: rc={rc}", flush=True)
                return rc
            agg = collections.defaultdict(float)
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                for r in csv.DictReader(open(f)):
                    if "gemm_nt" in r["Kernel_Name"] or "gemm_tn" in r["Kernel_Name"] or "conv" in r["Kernel_Name"]:
                        agg[r["Counter_Name"]] += float(r["Counter_Value"])
            row[ps] = dict(agg)
            for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
                if os.path.getsize(f) > 20 << 20:
                    os.remove(f)
        a, b = row["a"], row["b"]
        wc = a.get("SQ_WAVE_CYCLES") or 1.0
        mf = a.get("SQ_INSTS_MFMA") or 1.0
        summ = {
            "shape": shape,
            "mfma_util": round(b.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (b.get("GRBM_GUI_ACTIVE", 1) / 8 * 1024), 3),
            "valu_per_mfma": round(a.get("SQ_INSTS_VALU", 0) / mf, 2),
            "salu_per_mfma": round(b.get("SQ_INSTS_SALU", 0) / mf, 2),
            "lds_per_mfma": round(b.get("SQ_INSTS_LDS", 0) / mf, 2),
            "active": round(a.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3),
            "wait_dependency": round(a.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
            "wait_any": round(a.get("SQ_WAIT_ANY", 0) / wc, 3),
            "lds_bank_conflict": b.get("SQ_LDS_BANK_CONFLICT", 0),
        }
        res.append(summ)
        print(json.dumps(summ), flush=True)
    with open(os.path.join(out, "breakdown.jsonl"), "w") as f:
        for r in res:
            f.write(json.dumps(r) + "\n")
    print("[pmc_gemm] ALL OK", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
