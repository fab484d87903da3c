#!/bin/bash
# Round 3 (session 2): wave-cycle breakdown of the fp16x3 NT kernel (FM 11) on two shapes,
# two PMC passes each (the r03q recipe for FM 9).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ad
mkdir -p $O
i=0
for P in "conv 256 14 14 256 256 3 1" "nt 50176 1024 512" "tn 50176 1024 256"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d $O/a$i -o a --output-format csv -- python3 benchmarks/gemm_probe.py --f32 --f16x3 $P 5 > $O/a$i.log 2>&1 || { tail -5 $O/a$i.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE --kernel-trace -d $O/b$i -o b --output-format csv -- python3 benchmarks/gemm_probe.py --f32 --f16x3 $P 5 > $O/b$i.log 2>&1 || { tail -5 $O/b$i.log; exit 1; }
done
python3 - <<'PY' > $O/breakdown.txt
import csv, glob, collections
for i in (1, 2, 3):
    out = {}
    for ps in "ab":
        agg = collections.defaultdict(float)
        for f in glob.glob(f"gpurun_out/r03ad/{ps}{i}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "gemm_nt" in r["Kernel_Name"] or "gemm_tn" in r["Kernel_Name"]:
                    agg[r["Counter_Name"]] += float(r["Counter_Value"])
        wc = agg.get("SQ_WAVE_CYCLES") or 1
        for k, v in agg.items():
            out[k if k != "GRBM_GUI_ACTIVE" else k + "_" + ps] = round(v / wc, 3) if k.startswith(("SQ_WAIT", "SQ_ACTIVE")) else v
        if ps == "b" and agg.get("GRBM_GUI_ACTIVE"):
            out["mfma_util"] = round(agg["SQ_VALU_MFMA_BUSY_CYCLES"] / (agg["GRBM_GUI_ACTIVE"] / 8 * 1024), 3)
    print(i, out)
PY
cat $O/breakdown.txt
find $O -name "*.csv" -size +20M -delete
echo ALL OK
