#!/bin/bash
# Round 3: (1) what limits the fp32 (bf16x6) GEMMs — each shape timed as built and with the
# operand split removed (MPIT_F32_ABLATE=nosplit: timing-only ablation, wrong numbers), plus
# one counter pass each; (2) the 8-rank one-GPU collapse with 2 hardware queues per process.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
: > $O/probe.jsonl
for P in "nt 50176 1024 512" "nt 200704 512 128" "nt 802816 256 64" "conv 256 14 14 256 256 3 1" "conv 256 56 56 64 64 3 1" "dgrad 256 28 28 128 128 3 1" "wgrad 256 28 28 128 128 3 1"; do
  for A in none nosplit; do
    MPIT_F32_ABLATE=$A timeout -k 10 120 python3 benchmarks/gemm_probe.py --f32 $P 20 > $O/t.json || exit 1
    echo "{\"ablate\": \"$A\", \"r\": $(cat $O/t.json)}" >> $O/probe.jsonl
  done
done
cat $O/probe.jsonl
i=0
for A in none nosplit; do
  i=$((i+1))
  MPIT_F32_ABLATE=$A timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d $O/pmc$i -o p --output-format csv -- python3 benchmarks/gemm_probe.py --f32 conv 256 14 14 256 256 3 1 5 > $O/pmc$i.log 2>&1 || { tail -5 $O/pmc$i.log; exit 1; }
  MPIT_F32_ABLATE=$A timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d $O/pmcb$i -o p --output-format csv -- python3 benchmarks/gemm_probe.py --f32 conv 256 14 14 256 256 3 1 5 > $O/pmcb$i.log 2>&1 || { tail -5 $O/pmcb$i.log; exit 1; }
done
echo pmc done
CG=/sys/fs/cgroup/cpu.stat
cat $CG > $O/n8_hwq2.cpustat_before
GPU_MAX_HW_QUEUES=2 timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --master-port 29549 --nproc-per-node 8 bench.py --gpus 8 --batch 32 --steps 4 --warmup 2 > $O/n8_hwq2.json 2> $O/n8_hwq2.err || { tail -30 $O/n8_hwq2.err; exit 1; }
cat $CG > $O/n8_hwq2.cpustat_after
python3 - "$O/n8_hwq2.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d.get("secondary", {})
print("hwq2 ms/step", d["ms_per_step"], "allreduce", s.get("allreduce"), "pingpong agg", (s.get("ps_pingpong") or {}).get("aggregate_GBps_bidir"))
PY
echo ALL OK
