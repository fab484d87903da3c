#!/bin/bash
# Round 3: which operand's split costs what (MPIT_F32_ABLATE=splitA: only A split, B raw;
# splitB: only B split) on the fp32 GEMM shapes; emu8 with 2 shared link streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
: > $O/probe.jsonl
for P in "nt 50176 1024 512" "nt 200704 512 128" "conv 256 14 14 256 256 3 1" "conv 256 56 56 64 64 3 1" "dgrad 256 28 28 128 128 3 1"; do
  for A in none splitA splitB nosplit; do
    MPIT_F32_ABLATE=$A timeout -k 10 120 python3 benchmarks/gemm_probe.py --f32 $P 20 > $O/t.json || exit 1
    echo "{\"ablate\": \"$A\", \"r\": $(cat $O/t.json)}" >> $O/probe.jsonl
  done
done
cat $O/probe.jsonl
MPIT_PS_LINK_STREAMS=2 timeout -k 10 240 python -u bench.py --no-secondary --steps 20 --warmup 5 --emulate-shards 8 > $O/emu8_l2.json 2> $O/emu8_l2.err || { tail -20 $O/emu8_l2.err; exit 1; }
timeout -k 10 240 python -u bench.py --no-secondary --steps 20 --warmup 5 --emulate-shards 8 > $O/emu8.json 2> $O/emu8.err || { tail -20 $O/emu8.err; exit 1; }
echo "emu8 links=2: $(tail -1 $O/emu8_l2.json | cut -c1-160)"
echo "emu8 links=8: $(tail -1 $O/emu8.json | cut -c1-160)"
echo ALL OK
