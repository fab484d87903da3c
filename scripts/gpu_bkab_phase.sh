#!/bin/bash
# Same-box bench A/B of the fp32 k-tile depth (16 vs 32, alternating), then a roctx phase
# breakdown of the default step (1 rank) and of a 2-rank co-located PS run on the one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/bkab
mkdir -p $D
: > $D/ab.txt
for i in 1 2; do for bk in 16 32; do
  MPIT_F32_BK=$bk timeout -k 10 300 python -u bench.py --no-secondary > $D/b_${bk}_$i.log 2>&1 || { tail -20 $D/b_${bk}_$i.log; exit 1; }
  echo "bk=$bk run=$i $(tail -1 $D/b_${bk}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $D/ab.txt
done; done
MPIT_TRACE=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $D/ph1 -o ph -- python3 bench.py --steps 6 --warmup 2 --no-secondary > $D/ph1.log 2>&1 || { tail -20 $D/ph1.log; exit 1; }
python3 scripts/phase_summary.py $D/ph1 $D/phase_n1.md --skip 2 > /dev/null || exit 1
find $D/ph1 -name "*.csv" -size +30M -delete
echo phase done
