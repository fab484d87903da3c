#!/bin/bash
# Round 3: stream-hygiene GPU test, then the 8-rank one-GPU rehearsal (bench.py --gpus 8,
# batch 32) with cgroup cpu.stat around it: parked progress threads (default) vs the
# round-2 idle loop (MPIT_PROGRESS_PARK=0 MPIT_PROGRESS_YIELDS=4096).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_streams.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_streams.log 2>&1
rc=$?; tail -3 $O/pytest_streams.log; [ $rc -ge 124 ] && exit $rc
CG=/sys/fs/cgroup/cpu.stat
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --master-port 29547"
n8() {  # name env...
  local name=$1; shift
  cat $CG > $O/$name.cpustat_before
  env "$@" timeout -k 10 420 $TR --nproc-per-node 8 bench.py --gpus 8 --batch 32 --steps 4 --warmup 2 \
    > $O/$name.json 2> $O/$name.err || { echo "FAILED $name"; tail -30 $O/$name.err; cat $CG > $O/$name.cpustat_after; return 1; }
  cat $CG > $O/$name.cpustat_after
  echo "$name: $(tail -1 $O/$name.json | cut -c1-300)"
  python3 - "$O/$name.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d.get("secondary", {})
print("  ms/step", d["ms_per_step"], "allreduce", s.get("allreduce"), "pingpong", s.get("ps_pingpong"), "rccl", d.get("rccl"))
PY
}
n8 n8_park MPIT_X=0 || exit 1
n8 n8_spin MPIT_PROGRESS_PARK=0 MPIT_PROGRESS_YIELDS=4096 || exit 1
echo ALL OK
