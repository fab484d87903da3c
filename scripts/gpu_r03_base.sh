#!/bin/bash
# Round-3 baseline: default bench line (stderr kept), then the 8-rank one-GPU Allreduce
# collapse diagnosis: cgroup cpu.stat around 4- and 8-rank runs, and the 8-rank run with
# one hardware queue per process (GPU_MAX_HW_QUEUES=1) to separate CPU-quota throttling
# from GPU queue oversubscription.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-400
CG=/sys/fs/cgroup/cpu.stat
cat /sys/fs/cgroup/cpu.max > $O/cpu_max.txt 2>/dev/null
nproc > $O/nproc.txt
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --master-port 29541"
ar() {  # name nranks env...
  local name=$1 n=$2; shift 2
  cat $CG > $O/$name.cpustat_before 2>/dev/null
  env "$@" timeout -k 10 240 $TR --nproc-per-node $n benchmarks/allreduce_bench.py --megs 10 --iters 10 \
    > $O/$name.json 2> $O/$name.err || { echo "FAILED $name"; tail -20 $O/$name.err; cat $CG > $O/$name.cpustat_after; return 1; }
  cat $CG > $O/$name.cpustat_after 2>/dev/null
  echo "$name: $(tail -1 $O/$name.json)"
}
ar ar4 4 MPIT_X=0 || exit 1
ar ar8 8 MPIT_X=0 || exit 1
ar ar8_hwq1 8 GPU_MAX_HW_QUEUES=1 || exit 1
ar ar8_yield256 8 MPIT_PROGRESS_YIELDS=256 || exit 1
echo ALL OK
