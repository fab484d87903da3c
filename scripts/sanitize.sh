#!/bin/bash
# Host sanitizer runs of the native runtime (csrc/core + the host side of csrc/kernels) on the
# CPU: the multi-process API suite, parameter-server training (co-located, dedicated,
# EASGD, SSP) under ASan and under TSan. Reports land in profiles/sanitizer_<kind>_r03.log.
#   bash scripts/sanitize.sh [address|thread ...]
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
ROOT=$PWD
RT=$(ls /opt/rocm/llvm/lib/clang/*/lib/linux/ | head -0; ls -d /opt/rocm/llvm/lib/clang/*/lib/linux | head -1)
kinds=${*:-address thread}
for k in $kinds; do
  python -m mpit_amd._build -j 8 --sanitize $k > /dev/null || exit 1
  so=$ROOT/build/san_$k/_mpit$(python -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
  if [ $k = address ]; then pre=$RT/libclang_rt.asan-x86_64.so; else pre=$RT/libclang_rt.tsan-x86_64.so; fi
  logd=/tmp/mpit_san_$k; rm -rf $logd; mkdir -p $logd
  export MPIT_CPU_ONLY=1 MPIT_NATIVE_SO=$so PYTHONPATH=$ROOT
  export ASAN_OPTIONS="detect_leaks=0:log_path=$logd/asan:abort_on_error=0"
  export TSAN_OPTIONS="suppressions=$ROOT/scripts/tsan.supp:log_path=$logd/tsan:halt_on_error=0:report_signal_unsafe=0:second_deadlock_stack=1"
  out=$ROOT/profiles/sanitizer_${k}_r03.log
  echo "# $k sanitizer run $(date -u +%FT%TZ), module $so" > $out
  run() {  # name nranks script [env...]
    local name=$1 n=$2 script=$3; shift 3
    local port=$((29700 + RANDOM % 200))
    env "$@" LD_PRELOAD=$pre timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $port tests/mp/$script > $logd/$name.out 2>&1
    local rc=$?
    echo "$name: ranks=$n rc=$rc $(grep -cE '^OK |RESULT' $logd/$name.out) result lines" >> $out
  }
  run api_suite3 3 api_suite.py
  run api_suite2_dist 2 api_suite.py MPIT_DIST_HOST=1
  run ps_colocated3 3 ps_train.py
  run ps_dedicated3 3 ps_train.py T_TOPO=dedicated
  run ps_eamsgd2 2 ps_train.py T_OPT=eamsgd
  run ps_su2 2 ps_train.py T_SU=2
  run ssp3 3 ssp_check.py
  run ps_split2 2 ps_train.py T_SPS=3
  nrep=$(cat $logd/asan.* $logd/tsan.* 2>/dev/null | grep -cE "ERROR: AddressSanitizer|WARNING: ThreadSanitizer")
  echo "reports: $nrep" >> $out
  for f in $logd/asan.* $logd/tsan.*; do
    [ -f "$f" ] || continue
    echo "---- $(basename $f)" >> $out
    head -80 "$f" >> $out
  done
  cat $out
done
