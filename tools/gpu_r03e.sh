#!/bin/bash
# b2 pipelined loop: parity, C3 kernel stats of main and timing probes
TAG=${1:-r03e}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 $lim "$@" > $OUT/${TAG}_${name}.log 2>&1
  local rc=$?
  tail -3 $OUT/${TAG}_${name}.log | cut -c1-400
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
C3="--n 125000000 --d 64 --k 1000 --steps 6 --warmup 2 --no-cpu --only-headline"
step b2test 600 python -u -m pytest tests/test_gpu_b2.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
for v in main p1 p2; do
  lib=$PWD/dislib_amd/libdkm_$v.so; [ $v = main ] && lib=$PWD/dislib_amd/libdkm.so
  export DKM_LIB=$lib
  step c3_$v 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_c3_$v -o run -- python3 bench.py $C3
done
echo "== done"
