#!/bin/bash
# b2 optimisations: parity, C3 kernel stats of main / legacy b1 / variants,
# streaming-read microbenchmark.  usage: bash tools/gpu_r03c.sh TAG
TAG=${1:-r03c}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 $lim "$@" > $OUT/${TAG}_${name}.log 2>&1
  local rc=$?
  tail -3 $OUT/${TAG}_${name}.log | cut -c1-600
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
C3="--n 125000000 --d 64 --k 1000 --steps 6 --warmup 2 --no-cpu --only-headline"
step b2test 600 python -u -m pytest tests/test_gpu_b2.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
step membench32 120 ./tools/membench 100000000 32
step membench64 120 ./tools/membench 62500000 64
for v in main sb1024 pf512; do
  lib=$PWD/dislib_amd/libdkm_$v.so; [ $v = main ] && lib=$PWD/dislib_amd/libdkm.so
  export DKM_LIB=$lib
  step c3_$v 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_c3_$v -o run -- python3 bench.py $C3
done
unset DKM_LIB
export DKM_B1_LEGACY=1
step c3_b1 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_c3_b1 -o run -- python3 bench.py $C3
echo "== done"
