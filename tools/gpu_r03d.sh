#!/bin/bash
# coalesced-load b2: parity, membench (whole-line pattern), C3 kernel stats
TAG=${1:-r03d}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 $lim "$@" > $OUT/${TAG}_${name}.log 2>&1
  local rc=$?
  tail -6 $OUT/${TAG}_${name}.log | cut -c1-600
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
C3="--n 125000000 --d 64 --k 1000 --steps 6 --warmup 2 --no-cpu --only-headline"
step b2test 600 python -u -m pytest tests/test_gpu_b2.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
step membench32 120 ./tools/membench 100000000 32
step membench64 120 ./tools/membench 62500000 64
step c3_main 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_c3_main -o run -- python3 bench.py $C3
echo "== done"
