#!/bin/bash
# w32 whole-line loads + b2 producer/consumer: parity, C2 stats, C3 PC vs not
TAG=${1:-r03g}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
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
C2="--steps 20 --warmup 3 --no-cpu --only-headline"
step b2test 600 python -u -m pytest tests/test_gpu_b2.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
step c3_pc 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_c3_pc -o run -- python3 bench.py $C3
export DKM_B2_PC=0
step c3_nopc 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_c3_nopc -o run -- python3 bench.py $C3
unset DKM_B2_PC
step c2_main 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_c2_main -o run -- python3 bench.py $C2
step parity 900 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
echo "== done"
