#!/bin/bash
# C4 split/screen overlap, moved-sample sums grid, sort merge: tests + stats
TAG=${1:-r03h}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 $lim "$@" > $OUT/${TAG}_${name}.log 2>&1
  local rc=$?
  tail -3 $OUT/${TAG}_${name}.log | cut -c1-400
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_neighbors.py tests/test_gpu_parity.py tests/test_gpu_b2.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
step c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_c3 -o run -- python3 bench.py --n 125000000 --d 64 --k 1000 --steps 8 --warmup 2 --no-cpu --only-headline
step c4 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_c4 -o run -- python3 bench.py --n 10000000 --d 1024 --k 4096 --steps 4 --warmup 2 --no-cpu --only-headline
echo "== done"
