#!/bin/bash
# C4 (10M x 1024, k = 4096): GEMM-screen parity tests, then the bench line
# under rocprofv3 kernel stats.  usage: gpu_c4.sh TAG
TAG=${1:-r02}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 $lim "$@" > $OUT/${TAG}_${name}.log 2>&1
  local rc=$?
  tail -3 $OUT/${TAG}_${name}.log | cut -c1-1500
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
step c4test 400 python -u -m pytest tests/test_gpu_gemm.py -v -p no:cacheprovider -x --timeout 300 --timeout-method thread
step c4prof 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/${TAG}_c4prof -o run -- python3 bench.py --n 10000000 --d 1024 --k 4096 --steps 5 --warmup 3 --no-cpu --only-headline
echo "== done"
