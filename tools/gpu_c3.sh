#!/bin/bash
# C3 shard (125M x 64, k = 1000): parity tests of the single-product path,
# then the bench line under rocprofv3 kernel stats.  usage: gpu_c3.sh TAG
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
step c3test 300 python -u -m pytest tests/test_gpu_parity.py -k "1000 or c3 or stress" -v -p no:cacheprovider -x --timeout 200 --timeout-method thread
step c3prof 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/${TAG}_c3prof -o run -- python3 bench.py --n 125000000 --d 64 --k 1000 --steps 10 --warmup 2 --no-cpu --only-headline
echo "== done"
