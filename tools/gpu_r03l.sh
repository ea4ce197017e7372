#!/bin/bash
# b2: VALU dot for s_hat_p, one-asm block test: parity + C3
TAG=${1:-r03l}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 $lim "$@" > $OUT/${TAG}_${name}.log 2>&1
  local rc=$?
  tail -3 $OUT/${TAG}_${name}.log | cut -c1-600
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
step b2test 600 python -u -m pytest tests/test_gpu_b2.py tests/test_gpu_state.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
step c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_c3 -o run -- python3 bench.py --n 125000000 --d 64 --k 1000 --steps 8 --warmup 2 --no-cpu --only-headline
echo "== done"
