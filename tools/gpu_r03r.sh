#!/bin/bash
# split image for k_screen_w32: parity + C2 A/B
TAG=${1:-r03r}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 $lim "$@" > $OUT/${TAG}_${name}.log 2>&1
  local rc=$?
  tail -3 $OUT/${TAG}_${name}.log | cut -c1-600
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
step tests 700 python -u -m pytest tests/test_gpu_image.py tests/test_gpu_b2.py tests/test_gpu_prune.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
step c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_c2 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu --only-headline
export DKM_X_IMAGE=0
step c2noimg 300 python3 bench.py --steps 20 --warmup 3 --no-cpu --only-headline
echo "== done"
