#!/bin/bash
# Round 3: k_screen_b2 parity (both variants), C3 kernel stats b2 vs b1,
# PMC of both at 20M rows.  usage: bash tools/gpu_r03b.sh TAG
TAG=${1:-r03b}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 $lim "$@" > $OUT/${TAG}_${name}.log 2>&1
  local rc=$?
  tail -4 $OUT/${TAG}_${name}.log | cut -c1-1500
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
C3="--n 125000000 --d 64 --k 1000 --steps 10 --warmup 2 --no-cpu --only-headline"
step b2test 600 python -u -m pytest tests/test_gpu_b2.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
step c3b2 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/${TAG}_c3b2 -o run -- python3 bench.py $C3
export DKM_B1_LEGACY=1
step c3b1 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/${TAG}_c3b1 -o run -- python3 bench.py $C3
unset DKM_B1_LEGACY
BENCH_ARGS="--d 64 --k 1000" PMC_N=20000000 bash tools/pmc_session_sq.sh ${TAG}b2
echo "== done"
