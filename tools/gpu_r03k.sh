#!/bin/bash
# compensated state + REFRESH 64: tests, C3 trace, C3 PMC (b2 image path)
TAG=${1:-r03k}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 $lim "$@" > $OUT/${TAG}_${name}.log 2>&1
  local rc=$?
  tail -3 $OUT/${TAG}_${name}.log | cut -c1-600
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
step tests 600 python -u -m pytest tests/test_gpu_state.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
step c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_c3 -o run -- python3 bench.py --n 125000000 --d 64 --k 1000 --steps 8 --warmup 2 --no-cpu --only-headline
PMC_SUMMARY_ARGS="--d 64 --k 1000" BENCH_ARGS="--d 64 --k 1000" PMC_N=125000000 timeout -k 10 900 bash tools/pmc_session.sh ${TAG}_c3 bench > $OUT/${TAG}_pmc.log 2>&1
echo "== pmc rc=$?"; tail -5 $OUT/${TAG}_pmc.log
echo "== done"
