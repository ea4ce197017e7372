#!/bin/bash
# CSR path on the GPU: parity tests, then the C5 bench line and its kernel
# stats.   usage: bash tools/gpu_csr.sh TAG
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
step csrtest 500 python -u -m pytest tests/test_gpu_parity.py -k "csr or sparse" tests/test_gpu_loaders.py tests/test_gpu_fullsize.py -k "csr or sparse or c5" -v -p no:cacheprovider -x --timeout 200 --timeout-method thread
step c5 300 python tools/bench_csr.py --n 10000000 --d 10000 --nnz 10 --k 256 --steps 5
step c5prof 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/${TAG}_c5prof -o run -- python3 tools/bench_csr.py --n 10000000 --d 10000 --nnz 10 --k 256 --steps 5
echo "== done"
