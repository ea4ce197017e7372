#!/bin/bash
# Other BASELINE configs on one GPU (bench lines, not the driver's bench):
#   C3 per-GPU shard: 125M x 64, k = 1000 (chunked screen); exact-mode
#   reference point on 10M rows.  usage: bash tools/gpu_configs.sh TAG
TAG=${1:-r01}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 $lim "$@" > $OUT/${TAG}_${name}.log 2>&1
  local rc=$?
  tail -2 $OUT/${TAG}_${name}.log | cut -c1-600
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
step c3 300 python bench.py --n 125000000 --d 64 --k 1000 --steps 3 --warmup 1 --no-cpu
step c3exact 300 python bench.py --n 10000000 --d 64 --k 1000 --steps 1 --warmup 0 --no-cpu --mode exact
step c3prof 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/${TAG}_c3prof -o run -- python bench.py --n 125000000 --d 64 --k 1000 --steps 2 --warmup 1 --no-cpu
step c5 400 python tools/bench_csr.py --n 10000000 --d 10000 --nnz 10 --k 256 --steps 5
step c4exact 400 python bench.py --n 200000 --d 1024 --k 4096 --steps 1 --warmup 0 --no-cpu
echo "== done"
