#!/bin/bash
# One gpurun session: GPU tests -> smoke -> bench -> rocprofv3 kernel stats.
# Each GPU step has its own time limit; a crash/timeout/fault (anything other
# than exit 0/1) stops the session so nothing more touches the GPU.
# usage: bash tools/gpu_session.sh TAG [pytest-args...]
TAG=${1:-r01}; shift
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 $lim "$@" > $OUT/${TAG}_${name}.log 2>&1
  local rc=$?
  tail -4 $OUT/${TAG}_${name}.log
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
step pytest 900 python -m pytest tests -m gpu -q -p no:cacheprovider --maxfail=10 "$@"
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step modes 300 python tools/bench_modes.py --rounds 5 --modes screen32,bf16x3
step modes_init 300 python tools/bench_modes.py --rounds 3 --modes screen32,bf16x3 --centres init
step bench 400 python bench.py --steps 20 --warmup 3
step prof 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/${TAG}_prof -o run -- python bench.py --steps 10 --warmup 2 --no-cpu
echo "== done"
