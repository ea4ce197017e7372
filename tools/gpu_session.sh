#!/bin/bash
# One gpurun session: GPU tests -> smoke -> residency check -> A/B library
# variants -> bench -> rocprofv3 kernel stats.  Each GPU step has its own
# time limit; a crash/timeout/fault (anything other than exit 0/1) stops the
# session so nothing more touches the GPU.
# usage: bash tools/gpu_session.sh TAG [variant ...]
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
step pytest 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --maxfail=10 --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
# (resident-block sizing: build a -DDKM_AB_VERBOSE variant with variants.sh)
if [ $# -gt 0 ]; then
  bash tools/ab_libs.sh $TAG main "$@" || exit $?
fi
step bench 400 python bench.py --steps 20 --warmup 3
step prof 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/${TAG}_prof -o run -- python bench.py --steps 10 --warmup 2 --no-cpu
echo "== done"
