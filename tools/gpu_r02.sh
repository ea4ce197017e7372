#!/bin/bash
# Round-2 GPU session: GPU tests -> smoke -> bench -> rocprofv3 kernel stats
# of the bench.  Each GPU step runs under its own limit; anything other than
# exit 0/1 stops the session.   usage: bash tools/gpu_r02.sh TAG [steps...]
#   steps: any of  test smoke bench prof   (default: all four)
TAG=${1:-r02}; shift
STEPS=${*:-test smoke bench prof}
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 $lim "$@" > $OUT/${TAG}_${name}.log 2>&1
  local rc=$?
  tail -4 $OUT/${TAG}_${name}.log | cut -c1-800
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
for s in $STEPS; do case $s in
  test)  step pytest 700 python -u -m pytest tests -m gpu -v -p no:cacheprovider --maxfail=10 --timeout 200 --timeout-method thread ;;
  smoke) step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" ;;
  bench) step bench 500 python bench.py ;;
  prof)  step prof 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu ;;
esac; done
echo "== done"
