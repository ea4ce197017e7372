#!/bin/bash
# full GPU suite + smoke at HEAD
TAG=${1:-r03p}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/${TAG}_gpu.log 2>&1
rc=$?; tail -3 $OUT/${TAG}_gpu.log; echo "== gpu rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/${TAG}_smoke.log 2>&1
rc=$?; tail -2 $OUT/${TAG}_smoke.log; echo "== smoke rc=$rc"
exit $rc
