#!/bin/bash
# dist CSR case + smoke, then the default bench (headline + extras + CPU)
TAG=${1:-r03q}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -v -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/${TAG}_dist.log 2>&1
rc=$?; tail -2 $OUT/${TAG}_dist.log; echo "== dist rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/${TAG}_smoke.log 2>&1
rc=$?; tail -2 $OUT/${TAG}_smoke.log; echo "== smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err
rc=$?; tail -3 $OUT/${TAG}_bench.err; echo "== bench rc=$rc"; exit $rc
