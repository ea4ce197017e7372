#!/bin/bash
# sparse epsilon-query bench at eps 1.5 + the neighbours tests at HEAD
TAG=${1:-r03y}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_neighbors.py tests/test_gpu_b2.py -q -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/${TAG}_nb.log 2>&1
rc=$?; tail -1 $OUT/${TAG}_nb.log; echo "== tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u tools/bench_neighbors.py --no-cpu > $OUT/${TAG}_neighbors.json 2> $OUT/${TAG}_neighbors.err
rc=$?; echo "== neighbors bench rc=$rc"; exit $rc
