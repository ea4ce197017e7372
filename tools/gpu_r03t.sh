#!/bin/bash
# kNN > 32 neighbours + traffic PMC of the image paths
TAG=${1:-r03t}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_neighbors.py tests/test_gpu_b2.py -v -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/${TAG}_nb.log 2>&1
rc=$?; tail -2 $OUT/${TAG}_nb.log; echo "== neighbors rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_r03s.sh
