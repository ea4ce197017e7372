#!/bin/bash
# final HEAD: sparse epsilon-query bench at eps 1.5, then the full GPU suite + smoke
TAG=${1:-r03x}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 240 python -u tools/bench_neighbors.py > $OUT/${TAG}_neighbors.json 2> $OUT/${TAG}_neighbors.err
rc=$?; echo "== neighbors bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_r03p.sh $TAG
