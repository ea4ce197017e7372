#!/bin/bash
# HEAD: full GPU suite + smoke, then the default bench
TAG=${1:-r03u}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/gpu_r03p.sh $TAG || exit $?
timeout -k 10 600 python -u bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err
rc=$?; tail -c 1500 $OUT/${TAG}_bench.json; echo "== bench rc=$rc"
exit $rc
