#!/bin/bash
# b2 timing probes (image path): main vs no block loop vs loop without tests
export TMPDIR=/tmp
BENCH_ARGS="--n 125000000 --d 64 --k 1000 --only-headline" timeout -k 10 1000 bash tools/ab_libs.sh r03m main b2p1 b2p2
echo "== done rc=$?"
