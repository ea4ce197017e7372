#!/bin/bash
# b2 wave stagger A/B (image path)
export TMPDIR=/tmp
BENCH_ARGS="--n 125000000 --d 64 --k 1000 --only-headline" timeout -k 10 1000 bash tools/ab_libs.sh r03n main st60 st120
echo "== done rc=$?"
