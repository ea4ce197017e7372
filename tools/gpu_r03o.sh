#!/bin/bash
# b2 768 threads (3 waves/SIMD, one VGPR spill) vs 512 (2 waves, no spill)
export TMPDIR=/tmp
BENCH_ARGS="--n 125000000 --d 64 --k 1000 --only-headline" timeout -k 10 1000 bash tools/ab_libs.sh r03o main sb512
echo "== done rc=$?"
