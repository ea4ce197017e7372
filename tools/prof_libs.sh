#!/bin/bash
# Per-kernel times (rocprofv3 --kernel-trace --stats) of library variants
# dislib_amd/libdkm_<v>.so on the bench workload.
# usage: bash tools/prof_libs.sh TAG v1 v2 ...   (extra bench args: $BENCH_ARGS)
TAG=$1; shift
OUT=gpurun_out/${TAG}_prof; mkdir -p $OUT; export TMPDIR=/tmp
for v in "$@"; do
  lib=$PWD/dislib_amd/libdkm_$v.so
  [ "$v" = main ] && lib=$PWD/dislib_amd/libdkm.so
  DKM_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/$v -o run -- python bench.py --steps 8 \
    --warmup 2 --no-cpu $BENCH_ARGS > $OUT/$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"
  grep -h -E '"k_(screen|recheck)' $OUT/$v/run_kernel_stats.csv | cut -d, -f1-4
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo STOP; exit $rc; fi
done
