#!/bin/bash
# A/B of library variants with per-launch kernel times from rocprofv3
# (steady-state k_recheck_list / k_screen_w32).  usage: bash tools/gpu_ab_s1.sh TAG v...
TAG=$1; shift; OUT=gpurun_out/${TAG}_ab; mkdir -p $OUT; export TMPDIR=/tmp
for v in "$@"; do
  lib=$PWD/dislib_amd/libdkm_$v.so; [ "$v" = main ] && lib=$PWD/dislib_amd/libdkm.so
  DKM_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -T --output-format csv \
    -d $OUT/$v -o run -- python bench.py --steps 12 --warmup 2 --no-cpu > $OUT/$v.log 2>&1
  rc=$?
  python3 tools/trace_summary.py $OUT/$v/run_kernel_trace.csv "$v" || echo "$v summary failed rc=$rc"
  if [ $rc -ne 0 ]; then echo STOP; tail -5 $OUT/$v.log; exit $rc; fi
done
