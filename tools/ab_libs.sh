#!/bin/bash
# A/B library variants (dislib_amd/libdkm_<v>.so, built by csrc/variants.sh)
# on the bench workload, one process per variant, two rounds interleaved.
# usage: bash tools/ab_libs.sh TAG v1 v2 ...   (extra bench args via $BENCH_ARGS)
TAG=$1; shift
OUT=gpurun_out/${TAG}_ab; mkdir -p $OUT
for r in 1 2; do
  for v in "$@"; do
    lib=$PWD/dislib_amd/libdkm_$v.so; [ "$v" = main ] && lib=$PWD/dislib_amd/libdkm.so
    DKM_LIB=$lib timeout -k 10 240 python bench.py \
      --steps 10 --warmup 3 --no-cpu $BENCH_ARGS > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err
    rc=$?
    python3 -c "import json,sys; d=json.load(open('$OUT/${v}_$r.json')); print('$v r$r', 'kernel_ms %.3f'%d['roofline']['kernel_ms'], 'ms/step %.3f'%d['ms_per_step'], 'rechecked', d['rechecked_samples'])" || { echo "$v failed rc=$rc"; tail -5 $OUT/${v}_$r.err; }
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo STOP; exit $rc; fi
  done
done
