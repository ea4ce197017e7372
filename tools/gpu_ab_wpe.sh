#!/bin/bash
# A/B: k_screen_w32 occupancy (waves/EU 3 vs 4) x delta sums in the screen's
# LDS vs in k_label_sums (DKM_DELTA_POST).  usage: bash tools/gpu_ab_wpe.sh TAG
TAG=${1:-r01}; OUT=gpurun_out/${TAG}_ab; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2; do
  for v in main wpe4; do
    for post in 0 1; do
      lib=$PWD/dislib_amd/libdkm_$v.so; [ "$v" = main ] && lib=$PWD/dislib_amd/libdkm.so
      if [ $post = 1 ]; then export DKM_DELTA_POST=1; else unset DKM_DELTA_POST; fi
      DKM_LIB=$lib timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu \
        > $OUT/${v}_p${post}_$r.json 2> $OUT/${v}_p${post}_$r.err
      rc=$?
      python3 -c "import json; d=json.load(open('$OUT/${v}_p${post}_$r.json')); print('$v post$post r$r', 'kernel_ms %.3f'%d['roofline']['kernel_ms'], 'ms/step %.3f'%d['ms_per_step'])" || { echo "$v failed rc=$rc"; tail -5 $OUT/${v}_p${post}_$r.err; }
      if [ $rc -ne 0 ]; then echo STOP; exit $rc; fi
    done
  done
done
unset DKM_DELTA_POST
