#!/bin/bash
# A/B environment settings of the default library on the bench workload,
# one process per setting, two rounds interleaved.
# usage: bash tools/ab_env.sh TAG "ENV=.. ENV2=.." "ENV=.." ...  (label = index)
TAG=$1; shift
OUT=gpurun_out/${TAG}_abenv; mkdir -p $OUT
for r in 1 2; do
  i=0
  for e in "$@"; do
    env $e timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu \
      $BENCH_ARGS > $OUT/v${i}_$r.json 2> $OUT/v${i}_$r.err
    rc=$?
    python3 -c "import json; d=json.load(open('$OUT/v${i}_$r.json')); print('[$e] r$r', 'kernel_ms %.3f'%d['roofline']['kernel_ms'], 'ms/step %.3f'%d['ms_per_step'], 'rechecked', d['rechecked_samples'])" || { echo "[$e] failed rc=$rc"; tail -5 $OUT/v${i}_$r.err; }
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo STOP; exit $rc; fi
    i=$((i+1))
  done
done
