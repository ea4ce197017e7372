#!/bin/bash
# A/B of the fit's first iterations at C3 (env knobs), two rounds
OUT=gpurun_out/r04e_ab; mkdir -p $OUT
for r in 1 2; do
for v in base it0single it1hint; do
  case $v in base) E="";; it0single) E="DKM_IT0_MODE=bf16";; it1hint) E="DKM_IT1_HINT=1";; esac
  env $E timeout -k 10 200 python bench.py --n 125000000 --d 64 --k 1000 --steps 8 --warmup 2 --no-cpu --only-headline > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err
  rc=$?
  python3 -c "import json; d=json.load(open('$OUT/${v}_$r.json')); print('$v r$r', 'ms/step %.3f'%d['ms_per_step'], 'fit_ms/iter %.2f'%d['fit_ms_per_iter'])" || tail -3 $OUT/${v}_$r.err
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo STOP; exit $rc; fi
done; done
