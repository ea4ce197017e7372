#!/bin/bash
# HBM traffic PMC (FETCH_SIZE / WRITE_SIZE) of the image paths: C2 and C3
export TMPDIR=/tmp
for cfg in "c2 20000000 32 100" "c3 125000000 64 1000" "c4 2000000 1024 4096"; do
  set -- $cfg
  TAG=r03s_$1; N=$2; D=$3; K=$4; OUT=gpurun_out/${TAG}_pmc; mkdir -p $OUT
  PROG=(python bench.py --n $N --d $D --k $K --steps 8 --warmup 4 --no-cpu --only-headline)
  for pass in "p3 FETCH_SIZE" "p3b WRITE_SIZE" "p1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "p2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT"; do
    set -- $pass; name=$1; shift
    echo "== $TAG $name $*"
    timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$name -o run -- "${PROG[@]}" > $OUT/$name.log 2>&1
    rc=$?; echo "== rc=$rc"; tail -1 $OUT/$name.log | cut -c1-200
    if [ $rc -ne 0 ]; then echo STOP; exit $rc; fi
  done
  python tools/pmc_summary.py $OUT --n $N --d $D --k $K --traffic-out $OUT/traffic.json > $OUT/summary.txt 2>&1
  cat $OUT/traffic.json
done
echo "== done"
