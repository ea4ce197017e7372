#!/bin/bash
# Counter passes (rocprofv3 --pmc, kernel-trace only; never with sys/runtime
# traces).  usage: bash tools/pmc_session.sh TAG TARGET
#   TARGET = bench        -> bench.py on 20M rows (steady-state delta steps)
#   TARGET = csr          -> tools/bench_csr.py (C5 CSR rows) on N rows
#   TARGET = <mode list>  -> tools/bench_modes.py --modes <list> on 20M rows
TAG=${1:-r01}; TARGET=${2:-bench}; shift 2
OUT=gpurun_out/${TAG}_pmc; mkdir -p $OUT; export TMPDIR=/tmp
N=${PMC_N:-20000000}
if [ "$TARGET" = bench ]; then
  PROG=(python bench.py --n $N --steps 8 --warmup 4 --no-cpu --only-headline $BENCH_ARGS)
elif [ "$TARGET" = csr ]; then
  PROG=(python tools/bench_csr.py --n $N --steps 4 $BENCH_ARGS)
else
  PROG=(python tools/bench_modes.py --n $N --rounds 2 --modes $TARGET)
fi
run() {  # name counters...
  local name=$1; shift
  echo "== pmc $name: $*"
  timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv \
     -d $OUT/$name -o run -- "${PROG[@]}" > $OUT/$name.log 2>&1
  local rc=$?; echo "== rc=$rc"; tail -2 $OUT/$name.log
  # keep only the counter tables (the pull-back is capped at 64 MiB)
  find $OUT/$name -type f ! -name '*counter_collection.csv' -delete 2>/dev/null
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo STOP; exit $rc; fi
}
run p1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
run p2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT
run p3 FETCH_SIZE
run p3b WRITE_SIZE
run p4 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES
run p5 TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum
python tools/pmc_summary.py $OUT --n $N ${PMC_SUMMARY_ARGS} --traffic-out $OUT/traffic.json \
  > $OUT/summary.txt 2>&1
echo "== done"
