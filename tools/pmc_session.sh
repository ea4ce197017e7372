#!/bin/bash
# Counter passes (rocprofv3 --pmc, kernel-trace only; never with sys/runtime
# traces) over a short bench_modes run.  usage: bash tools/pmc_session.sh TAG MODE
TAG=${1:-r01}; MODE=${2:-bf16x3}; shift 2
OUT=gpurun_out/${TAG}_pmc; mkdir -p $OUT; export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
run() {  # name counters...
  local name=$1; shift
  echo "== pmc $name: $*"
  timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv \
     -d $OUT/$name -o run -- python tools/bench_modes.py --n 20000000 \
     --rounds 2 --modes $MODE > $OUT/$name.log 2>&1
  local rc=$?; echo "== rc=$rc"; tail -2 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo STOP; exit $rc; fi
}
run p1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
run p2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT
run p3 FETCH_SIZE
run p4 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES
run p5 TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum
echo "== done"
