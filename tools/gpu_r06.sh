#!/bin/bash
# Round-6 GPU session steps (each GPU step under its own time limit; a
# crash / timeout / fault stops the session).  usage: gpu_r06.sh TAG STEP...
#   t_new     the tests added this round (world 4, CSR near ties)
#   t_sorted  sorted-image / b2 / C3 full-size label tests
#   t_all     the whole GPU suite
#   smoke     __graft_entry__.smoke()
#   bench     default bench.py (CPU baselines included)
#   prof      rocprofv3 --kernel-trace --stats of bench.py --no-cpu
#   c3it/c2it/c4it  one config's bench line under a kernel trace, per iteration
#   c3ab/c2ab/c4ab one config, main vs libdkm_$AB.so, two rounds
TAG=${1:-r06}; shift
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 $lim "$@" > $OUT/${TAG}_${name}.log 2>&1
  local rc=$?
  tail -4 $OUT/${TAG}_${name}.log | cut -c1-600
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
summ() {  # log -> one line: value, ms/step (whole fit), steady, kernel
  python - "$1" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
def one(e, name):
    rf = e['roofline']
    print(name, 'fit_ms/it', round(e['ms_per_step'], 3), 'steady', round(e['steady_ms_per_step'], 3),
          'kern', round(rf['kernel_ms'], 3), 'steady_kern', round(rf['steady']['kernel_ms'], 3),
          'frac', round(rf['frac'], 3), 'steady_frac', round(rf['steady']['frac'], 3))
    print('   iter_ms', e['iter_ms'])
one(d, 'head')
for e in d.get('extra_configs', []):
    one(e, e['workload'][:24])
PY
}
PT="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -q"
C3="python bench.py --n 125000000 --d 64 --k 1000 --steps 10 --warmup 2 --no-cpu --only-headline"
C4="python bench.py --n 10000000 --d 1024 --k 4096 --steps 5 --warmup 1 --no-cpu --only-headline"
C2="python bench.py --steps 20 --warmup 3 --no-cpu --only-headline"
trace() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  P=$OUT/${TAG}_$name; mkdir -p $P
  step $name $lim rocprofv3 --kernel-trace --stats -f csv rocpd -d $P -o run -- "$@"
  DB=$(find $P -name '*.db' | head -1)
  [ -n "$DB" ] && python tools/prof_iters.py $DB > $P/iters.txt 2>&1 && rm -f $DB
  find $P -type f ! -name 'iters.txt' ! -name '*kernel_stats.csv' -delete
  cut -c1-400 $P/iters.txt
  summ $OUT/${TAG}_$name.log
}
for s in "$@"; do
  case $s in
    t_new) step t_new 900 $PT tests/test_gpu_dist.py tests/test_gpu_parity.py::test_csr_near_ties_at_the_bf16_table_rounding ;;
    t_core) step t_core 900 $PT tests/test_gpu_image.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py::test_c2_full_size_labels tests/test_gpu_fullsize.py::test_c3_full_size_labels ;;
    t_w32) step t_w32 900 $PT tests/test_gpu_image.py tests/test_gpu_nonfinite.py tests/test_gpu_parity.py tests/test_gpu_state.py tests/test_gpu_fullsize.py::test_c2_full_size_labels ;;
    t_sorted) step t_sorted 900 $PT tests/test_gpu_sorted.py tests/test_gpu_b2.py tests/test_gpu_fullsize.py::test_c3_full_size_labels ;;
    t_all) step t_all 1100 $PT -m gpu tests ;;
    diag) step diag 300 python tools/c3_diag.py; cat $OUT/${TAG}_diag.log | cut -c1-300 ;;
    rsdiag) step rsdiag 300 python tools/rescreen_diag.py; cat $OUT/${TAG}_rsdiag.log | cut -c1-300 ;;
    rstrace) trace rstrace 300 python tools/rescreen_diag.py ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py; summ $OUT/${TAG}_bench.log ;;
    prof) trace prof 600 python bench.py --no-cpu ;;
    c3it) trace c3it 300 $C3 ;;
    c2it) trace c2it 300 $C2 ;;
    c4it) trace c4it 400 $C4 ;;
    c3ab|c2ab|c4ab) CMD=$C3; [ $s = c2ab ] && CMD=$C2; [ $s = c4ab ] && CMD=$C4
      for r in 1 2; do for v in main ${AB:-ab}; do
        if [ $v = main ]; then unset DKM_LIB; else export DKM_LIB=$PWD/dislib_amd/libdkm_$v.so; fi
        step ${s}_$v$r 300 $CMD; summ $OUT/${TAG}_${s}_$v$r.log
      done; done; unset DKM_LIB ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
