#!/bin/bash
# Round-5 GPU session steps (each GPU step under its own time limit; a
# crash / timeout / fault stops the session).  usage: gpu_r05.sh TAG STEP...
#   t_sorted  sorted-image / b2 / C3 full-size label tests
#   t_all     the whole GPU suite
#   diag      tools/c3_diag.py on the main library (and libdkm_old.so when built:
#             bash dislib_amd/csrc/variants_b2.sh old -DDKM_AB_NO_SORTED_FAST=1 dkm_b2)
#   c3it      C3 bench line under a rocprofv3 kernel trace, per iteration
#   c4it      C4 bench line under a rocprofv3 kernel trace, per iteration
#   c3ab      C3 bench line, main vs libdkm_$AB.so (default old), two rounds
#   c2ab      C2 headline line, main vs libdkm_$AB.so (AB env, default w32pf2), two rounds
#   bench     default bench.py
TAG=${1:-r05}; shift
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 $lim "$@" > $OUT/${TAG}_${name}.log 2>&1
  local rc=$?
  tail -4 $OUT/${TAG}_${name}.log | cut -c1-400
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
PT="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -q"
C3="python bench.py --n 125000000 --d 64 --k 1000 --steps 8 --warmup 2 --no-cpu --only-headline"
C4="python bench.py --n 10000000 --d 1024 --k 4096 --steps 3 --warmup 1 --no-cpu --only-headline"
OLD=$PWD/dislib_amd/libdkm_old.so
for s in "$@"; do
  case $s in
    t_sorted) step t_sorted 900 $PT tests/test_gpu_sorted.py tests/test_gpu_b2.py tests/test_gpu_fullsize.py::test_c3_full_size_labels ;;
    t_all) step t_all 1100 $PT -m gpu tests ;;
    diag) step diag_main 240 python tools/c3_diag.py
          [ -f $OLD ] && DKM_LIB=$OLD step diag_old 240 python tools/c3_diag.py ;;
    c3it) P=$OUT/${TAG}_c3it; mkdir -p $P
      step c3it 300 rocprofv3 --kernel-trace --stats -d $P -o run -- $C3
      DB=$(find $P -name '*.db' | head -1)
      [ -n "$DB" ] && python tools/prof_iters.py $DB > $P/iters.txt 2>&1 && rm -f $DB
      find $P -type f ! -name 'iters.txt' ! -name '*kernel_stats.csv' -delete
      cut -c1-300 $P/iters.txt ;;
    c2it) P=$OUT/${TAG}_c2it; mkdir -p $P
      step c2it 300 rocprofv3 --kernel-trace --stats -d $P -o run -- python bench.py --steps 8 --warmup 2 --no-cpu --only-headline
      DB=$(find $P -name '*.db' | head -1)
      [ -n "$DB" ] && python tools/prof_iters.py $DB > $P/iters.txt 2>&1 && rm -f $DB
      find $P -type f ! -name 'iters.txt' -delete
      cut -c1-300 $P/iters.txt ;;
    c4it) P=$OUT/${TAG}_c4it; mkdir -p $P
      step c4it 400 rocprofv3 --kernel-trace --stats -d $P -o run -- $C4
      DB=$(find $P -name "*.db" | head -1); [ -n "$DB" ] && python tools/prof_iters.py $DB > $P/iters.txt 2>&1 && rm -f $DB; find $P -type f ! -name iters.txt -delete
      cut -c1-400 $P/iters.txt ;;
    c3ab) V=${AB:-old}; for r in 1 2; do for v in main $V; do
        if [ $v = main ]; then unset DKM_LIB; else export DKM_LIB=$PWD/dislib_amd/libdkm_$v.so; fi
        step c3_$v$r 300 $C3
        python -c "import json;d=json.loads([l for l in open('$OUT/${TAG}_c3_$v$r.log') if l.startswith('{')][-1]);print('$v', round(d['ms_per_step'],3), 'fit', round(d['fit_ms_per_iter'],2), 'kern', round(d['roofline']['kernel_ms'],3))"
      done; done; unset DKM_LIB ;;
    c2ab) for r in 1 2; do for v in main ${AB:-w32pf2}; do
        if [ $v = main ]; then unset DKM_LIB; else export DKM_LIB=$PWD/dislib_amd/libdkm_$v.so; fi
        step c2_$v$r 300 python bench.py --steps 20 --warmup 3 --no-cpu --only-headline
        python -c "import json;d=json.loads([l for l in open('$OUT/${TAG}_c2_$v$r.log') if l.startswith('{')][-1]);print('$v', round(d['ms_per_step'],3), 'fit', round(d['fit_ms_per_iter'],2), 'kern', round(d['roofline']['kernel_ms'],3))"
      done; done; unset DKM_LIB ;;
    bench) step bench 900 python bench.py ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done"
