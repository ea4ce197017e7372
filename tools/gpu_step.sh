#!/bin/bash
# One gpurun session of named steps; each GPU step has its own time limit
# and a crash / timeout / fault (anything but exit 0 or 1) stops the
# session so nothing more touches the GPU.
# usage: bash tools/gpu_step.sh TAG STEP...   (steps: see the case below)
TAG=${1:-r04}; shift
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 $lim "$@" > $OUT/${TAG}_${name}.log 2>&1
  local rc=$?
  tail -4 $OUT/${TAG}_${name}.log
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
PT="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -v"
for s in "$@"; do
  case $s in
    t_new) step t_new 600 $PT tests/test_gpu_sorted.py tests/test_gpu_b2.py tests/test_gpu_nonfinite.py tests/test_gpu_fullsize.py ;;
    t_sorted) step t_sorted 300 $PT tests/test_gpu_sorted.py ;;
    c3fab) for r in 1 2; do for v in 0 1; do
        DKM_FUSED_SORT_SUMS=$v step c3f$v$r 300 python bench.py --n 125000000 --d 64 --k 1000 --steps 8 --warmup 2 --no-cpu --only-headline
        python -c "import json,sys;d=json.loads([l for l in open('$OUT/${TAG}_c3f$v$r.log') if l.startswith('{')][-1]);print('fused=$v', round(d['ms_per_step'],3), 'fit', round(d['fit_ms_per_iter'],2), d.get('fit_iters'))"
      done; done ;;
    t_gemm) step t_gemm 600 $PT tests/test_gpu_gemm.py ;;
    t_nb) step t_nb 600 $PT tests/test_gpu_neighbors.py ;;
    t_c5) step t_c5 600 $PT tests/test_gpu_fullsize.py -k c5 ;;
    t_all) step t_all 900 $PT -m gpu tests ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py --steps 20 --warmup 3 ;;
    benchprof) P=$OUT/${TAG}_benchprof; mkdir -p $P
      step benchprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o run -- python bench.py --steps 20 --warmup 3 --no-cpu
      find $P -type f ! -name '*kernel_stats.csv' -delete 2>/dev/null; find $P -name '*kernel_stats.csv' | head -2 ;;
    c3) step c3 300 python bench.py --n 125000000 --d 64 --k 1000 --steps 8 --warmup 2 --no-cpu --only-headline ;;
    c3prof) P=$OUT/${TAG}_c3it; mkdir -p $P
      step c3prof 300 rocprofv3 --kernel-trace --stats -d $P -o run -- python bench.py --n 125000000 --d 64 --k 1000 --steps 8 --warmup 2 --no-cpu --only-headline
      DB=$(find $P -name '*.db' | head -1)
      [ -n "$DB" ] && python tools/prof_iters.py $DB > $P/iters.txt 2>&1 && rm -f $DB
      cut -c1-300 $P/iters.txt ;;
    c3ns) DKM_SORTED_IMAGE=0 step c3ns 300 python bench.py --n 125000000 --d 64 --k 1000 --steps 8 --warmup 2 --no-cpu --only-headline ;;
    c4) step c4 300 python bench.py --n 10000000 --d 1024 --k 4096 --steps 4 --warmup 2 --no-cpu --only-headline ;;
    c4it) P=$OUT/${TAG}_c4it; mkdir -p $P
      step c4it 300 rocprofv3 --kernel-trace --stats -d $P -o run -- python bench.py --n 10000000 --d 1024 --k 4096 --steps 4 --warmup 2 --no-cpu --only-headline
      DB=$(find $P -name '*.db' | head -1)
      [ -n "$DB" ] && python tools/prof_iters.py $DB > $P/iters.txt 2>&1 && rm -f $DB
      cut -c1-400 $P/iters.txt ;;
    c4prof) step c4prof 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/${TAG}_c4prof -o run -- python bench.py --n 10000000 --d 1024 --k 4096 --steps 4 --warmup 2 --no-cpu --only-headline ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done"
