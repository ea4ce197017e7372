#!/bin/bash
# k_gemm_screen1 diagnostic variants (libdkm_g1*.so): kernel time per launch
# under rocprofv3 kernel stats.  usage: gpu_g1ab.sh TAG LIB...
TAG=$1; shift; OUT=gpurun_out/${TAG}_g1ab; mkdir -p $OUT; export TMPDIR=/tmp
for v in "$@"; do
  L=$PWD/dislib_amd/libdkm_$v.so; [ $v = main ] && L=$PWD/dislib_amd/libdkm.so
  DKM_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/$v -o run -- python tools/bench_gemm.py --n 2000000 --mode bf16 --kind predict --reps 3 \
    > $OUT/$v.log 2>&1
  rc=$?; echo "== $v rc=$rc"; grep '^{' $OUT/$v.log | cut -c1-200
  find $OUT/$v -type f ! -name '*kernel_stats.csv' -delete
  python -c "import csv,glob;r=list(csv.DictReader(open(glob.glob('$OUT/$v/**/*kernel_stats.csv',recursive=True)[0])));[print(' ',x['Name'][:40],x['Calls'],round(float(x['AverageNs'])/1e3,1),'us') for x in r[:5]]"
  if [ $rc -ne 0 ]; then echo STOP; exit $rc; fi
done
