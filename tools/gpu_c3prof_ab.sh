# Per-iteration kernel traces of the C3 bench line for library variants
# (dislib_amd/libdkm_<v>.so; main = libdkm.so).  usage: TAG v1 v2 ...
TAG=$1; shift; export TMPDIR=/tmp
for v in "$@"; do
  lib=$PWD/dislib_amd/libdkm_$v.so; [ $v = main ] && lib=$PWD/dislib_amd/libdkm.so
  P=gpurun_out/${TAG}_$v; mkdir -p $P
  DKM_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P -o run -- python bench.py --n 125000000 --d 64 --k 1000 --steps 8 --warmup 2 --no-cpu --only-headline > $P/log.txt 2>&1 || { echo "$v failed"; exit 1; }
  DB=$(find $P -name '*.db' | head -1)
  [ -n "$DB" ] && python tools/prof_iters.py $DB > $P/iters.txt 2>&1 && rm -f $DB
  echo "== $v"; tail -3 $P/iters.txt | cut -c1-400
done
