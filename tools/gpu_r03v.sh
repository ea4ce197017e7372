#!/bin/bash
# HEAD suite + smoke + default bench (gpu_r03u.sh), then a per-iteration
# kernel breakdown of a whole C3 fit (iteration 0 / 1 vs steady state)
TAG=${1:-r03v}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/gpu_r03u.sh $TAG || exit $?
P=$OUT/${TAG}_c3it; mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P -o run -- python bench.py --n 125000000 --d 64 --k 1000 --steps 8 --warmup 2 --no-cpu --only-headline > $P/bench.log 2>&1
rc=$?; echo "== c3 prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
DB=$(find $P -name '*.db' | head -1); echo "db=$DB"
[ -n "$DB" ] && python tools/prof_iters.py $DB > $P/iters.txt 2>&1; cat $P/iters.txt | cut -c1-300
rm -f $DB
timeout -k 10 240 python -u tools/bench_neighbors.py > $OUT/${TAG}_neighbors.json 2> $OUT/${TAG}_neighbors.err
rc=$?; echo "== neighbors rc=$rc"; cut -c1-600 $OUT/${TAG}_neighbors.json
exit $rc
