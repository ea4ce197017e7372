#!/bin/bash
# neighbours tests (sparse grid case fixed), smoke, default bench, C3
# per-iteration breakdown, neighbours bench
TAG=${1:-r03w}; OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_neighbors.py -v -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/${TAG}_nb.log 2>&1
rc=$?; tail -2 $OUT/${TAG}_nb.log; echo "== neighbors rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/${TAG}_smoke.log 2>&1
rc=$?; tail -2 $OUT/${TAG}_smoke.log; echo "== smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err
rc=$?; tail -c 600 $OUT/${TAG}_bench.json; echo "== bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
P=$OUT/${TAG}_c3it; mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P -o run -- python bench.py --n 125000000 --d 64 --k 1000 --steps 8 --warmup 2 --no-cpu --only-headline > $P/bench.log 2>&1
rc=$?; echo "== c3 prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
DB=$(find $P -name '*.db' | head -1); echo "db=$DB"
[ -n "$DB" ] && python tools/prof_iters.py $DB > $P/iters.txt 2>&1; cut -c1-300 $P/iters.txt
rm -f $DB
timeout -k 10 240 python -u tools/bench_neighbors.py > $OUT/${TAG}_neighbors.json 2> $OUT/${TAG}_neighbors.err
rc=$?; echo "== neighbors bench rc=$rc"; cut -c1-600 $OUT/${TAG}_neighbors.json
exit $rc
