# C3 fit with the iteration-0/1 knobs (kmeans.py IT0_MODE / IT1_HINT), then
# a per-iteration trace with idle gaps.  usage: TAG
TAG=$1; export TMPDIR=/tmp
B="python bench.py --n 125000000 --d 64 --k 1000 --steps 8 --warmup 2 --no-cpu --only-headline"
for v in default it0bf16 it1hint; do
  E=""; [ $v = it0bf16 ] && E="DKM_IT0_MODE=bf16"; [ $v = it1hint ] && E="DKM_IT1_HINT=1"
  env $E timeout -k 10 300 $B > gpurun_out/${TAG}_$v.json 2>/dev/null || { echo "$v failed"; exit 1; }
  python -c "import json;d=json.loads([l for l in open('gpurun_out/${TAG}_$v.json') if l.startswith('{')][-1]);print('$v', round(d['ms_per_step'],3), 'fit', round(d['fit_ms_per_iter'],2), 'kern', round(d['roofline']['kernel_ms'],3))"
done
P=gpurun_out/${TAG}_trace; mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P -o run -- $B > $P/log.txt 2>&1 || { echo "trace failed"; exit 1; }
DB=$(find $P -name '*.db' | head -1)
[ -n "$DB" ] && python tools/prof_iters.py $DB > $P/iters.txt 2>&1 && rm -f $DB
cut -c1-300 $P/iters.txt
