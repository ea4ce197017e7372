export TMPDIR=/tmp; P=gpurun_out/r04c4f; mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P -o run -- python tools/c4_f32_run.py > $P/log.txt 2>&1 || { echo failed; tail -5 $P/log.txt; exit 1; }
DB=$(find $P -name '*.db' | head -1)
[ -n "$DB" ] && python tools/prof_iters.py $DB > $P/iters.txt 2>&1 && rm -f $DB
cut -c1-420 $P/iters.txt; grep '^{' $P/log.txt | cut -c1-300
