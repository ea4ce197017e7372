# C2 A/B: AUTO's bf16x3 w32 screen vs the single-product screen with the
# label-sorted image (DKM_AB_AUTO_SINGLE=1), two rounds interleaved.
TAG=${1:-r04x}
for r in 1 2; do for v in 0 1; do
  DKM_AB_AUTO_SINGLE=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --only-headline > gpurun_out/${TAG}_c2_$v$r.json 2> gpurun_out/${TAG}_c2_$v$r.err || { echo "v$v failed"; tail -3 gpurun_out/${TAG}_c2_$v$r.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_c2_$v$r.json'));print('single=$v', round(d['ms_per_step'],3), 'fit', round(d['fit_ms_per_iter'],2), 'rech', d['rechecked_samples'], d['roofline'].get('image'))"
done; done
