OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_loaders.py tests/test_gpu_gm_init.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/r01s2_pytest_new.log 2>&1; rc=$?; tail -8 $OUT/r01s2_pytest_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_loaders.py --rows 2000000 --ref-rows 100000 --csv-rows 400000 > $OUT/r01s2_loaders.json 2> $OUT/r01s2_loaders.err; rc=$?; cat $OUT/r01s2_loaders.json; tail -3 $OUT/r01s2_loaders.err; exit $rc
