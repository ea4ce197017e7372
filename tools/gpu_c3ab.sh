# C3 A/B of library variants (dislib_amd/libdkm_<v>.so; main = libdkm.so):
# the sorted-image / full-size GPU tests on the main library, then the C3
# bench line per variant, two rounds interleaved.
# usage: bash tools/gpu_c3ab.sh TAG v1 v2 ...
set -o pipefail
TAG=$1; shift
PT="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -q"
timeout -k 10 600 $PT tests/test_gpu_sorted.py tests/test_gpu_b2.py tests/test_gpu_fullsize.py::test_c3_full_size_labels > gpurun_out/${TAG}_c3tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_c3tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for r in 1 2; do for v in "$@"; do
  lib=$PWD/dislib_amd/libdkm_$v.so; [ $v = main ] && lib=$PWD/dislib_amd/libdkm.so
  DKM_LIB=$lib timeout -k 10 300 python bench.py --n 125000000 --d 64 --k 1000 --steps 8 --warmup 2 --no-cpu --only-headline > gpurun_out/${TAG}_$v$r.json 2>/dev/null || { echo "$v failed"; exit 1; }
  python -c "import json;d=json.loads([l for l in open('gpurun_out/${TAG}_$v$r.json') if l.startswith('{')][-1]);print('$v', round(d['ms_per_step'],3), 'fit', round(d['fit_ms_per_iter'],2), 'rech', d['rechecked_samples'])"
done; done
