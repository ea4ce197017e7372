# C4 fp32 line per library variant (libdkm_<v>.so; main = libdkm.so), two
# rounds interleaved, after the fp32 parity / full-size tests on main.
TAG=$1; shift
timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -q tests/test_gpu_fullsize.py::test_c4_fp32_full_size_labels tests/test_gpu_parity.py -k "f32 or fp32" > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/${TAG}_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for r in 1 2; do for v in "$@"; do
  lib=$PWD/dislib_amd/libdkm_$v.so; [ $v = main ] && lib=$PWD/dislib_amd/libdkm.so
  DKM_LIB=$lib timeout -k 10 300 python tools/c4_f32_run.py > gpurun_out/${TAG}_$v$r.json 2>/dev/null || { echo "$v failed"; exit 1; }
  python -c "import json;d=json.loads([l for l in open('gpurun_out/${TAG}_$v$r.json') if l.startswith('{')][-1]);print('$v', 'step', round(d['el']/4*1e3,2), 'kern', round(d['kern_ms'],2), 'fit', round(d['fit_s']/d['fit_iters']*1e3,1))"
done; done
