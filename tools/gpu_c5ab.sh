# C5 A/B of library variants (dislib_amd/libdkm_<v>.so; main = libdkm.so):
# CSR parity tests on the main library, then tools/bench_csr.py per variant,
# two rounds interleaved.  usage: bash tools/gpu_c5ab.sh TAG v1 v2 ...
set -o pipefail
TAG=$1; shift
PT="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -q"
timeout -k 10 400 $PT tests/test_gpu_parity.py -k "csr or f07" tests/test_gpu_nonfinite.py -k "sparse or csr" > gpurun_out/${TAG}_csrtests.log 2>&1; echo "tests rc=$?"; tail -1 gpurun_out/${TAG}_csrtests.log
for r in 1 2; do for v in "$@"; do
  lib=$PWD/dislib_amd/libdkm_$v.so; [ $v = main ] && lib=$PWD/dislib_amd/libdkm.so
  DKM_LIB=$lib timeout -k 10 200 python tools/bench_csr.py --steps 5 > gpurun_out/${TAG}_$v$r.json 2>/dev/null || { echo "$v failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$v$r.json'));print('$v', round(d['ms_per_step'],2), 'full', round(d['full_sums_iteration_ms'],1), 'pred', round(d['predict_ms'],2), 'rech', d['rechecked_total'])"
done; done
