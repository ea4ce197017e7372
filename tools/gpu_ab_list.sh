bash tools/gpu_ab_s1.sh r01s6 main nospread main || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/r01s6_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r01s6_pytest.log; exit $rc
