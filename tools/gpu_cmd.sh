set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gemm.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/g12.log 2>&1
rc=$?; tail -3 gpurun_out/g12.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g12 -o run -- python3 bench.py --n 125000000 --d 64 --k 1000 --steps 9 --warmup 1 --no-cpu --only-headline > gpurun_out/g12b.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g12c4 -o run -- python3 bench.py --n 10000000 --d 1024 --k 4096 --steps 5 --warmup 1 --no-cpu --only-headline > gpurun_out/g12c.log 2>&1
