set -o pipefail
export TMPDIR=/tmp
BENCH_ARGS="--d 64 --k 1000" PMC_N=20000000 bash tools/pmc_session.sh r03a bench && \
timeout -k 10 300 python tools/b1_stats.py --n 125000000 --iters 12 > gpurun_out/r03a_b1stats.txt 2>&1
