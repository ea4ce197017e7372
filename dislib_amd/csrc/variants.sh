#!/bin/bash
# Build A/B variants of libdkm.so (screen-kernel compile-time knobs) next to
# the default library: ../libdkm_<name>.so.  usage: bash variants.sh name "DEFS" ...
# A/B switches are compile-time only (-DDKM_AB_NO_W32=1, -DDKM_AB_DELTA_POST=1,
# -DDKM_AB_NO_POST=1, -DDKM_AB_NO_LIST=1, -DDKM_AB_CSR_OLD=1,
# -DDKM_AB_BLOCKS_PER_CU=n, -DDKM_AB_VERBOSE, -DDKM_AB_SBB=n (k_screen_b1
# block size), -DDKM_AB_B1_PREFETCH=1 (k_screen_b1 next-tile prefetch)): the
# product build reads no
# environment variable.
set -e
cd "$(dirname "$0")"
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  d=build_$name; mkdir -p $d
  for f in dkm_util dkm_dense dkm_b2 dkm_sparse dkm_gemm dkm_sums dkm_neighbors; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
      -fno-slp-vectorize $defs -c $f.hip -o $d/$f.o &
  done
  g++ -O3 -std=c++17 -fPIC -pthread -c dkm_io.cpp -o $d/dkm_io.o &
  /opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -c dkm_comm.cpp -o $d/dkm_comm.o &
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -pthread -o ../libdkm_$name.so $d/*.o -ldl
  echo built ../libdkm_$name.so
done
