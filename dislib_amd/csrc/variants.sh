#!/bin/bash
# Build A/B variants of libdkm.so (screen-kernel compile-time knobs) next to
# the default library: ../libdkm_<name>.so.  usage: bash variants.sh name "DEFS" ...
# A/B switches are compile-time only (-DDKM_AB_NO_W32=1, -DDKM_AB_DELTA_POST=1,
# -DDKM_AB_NO_POST=1, -DDKM_AB_NO_LIST=1, -DDKM_AB_CSR_OLD=1,
# -DDKM_AB_BLOCKS_PER_CU=n, -DDKM_AB_VERBOSE, -DDKM_AB_SBB=n (k_screen_b1
# block size), -DDKM_AB_B1_PREFETCH=1 (k_screen_b1 next-tile prefetch)): the
# product build reads no
# environment variable.  Every object is compiled with -DDKM_AB_VARIANT=1,
# so dkm_build_flags() of such a library is non-zero (bench.py records it,
# the tests refuse it).
set -e
cd "$(dirname "$0")"
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  d=build_$name; mkdir -p $d
  # every kernel source of the product library (the Makefile's SRCS)
  for f in $(sed -n '/^SRCS/,/[^\\]$/p' Makefile | sed 's/^SRCS *:= *//; s/\\//g'); do
    f=${f%.hip}
    x=""; [ $f = dkm_sorted ] && x="-mllvm -amdgpu-atomic-optimizer-strategy=None"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
      -fno-slp-vectorize $x -DDKM_AB_VARIANT=1 $defs -c $f.hip -o $d/$f.o &
  done
  g++ -O3 -std=c++17 -fPIC -pthread -c dkm_io.cpp -o $d/dkm_io.o &
  /opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -c dkm_comm.cpp -o $d/dkm_comm.o &
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -pthread -o ../libdkm_$name.so $d/*.o -ldl
  echo built ../libdkm_$name.so
done
