#!/bin/bash
# A/B variants of the b2 screen only (dkm_b2.hip with compile-time knobs,
# linked with the product objects): ../libdkm_<name>.so.
# usage: bash variants_b2.sh name "DEFS" ...   (run `make` first)
set -e
cd "$(dirname "$0")"
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
    -fno-slp-vectorize $defs -c dkm_b2.hip -o b2_$name.o
  objs=$(ls dkm_*.o | grep -v '^dkm_b2.o$')
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -pthread -o ../libdkm_$name.so $objs b2_$name.o -ldl
  echo built ../libdkm_$name.so
done
