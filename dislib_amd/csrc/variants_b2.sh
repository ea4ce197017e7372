#!/bin/bash
# A/B and debug variants of the screens that rebuild only the named sources
# (dkm_b2.hip, dkm_sorted.hip, ...) with compile-time knobs and link them
# with the product objects: ../libdkm_<name>.so.  Run `make` first.
# usage: bash variants_b2.sh name "DEFS" [sources...]   (default dkm_b2 dkm_sorted)
set -e
cd "$(dirname "$0")"
name=$1; defs=$2; shift 2
srcs=${*:-dkm_b2 dkm_sorted}
objs=""
for f in $srcs; do
  x=""; [ $f = dkm_sorted ] && x="-mllvm -amdgpu-atomic-optimizer-strategy=None"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
    -fno-slp-vectorize $x -DDKM_AB_VARIANT=1 $defs -c $f.hip -o v_${name}_$f.o
  objs="$objs v_${name}_$f.o"
done
keep=$(for o in dkm_*.o; do b=${o%.o}; case " $srcs " in *" $b "*) ;; *) echo $o;; esac; done)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -pthread -o ../libdkm_$name.so $keep $objs -ldl
echo built ../libdkm_$name.so
