#!/bin/bash
# Build libldpc_hip.so variants with compile-time switches into variants/<name>.so
# (in this container; the .so files travel to the GPU box with the tree).
# usage: tools/build_variants.sh name1 "-DFOO=1 -DBAR" name2 "-DBAZ" ...
set -e
cd "$(dirname "$0")/.."
mkdir -p variants
CS=ldpc-simulator_amd/csrc
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  bd=$CS/build_$name
  rm -rf $bd; mkdir -p $bd
  objs=""
  for f in $(sed -n "s/^SRCS = //p" $CS/Makefile); do
    x=""; case $f in *.cpp) x="-x hip";; esac
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math $defs $x -c $CS/$f -o $bd/$f.o &
    objs="$objs $bd/$f.o"
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o variants/$name.so $objs -ldl
  rm -rf $bd
  echo "variants/$name.so ($defs)"
done
