#!/bin/bash
# Lab A/B build (development only): libcmpc.so with one source rebuilt under extra flags, as lab/_ab/libcmpc_NAME.so;
# load it with CMPC_LIB=lab/_ab/libcmpc_NAME.so. Usage: lab/ab_build.sh NAME csrc/FILE.hip -DFLAG=V ...
set -e
name=$1; src=$2; shift 2
cd "$(dirname "$0")/../cheeta-mpc_amd"
make -s
mkdir -p ../lab/_ab
obj=../lab/_ab/$(basename "$src" .hip)_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Icsrc -Ibuild "$@" -c "$src" -o "$obj"
base=build/csrc/$(basename "$src" .hip).o
objs=$(ls build/csrc/*.o | grep -v "^$base\$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../lab/_ab/libcmpc_$name.so $objs "$obj" -Wl,-rpath,/opt/rocm/lib
echo built lab/_ab/libcmpc_$name.so
