#!/bin/bash
# Lab build (development only): libcmpc.so with k_ipm72's phase stamps (-DCMPC_IPM72_STAMPS) as
# lab/_stamps/libcmpc_ipm72stamps.so; run lab/ipm72_stamps.py with CMPC_LIB pointing at it.
set -e
cd "$(dirname "$0")/../cheeta-mpc_amd"
make -s
mkdir -p ../lab/_stamps
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Icsrc -Ibuild -DCMPC_IPM72_STAMPS \
  -c csrc/k_ipm72_f64.hip -o ../lab/_stamps/k_ipm72_stamps.o
objs=$(ls build/csrc/*.o | grep -v '/k_ipm72_f64.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../lab/_stamps/libcmpc_ipm72stamps.so $objs ../lab/_stamps/k_ipm72_stamps.o \
  -Wl,-rpath,/opt/rocm/lib
echo built ../lab/_stamps/libcmpc_ipm72stamps.so
