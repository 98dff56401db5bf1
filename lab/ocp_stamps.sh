#!/bin/bash
# Lab build (development only): libcmpc.so with the OCP kernel's phase stamps (-DCMPC_OCP_STAMPS) as
# lab/_stamps/libcmpc_ocpstamps.so; run tools/ocp_probe.py --stamps with CMPC_LIB pointing at it.
set -e
cd "$(dirname "$0")/../cheeta-mpc_amd"
make -s
mkdir -p ../lab/_stamps
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Icsrc -Ibuild -DCMPC_OCP_STAMPS \
  -c csrc/k_ocp.hip -o ../lab/_stamps/k_ocp_stamps.o
objs=$(ls build/csrc/*.o | grep -v '/k_ocp.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../lab/_stamps/libcmpc_ocpstamps.so $objs ../lab/_stamps/k_ocp_stamps.o \
  -Wl,-rpath,/opt/rocm/lib
echo built ../lab/_stamps/libcmpc_ocpstamps.so
