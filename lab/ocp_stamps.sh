#!/bin/bash
# Lab build (development only): libcmpc.so with the OCP kernel's phase stamps (-DCMPC_OCP_STAMPS) and the chain-only
# timing entry point (-DCMPC_OCP_CHAIN_LAB, cmpc_ocp_debug_chain) as lab/_stamps/libcmpc_ocpstamps.so, and the
# chain-only entry point without stamps as lab/_stamps/libcmpc_ocpchain.so; run tools/ocp_probe.py --stamps /
# --chain with CMPC_LIB pointing at them.
set -e
cd "$(dirname "$0")/../cheeta-mpc_amd"
make -s
mkdir -p ../lab/_stamps
HC="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Icsrc -Ibuild"
objs=$(ls build/csrc/*.o | grep -v '/k_ocp.o$' | grep -v '/ocp_api.o$')
$HC -DCMPC_OCP_STAMPS -DCMPC_OCP_CHAIN_LAB -c csrc/k_ocp.hip -o ../lab/_stamps/k_ocp_stamps.o &
p1=$!
$HC -DCMPC_OCP_CHAIN_LAB -c csrc/ocp_api.cpp -o ../lab/_stamps/ocp_api_lab.o
if [ "${OCP_STAMPS_ONLY:-0}" = 0 ]; then $HC -DCMPC_OCP_CHAIN_LAB -c csrc/k_ocp.hip -o ../lab/_stamps/k_ocp_chain.o; fi
wait $p1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../lab/_stamps/libcmpc_ocpstamps.so $objs ../lab/_stamps/k_ocp_stamps.o \
  ../lab/_stamps/ocp_api_lab.o -Wl,-rpath,/opt/rocm/lib
[ "${OCP_STAMPS_ONLY:-0}" = 0 ] && /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../lab/_stamps/libcmpc_ocpchain.so $objs ../lab/_stamps/k_ocp_chain.o \
  ../lab/_stamps/ocp_api_lab.o -Wl,-rpath,/opt/rocm/lib
echo built ../lab/_stamps/libcmpc_ocpstamps.so ../lab/_stamps/libcmpc_ocpchain.so
