#!/bin/bash
# Lab build (development only): libcmpc.so with k_sqp_step's (-DCMPC_SQP_STAMPS) and the foothold condensing's
# (-DCMPC_COND_STAMPS) phase stamps as lab/_stamps/libcmpc_nlpstamps.so; run lab/nlp_stamps.py with CMPC_LIB set.
set -e
cd "$(dirname "$0")/../cheeta-mpc_amd"
make -s
mkdir -p ../lab/_stamps
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Icsrc -Ibuild"
$H -DCMPC_SQP_STAMPS -c csrc/k_sqp.hip -o ../lab/_stamps/k_sqp_stamps.o
$H -DCMPC_COND_STAMPS -c csrc/k_condense.hip -o ../lab/_stamps/k_condense_stamps.o
objs=$(ls build/csrc/*.o | grep -v -e '/k_sqp.o$' -e '/k_condense.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../lab/_stamps/libcmpc_nlpstamps.so $objs \
  ../lab/_stamps/k_sqp_stamps.o ../lab/_stamps/k_condense_stamps.o -Wl,-rpath,/opt/rocm/lib
echo built ../lab/_stamps/libcmpc_nlpstamps.so
