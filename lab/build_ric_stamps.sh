#!/bin/bash
# Lab build (CPU): libcmpc with the s_memtime phase stamps of k_ric compiled in (-DCMPC_RIC_STAMPS) ->
# lab/build/libcmpc_ricst.so. The product objects come from cheeta-mpc_amd/build (make -C cheeta-mpc_amd first).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/cheeta-mpc_amd
O=$R/lab/build/ricst; mkdir -p $O
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$R/include -I$P/csrc -I$P/build -DCMPC_RIC_STAMPS ${RIC_EXTRA}"
$H -c $P/csrc/k_ric_f64.hip -o $O/k_ric_f64.o &
$H -c $P/csrc/k_ric_f32.hip -o $O/k_ric_f32.o &
wait
OBJS=$(ls $P/build/csrc/*.o | grep -v k_ric_)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $R/lab/build/libcmpc_ricst.so $OBJS $O/k_ric_f64.o $O/k_ric_f32.o -Wl,-rpath,/opt/rocm/lib
echo built $R/lab/build/libcmpc_ricst.so
