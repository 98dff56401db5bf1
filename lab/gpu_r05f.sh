#!/bin/bash
# Session script (round 5): SQ counters of the chain-only lab kernel (k_ocp_chain_lab) and of the grid-form solve
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05f; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "exit $1 in $2"; cat $O/$2.log | tail -20; exit 1;; esac; }
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD"; do
  i=$((i+1))
  CMPC_LIB=$R/lab/_stamps/libcmpc_ocpchain.so timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --stats -d $O/pmc$i -o run --output-format csv -- python3 $R/tools/ocp_probe.py --chain > $O/pmc$i.log 2>&1; fatal $? pmc$i
done
echo done
