#!/bin/bash
# GPU-box script (round 6 final evidence, part 1 of 2): FETCH_SIZE / WRITE_SIZE traffic passes and SQ counter passes
# (separate rocprofv3 runs, md5-stamped summaries) for the headline, configs 3 / 5 and the OCP lines (projected / rows,
# B = 1 and 4096); ONLY = a shell pattern of the workload keys to run (e.g. 'ocp_*'). Every pass has its own hard time
# limit; a failed pass ends the script. Run before gpu_final_r06a.sh on the same build: the summaries go to profiles/
# and the bench lines of part 2 read them (roofline.traffic, sq_counters).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/final_r06; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
WL=("N10_B4096_f64_trot|--steps 3 --warmup 1 --cpu-sample 0"
    "N20_B4096_f32_trot|--steps 3 --warmup 1 --cpu-sample 0 --horizon 20 --precision f32"
    "N10_B4096_f64_mixed|--steps 3 --warmup 1 --cpu-sample 0 --gait 1"
    "ocp_projected_B1|--ocp projected --batch 1 --steps 20 --warmup 2 --cpu-sample 0 --no-tick"
    "ocp_rows_B1|--ocp rows --batch 1 --steps 5 --warmup 1 --cpu-sample 0 --no-tick"
    "ocp_projected_B4096|--ocp projected --steps 3 --warmup 1 --cpu-sample 0 --no-tick"
    "ocp_rows_B4096|--ocp rows --steps 2 --warmup 1 --cpu-sample 0 --no-tick")
for W in "${WL[@]}"; do
  KEY=${W%%|*}; BA=${W#*|}; D=$O/traffic_$KEY; mkdir -p $D
  case "$KEY" in ${ONLY:-*}) ;; *) continue;; esac
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace --stats -d $D/pmc_$c -o run --output-format csv -- python3 $R/bench.py $BA > $D/pmc_$c.log 2>&1; rc=$?
    echo "$KEY $c rc=$rc"; [ $rc -ne 0 ] && { tail -5 $D/pmc_$c.log; exit 1; }
  done
  python3 $R/cheeta-mpc_amd/tools/pmc_traffic.py $D $O/traffic_$KEY.json "$BA" > $D/summary.txt || exit 1
  D=$O/sq_$KEY; mkdir -p $D; i=0
  for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $P --kernel-trace --stats -d $D/p$i -o run --output-format csv -- python3 $R/bench.py $BA > $D/p$i.log 2>&1; rc=$?
    echo "sq $KEY pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $D/p$i.log; exit 1; }
  done
  python3 $R/cheeta-mpc_amd/tools/pmc_summary.py $D --json $O/pmc_sq_$KEY.json > $O/sq_$KEY.txt || exit 1
done
echo all_done
