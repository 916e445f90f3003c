#!/bin/bash
# PMC A/B of library builds (run on the GPU box): per build in $LIBS and per counter pass, one rocprofv3 --pmc run of
# tools/prof_target.py C3 2 ${VIEWS:-16}, summed per kernel (tools/pmc_by_kernel.py) into gpurun_out/pmcab_${TAG}_<lib>_<pass>.txt
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=${TMPDIR:-/tmp}
mkdir -p gpurun_out
PASSES=("TD_TD_BUSY_sum TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
        "TCC_HIT_sum TCC_MISS_sum TCC_BUSY_sum GRBM_GUI_ACTIVE"
        "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE")
for lib in $LIBS; do
  n=$(basename $lib .so)
  for i in 0 1 2; do
    out=gpurun_out/pmcab_${TAG}_${n}_$i
    PT_LIB=$lib timeout -s KILL 100 rocprofv3 --pmc ${PASSES[$i]} --kernel-trace --output-format csv -d $out -o run -- python3 tools/prof_target.py ${CFG:-C3} 2 ${VIEWS:-16} > $out.log 2>&1 || { echo "pass $i of $lib failed"; tail -5 $out.log; exit 1; }
    python3 tools/pmc_by_kernel.py $out 2 | grep "persistent" | cut -c1-600 | tee $out.txt
  done
done
