#!/bin/bash
# SQ/GRBM counter passes for the kernels matching REGEX in a python command (run via gpurun).
# Usage: tools/kernel_pmc.sh TAG REGEX script.py [args...]
TAG=$1; REGEX=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
i=0
for SET in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS" \
           "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --kernel-include-regex "$REGEX" -d /tmp/$TAG-p$i -o run \
      --output-format csv -- python3 "$R/$@" > gpurun_out/$TAG/pmc_p$i.log 2>&1 || exit $?
  cp /tmp/$TAG-p$i/*counter_collection* gpurun_out/$TAG/pmc_p$i.csv
done
python3 $R/tools/pmc_table.py gpurun_out/$TAG/pmc_p*.csv > gpurun_out/$TAG/table.txt
