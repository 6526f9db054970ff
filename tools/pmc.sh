#!/bin/bash
# Counter passes (one rocprofv3 run per counter group; --pmc never combined with other traces).
# Usage: bash tools/pmc.sh TAG REGEX -- cmd...
TAG=$1; RE=$2; shift 3
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$RE" -d gpurun_out/$TAG/p$i -o pmc --output-format csv -- "$@" \
    > gpurun_out/$TAG/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 gpurun_out/$TAG/p$i.log; exit 1; }
done
echo "pmc done"
