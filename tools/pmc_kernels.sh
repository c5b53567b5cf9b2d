#!/bin/bash
# PMC passes restricted to kernels matching a regex, one counter group per run:
#   tools/pmc_kernels.sh <outdir> <regex> <command...>
out=$1; re=$2; shift 2
mkdir -p "$out"
i=0
for ctrs in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
  "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
  "FETCH_SIZE" \
  "WRITE_SIZE" ; do
  i=$((i+1))
  echo "=== pass $i: $ctrs"
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex "$re" --output-format csv -d "$out/p$i" -o run -- "$@" > "$out/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -3 "$out/p$i.log"; exit 1; }
done
