#!/bin/bash
# Memory-system PMC passes (TLB, L1/L2 hits, request latency) for kernels matching a regex:
#   tools/pmc_diag.sh <outdir> <regex> <command...>
out=$1; re=$2; shift 2
mkdir -p "$out"
i=0
for ctrs in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
  "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum" \
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum" \
  "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_UTCL1_THRASHING_STALL_sum" \
  "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT" ; do
  i=$((i+1))
  echo "=== pass $i: $ctrs"
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex "$re" --output-format csv -d "$out/p$i" -o run -- "$@" > "$out/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -3 "$out/p$i.log"; exit 1; }
done
