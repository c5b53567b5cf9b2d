#!/bin/bash
# PMC passes over the C3 build (10k-node BA graph, AUTO = delta buckets) into gpurun_out/pmc_c3_*
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
export PROBE_GRAPH=c3
run() { timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_c3_$1 -o run -- python3 tools/c2_probe.py 0; }
run SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS &&
run TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES
