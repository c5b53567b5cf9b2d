#!/bin/bash
# PMC passes over the C2 build (tools/c2_probe.py, AUTO engine) into gpurun_out/pmc_c2_*
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_c2_a -o run -- python3 tools/c2_probe.py 0 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_c2_b -o run -- python3 tools/c2_probe.py 0
