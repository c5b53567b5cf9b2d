#!/bin/bash
# PMC passes over the pipeline-7 relay kernels (tools/relay_only.py 4: C5 rounds) into
# gpurun_out/pmc_relay_*: SQ issue/wait counters and LDS counters (one pass each)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
run() { local tag=$1; shift; timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_relay_$tag -o run -- python3 tools/relay_only.py 4; }
run a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS &&
run b SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS
