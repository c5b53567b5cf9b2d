#!/bin/bash
# PMC passes over the C4 global-label kernel (rows 0-4095 of the 50k-node BA graph, DELTA) into
# gpurun_out/pmc_c4_*: SQ issue/wait counters, cache hit rates, HBM bytes (one pass each)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
run() { timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_c4_$1 -o run -- python3 tools/c4_probe.py 0 4096 3; }
run SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS &&
run TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum SQ_WAVES SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES &&
run FETCH_SIZE &&
run WRITE_SIZE
