#!/bin/bash
# Round 4 start: baseline bench at HEAD plus fresh PMC passes over the shipped C2/C3/C4 kernels.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r04_start_bench.log 2>&1 &&
bash tools/pmc_c2.sh > gpurun_out/r04_pmc_c2.log 2>&1 &&
bash tools/pmc_c3.sh > gpurun_out/r04_pmc_c3.log 2>&1 &&
bash tools/pmc_c4.sh > gpurun_out/r04_pmc_c4.log 2>&1
