#!/bin/bash
# C4 rows 0-4095 at one and two label slots per CU (SHD_SSSP_SLOTS): cache hits and HBM bytes of
# the global-label kernel, one --pmc pass each, into gpurun_out/r06_c4s<slots>_*; then the
# per-dispatch summary profiles/-style CSV gpurun_out/r06_pmc_c4_slots.csv.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for sl in 1 2; do
  run() { local tag=$1; shift; SHD_SSSP_SLOTS=$sl timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/r06_c4s${sl}_$tag -o run -- python3 tools/c4_probe.py 0 4096 3 > gpurun_out/r06_c4s${sl}_$tag.log 2>&1; }
  run a TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY &&
  run f FETCH_SIZE &&
  run w WRITE_SIZE || exit 3
done
for sl in 1 2; do
  python3 tools/pmc_summary.py gpurun_out/r06_pmc_c4_slots$sl.csv sssp_global_group gpurun_out/r06_c4s${sl}_a gpurun_out/r06_c4s${sl}_f gpurun_out/r06_c4s${sl}_w | sed "s/^/slots=$sl /"
done
