#!/bin/bash
# LDS bank-conflict share and timing of library variants on the C2 build and the C3 build:
#   tools/ab_pmc_lds.sh <lib.so> ...   (each: one --pmc pass on C2, C2 step timing, C3 AUTO timing)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for lib in "$@"; do
  export SHD_ACCEL_LIB=$lib
  name=$(basename $lib .so)
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pmclds_$name -o run -- python3 tools/c2_probe.py 0 > /dev/null 2>&1 || exit 3
  python3 tools/pmc_summary.py gpurun_out/pmclds_$name.csv sssp_lds gpurun_out/pmclds_$name
  timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-relay \
      --no-c3 --no-c4 --no-codel --no-tbucket --no-e2e 2>/dev/null > gpurun_out/libab.json || exit 3
  c2=$(python3 -c "import json; d=json.loads(open('gpurun_out/libab.json').readline()); print(round(d['ms_per_step'], 4), round(d['roofline']['kernel_ms'], 4))")
  c3=$(PROBE_GRAPH=c3 timeout -k 10 120 python3 tools/c2_probe.py 0 2>/dev/null | tail -1)
  echo "$name C2 step/kernel $c2 | C3 $c3"
done
