#!/bin/bash
# Round 6 relay A/B: relay parity tests on the default library, then per tuning library
# (ablibs/<name>.so, SHD_ACCEL_LIB) a kernel trace of 10 C5 rounds and the relay bench leg, then
# optional PMC passes of the default library's relay kernels (PMC=1).
#   tools/r06_relay_ab.sh base v1 ...
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_relay_gpu.py \
    tests/test_relay_shapes_gpu.py tests/test_flush_gpu.py tests/test_comm_gpu.py tests/test_hostcomm.py > gpurun_out/r06_relay_tests.log 2>&1 \
    || { tail -40 gpurun_out/r06_relay_tests.log; exit 1; }
  tail -2 gpurun_out/r06_relay_tests.log
fi
for lib in "$@"; do
  export SHD_ACCEL_LIB=$PWD/ablibs/$lib.so
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_kt_$lib -o run \
    -- python3 tools/relay_only.py 10 > gpurun_out/r06_kt_$lib.log 2>&1 || { tail -20 gpurun_out/r06_kt_$lib.log; exit 3; }
  echo "$lib $(tail -1 gpurun_out/r06_kt_$lib.log)"
  python3 tools/kstats.py gpurun_out/r06_kt_$lib
done
for rep in $( [ -z "$NO_AB" ] && echo 1 2 ); do
  for lib in "$@"; do
    export SHD_ACCEL_LIB=$PWD/ablibs/$lib.so
    timeout -k 10 150 python3 bench.py --steps 5 --no-cpu-baseline --no-c3 --no-c4 --no-codel --no-tbucket \
      --no-e2e 2>/dev/null > gpurun_out/r06_ab.json || exit 3
    python3 - "$lib" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/r06_ab.json").readline()); r = d["relay"]; e = r["equeue"]
print(sys.argv[1], "relay ms/round", round(r["ms_per_round"], 4), "advance", round(e["advance_ms_per_round"], 4),
      "relay+merge", round(e["ms_per_round"], 4), "C2", round(d["ms_per_step"], 4))
PY
  done
done
unset SHD_ACCEL_LIB
if [ -n "$PMC" ]; then
  run() { local tag=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/r06_pmc_relay_$tag -o run -- python3 tools/relay_only.py 4 > /dev/null 2>&1; }
  run a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR &&
  run b SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAVES &&
  run c FETCH_SIZE &&
  run d WRITE_SIZE &&
  python3 tools/pmc_summary.py gpurun_out/r06_pmc_relay.csv "" gpurun_out/r06_pmc_relay_a gpurun_out/r06_pmc_relay_b \
    gpurun_out/r06_pmc_relay_c gpurun_out/r06_pmc_relay_d | grep -E "stamp|bin_sort|draws|hist|col_scan" || exit 4
fi
