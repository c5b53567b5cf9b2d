#!/bin/bash
# Event-queue kernels of the bench's equeue leg (tools/equeue_only.py) under a kernel trace, then
# the queue tests and the relay + queue bench leg twice.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_eqp -o run -- \
  python3 tools/equeue_only.py > gpurun_out/r06_eqp.log 2>&1 || { tail -5 gpurun_out/r06_eqp.log; exit 3; }
python3 - <<'PY'
import csv
for x in csv.DictReader(open("gpurun_out/r06_eqp/run_kernel_stats.csv")):
    n = x["Name"]
    if any(k in n for k in ("eq", "scan_excl")):
        print("  %-50s %5s %8.1f us" % (n[:50], x["Calls"], float(x["AverageNs"]) / 1e3))
PY
[ -n "$NO_TESTS" ] || timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_equeue_gpu.py \
  > gpurun_out/r06_eqp_tests.log 2>&1 || { tail -20 gpurun_out/r06_eqp_tests.log; exit 1; }
tail -1 gpurun_out/r06_eqp_tests.log
NO_TESTS=1 tools/r06_env_ab.sh DEFAULT=1 | grep "relay ms"
