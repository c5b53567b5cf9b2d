#!/bin/bash
# event-queue tests + kernel traces of tools/equeue_only.py per variant.  VARIANTS: space-separated
# NAME=value environment settings; traces into gpurun_out/eq_cmp_<NAME=value>.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_equeue_gpu.py \
  > gpurun_out/eq_tests.log 2>&1 || { tail -40 gpurun_out/eq_tests.log; exit 1; }
tail -3 gpurun_out/eq_tests.log
for v in ${VARIANTS:-DEFAULT=1}; do
  n=$(echo "$v" | tr '/' '_')
  env "$v" timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "gpurun_out/eq_cmp_$n" -o run -- python3 tools/equeue_only.py > "gpurun_out/eq_cmp_$n.log" 2>&1 || exit 3
  echo "$v $(tail -1 "gpurun_out/eq_cmp_$n.log")"
  python3 tools/kstats.py "gpurun_out/eq_cmp_$n"
done
