#!/bin/bash
# relay tests + kernel traces of 10 C5 rounds per variant.  VARIANTS: space-separated NAME=value
# environment settings (default: the build's defaults, "DEFAULT=1"); traces into
# gpurun_out/relay_cmp_<NAME=value>.  B7_STOPS="1 2 3 4": bin_sort_v7 phase pricing.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_relay_gpu.py \
  tests/test_advice_gpu.py tests/test_configs_gpu.py > gpurun_out/relay_tests.log 2>&1 || { tail -40 gpurun_out/relay_tests.log; exit 1; }
tail -3 gpurun_out/relay_tests.log
for v in ${VARIANTS:-DEFAULT=1}; do
  n=$(echo "$v" | tr '/' '_')
  env "$v" timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "gpurun_out/relay_cmp_$n" -o run -- python3 tools/relay_only.py 10 > "gpurun_out/relay_cmp_$n.log" 2>&1 || exit 3
  echo "$v $(tail -1 "gpurun_out/relay_cmp_$n.log")"
  python3 tools/kstats.py "gpurun_out/relay_cmp_$n"
done
# bin_sort_v7 phase pricing (SHD_B7_STOP=k returns after phase k: output wrong, timing only)
if [ -n "$B7_STOPS" ]; then
  for k in $B7_STOPS; do
    SHD_B7_STOP=$k timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/b7stop_$k -o run -- python3 tools/relay_only.py 5 > gpurun_out/b7stop_$k.log 2>&1 || exit 3
  done
fi
