#!/bin/bash
# relay tests + kernel traces of 10 C5 rounds (one per entry of STAMPS, default "6": an entry
# names a variant selected through the environment while tuning), into gpurun_out/relay_cmp_<entry>
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_relay_gpu.py \
  tests/test_advice_gpu.py tests/test_configs_gpu.py > gpurun_out/relay_tests.log 2>&1 || { tail -40 gpurun_out/relay_tests.log; exit 1; }
tail -3 gpurun_out/relay_tests.log
for st in ${STAMPS:-6}; do
  SHD_RELAY_STAMP=$st timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/relay_cmp_$st -o run -- python3 tools/relay_only.py 10 > gpurun_out/relay_cmp_$st.log 2>&1 || exit 3
  tail -1 gpurun_out/relay_cmp_$st.log
done
# bin_sort_v7 phase pricing (SHD_B7_STOP=k returns after phase k: output wrong, timing only)
if [ -n "$B7_STOPS" ]; then
  for k in $B7_STOPS; do
    SHD_B7_STOP=$k timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/b7stop_$k -o run -- python3 tools/relay_only.py 5 > gpurun_out/b7stop_$k.log 2>&1 || exit 3
  done
fi
