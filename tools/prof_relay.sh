#!/bin/bash
# kernel trace of C5 relay rounds under stamp tuning knobs (SHD_STAMP_SKIP: wrong output)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for sk in 0 1 2 4 7; do
  SHD_STAMP_SKIP=$sk timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_k$sk -o run -- python3 tools/relay_only.py 10 > gpurun_out/prof_k$sk.log 2>&1 || exit 1
done
