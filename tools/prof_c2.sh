#!/bin/bash
# kernel trace of the C2 build (tools/c2_probe.py, AUTO engine) into gpurun_out/prof_c2
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o run -- python3 tools/c2_probe.py "${@:-0}"
