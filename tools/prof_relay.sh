#!/bin/bash
# kernel trace of 10 C5 relay rounds (tools/relay_only.py) into gpurun_out/prof_relay
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_relay -o run -- python3 tools/relay_only.py 10
