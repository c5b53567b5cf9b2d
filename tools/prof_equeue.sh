#!/bin/bash
# kernel trace of the C5 relay + event-queue rounds (tools/equeue_only.py) into gpurun_out/prof_equeue
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_equeue -o run -- python3 tools/equeue_only.py
