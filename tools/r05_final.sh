#!/bin/bash
# Round 5 record: the default bench line, its kernel trace, the relay / event-queue traces,
# then (part 2) fresh PMC traffic and counter passes over the shipped kernels.
#   tools/r05_final.sh 1   (bench + traces)      tools/r05_final.sh 2   (PMC)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$1" = 1 ]; then
  timeout -k 10 400 python3 -u bench.py > gpurun_out/r05_bench.json 2> gpurun_out/r05_bench.err &&
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05_prof_bench -o run -- \
    python3 bench.py --no-cpu-baseline > gpurun_out/r05_prof_bench.log 2>&1 &&
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05_prof_relay -o run -- \
    python3 tools/relay_only.py 10 > gpurun_out/r05_prof_relay.log 2>&1 &&
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05_prof_equeue -o run -- \
    python3 tools/equeue_only.py > gpurun_out/r05_prof_equeue.log 2>&1 &&
  timeout -k 10 200 python3 -u tools/sharded_round_probe.py 8 > gpurun_out/r05_sharded_round_probe.txt 2>&1 &&
  timeout -k 10 200 python3 -u tools/flush_probe.py 4 > gpurun_out/r05_flush_probe.txt 2>&1
else
  bash tools/pmc_traffic.sh gpurun_out/pmc_traffic > gpurun_out/r05_pmc_traffic.log 2>&1 &&
  bash tools/pmc_c2.sh > gpurun_out/r05_pmc_c2.log 2>&1 &&
  bash tools/pmc_c3.sh > gpurun_out/r05_pmc_c3.log 2>&1 &&
  bash tools/pmc_c4.sh > gpurun_out/r05_pmc_c4.log 2>&1
fi
