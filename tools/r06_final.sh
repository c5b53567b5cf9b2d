#!/bin/bash
# Round 6 record.
#   tools/r06_final.sh tests   the whole -m gpu suite (one process, per-test time limits)
#   tools/r06_final.sh 1       the default bench line, its kernel trace, relay / event-queue traces,
#                              the sharded-round and flush probes
#   tools/r06_final.sh 2       PMC traffic and counter passes over the shipped kernels
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$1" = tests ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/r06_gputests.log 2>&1; rc=$?; tail -5 gpurun_out/r06_gputests.log; exit $rc
elif [ "$1" = 1 ]; then
  timeout -k 10 500 python3 -u bench.py > gpurun_out/r06_bench.json 2> gpurun_out/r06_bench.err &&
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_prof_bench -o run -- \
    python3 bench.py --no-cpu-baseline > gpurun_out/r06_prof_bench.log 2>&1 &&
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_prof_relay -o run -- \
    python3 tools/relay_only.py 10 > gpurun_out/r06_prof_relay.log 2>&1 &&
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_prof_equeue -o run -- \
    python3 tools/equeue_only.py > gpurun_out/r06_prof_equeue.log 2>&1 &&
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_prof_c5b -o run -- \
    python3 tools/r06_c5b_probe.py > gpurun_out/r06_prof_c5b.log 2>&1 &&
  timeout -k 10 200 python3 -u tools/sharded_round_probe.py 8 > gpurun_out/r06_sharded_round_probe.txt 2>&1 &&
  timeout -k 10 200 python3 -u tools/flush_probe.py 4 > gpurun_out/r06_flush_probe.txt 2>&1
else
  bash tools/pmc_traffic.sh gpurun_out/pmc_traffic > gpurun_out/r06_pmc_traffic.log 2>&1 &&
  bash tools/pmc_c2.sh > gpurun_out/r06_pmc_c2.log 2>&1 &&
  bash tools/pmc_c3.sh > gpurun_out/r06_pmc_c3.log 2>&1 &&
  bash tools/pmc_c4.sh > gpurun_out/r06_pmc_c4.log 2>&1
fi
