#!/bin/bash
# This round's profile evidence (one gpurun call): kernel stats of the bench, of the relay
# rounds alone, and the HBM traffic passes.  Outputs under gpurun_out/; copy into profiles/.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- \
  python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 &&
bash tools/prof_relay.sh > gpurun_out/prof_relay.log 2>&1 &&
bash tools/pmc_traffic.sh gpurun_out/pmc_traffic > gpurun_out/pmc_traffic.log 2>&1
