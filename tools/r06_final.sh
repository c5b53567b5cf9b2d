#!/bin/bash
# Round 6 record.
#   tools/r06_final.sh tests   the whole -m gpu suite (one process, per-test time limits)
#   tools/r06_final.sh 1       the default bench line, its kernel trace, relay / event-queue traces,
#                              the sharded-round trace and probe, the flush probe
#   tools/r06_final.sh 2       PMC traffic and counter passes over the shipped kernels
#   tools/r06_final.sh relay   SQ / traffic counters of the relay kernels (profiles/r06_pmc_relay.csv)
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
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r06_shtr -o run -- \
    python3 tools/sharded_round_probe.py 8 > gpurun_out/r06_shtr.log 2>&1 &&
  python3 tools/r06_shard_trace.py gpurun_out/r06_shtr 8 > gpurun_out/r06_sharded_round_trace.txt &&
  timeout -k 10 200 python3 -u tools/sharded_round_probe.py 8 > gpurun_out/r06_sharded_round_probe.txt 2>&1 &&
  timeout -k 10 200 python3 -u tools/flush_probe.py 4 > gpurun_out/r06_flush_probe.txt 2>&1
elif [ "$1" = relay ]; then
  # counters of the relay kernels, one pass per counter group
  run() { local tag=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/r06_pmc_relay_$tag -o run -- python3 tools/relay_only.py 4 > gpurun_out/r06_pmc_relay_$tag.log 2>&1; }
  run a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR &&
  run b SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAVES &&
  run c FETCH_SIZE &&
  run d WRITE_SIZE &&
  python3 tools/pmc_summary.py gpurun_out/r06_pmc_relay.csv "" gpurun_out/r06_pmc_relay_a gpurun_out/r06_pmc_relay_b \
    gpurun_out/r06_pmc_relay_c gpurun_out/r06_pmc_relay_d > gpurun_out/r06_pmc_relay.txt &&
  grep -E "stamp|bin_sort|draws|hist|col_scan" gpurun_out/r06_pmc_relay.csv
else
  bash tools/pmc_traffic.sh gpurun_out/pmc_traffic > gpurun_out/r06_pmc_traffic.log 2>&1 &&
  bash tools/pmc_c2.sh > gpurun_out/r06_pmc_c2.log 2>&1 &&
  bash tools/pmc_c3.sh > gpurun_out/r06_pmc_c3.log 2>&1 &&
  bash tools/pmc_c4.sh > gpurun_out/r06_pmc_c4.log 2>&1
fi
