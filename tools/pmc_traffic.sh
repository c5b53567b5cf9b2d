#!/bin/bash
# HBM traffic passes (FETCH_SIZE and WRITE_SIZE each in a run of its own, as the pool requires)
# over the bench's routing + relay legs and over tools/bw_probe (a known byte count, used to
# calibrate the counters for this code's access widths):  tools/pmc_traffic.sh <outdir>
out=${1:-gpurun_out/pmc_traffic}
mkdir -p "$out"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$out/bench_$c" -o run -- \
    python bench.py --steps 3 --warmup 1 --relay-steps 3 --no-cpu-baseline --no-c3 --no-c4 \
    > "$out/bench_$c.log" 2>&1 || { echo "bench pass $c failed"; tail -3 "$out/bench_$c.log"; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d "$out/probe_$c" -o run -- \
    tools/bw_probe > "$out/probe_$c.log" 2>&1 || { echo "probe pass $c failed"; tail -3 "$out/probe_$c.log"; exit 1; }
done
echo done
