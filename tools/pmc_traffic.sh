#!/bin/bash
# HBM traffic passes (FETCH_SIZE and WRITE_SIZE each in a run of its own, as the pool requires):
# the C2 routing build (bench.py without the relay legs), 10 C5 relay rounds alone
# (tools/relay_only.py: no counters, no event-queue leg), the C3 and C4 builds, and tools/bw_probe (a known byte count,
# used to calibrate the counters for this code's access widths):  tools/pmc_traffic.sh <outdir>
out=${1:-gpurun_out/pmc_traffic}
mkdir -p "$out"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$out/bench_$c" -o run -- \
    python bench.py --steps 3 --warmup 1 --no-relay --no-cpu-baseline --no-c3 --no-c4 --no-codel --no-tbucket \
    --no-e2e > "$out/bench_$c.log" 2>&1 || { echo "bench pass $c failed"; tail -3 "$out/bench_$c.log"; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$out/relay_$c" -o run -- \
    python tools/relay_only.py 10 > "$out/relay_$c.log" 2>&1 || { echo "relay pass $c failed"; tail -3 "$out/relay_$c.log"; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d "$out/probe_$c" -o run -- \
    tools/bw_probe > "$out/probe_$c.log" 2>&1 || { echo "probe pass $c failed"; tail -3 "$out/probe_$c.log"; exit 1; }
  # C3: the whole 10k x 10k build on the AUTO engine (delta buckets, LDS labels); C4: one full
  # 50k x 50k build (global-label delta-stepping), the bench's c4 step
  PROBE_GRAPH=c3 timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$out/c3_$c" -o run -- \
    python tools/c2_probe.py 0 > "$out/c3_$c.log" 2>&1 || { echo "c3 pass $c failed"; tail -3 "$out/c3_$c.log"; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$out/c4_$c" -o run -- \
    python tools/c4_probe.py 0 50000 3 > "$out/c4_$c.log" 2>&1 || { echo "c4 pass $c failed"; tail -3 "$out/c4_$c.log"; exit 1; }
done
echo done
