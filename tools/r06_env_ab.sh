#!/bin/bash
# Relay parity tests (TESTS, default the relay files), then per environment variant (NAME=value[,NAME=value],
# "DEFAULT=1" for the build's defaults) a kernel trace of 10 C5 rounds and the relay bench leg.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
    ${TESTS:-tests/test_relay_gpu.py tests/test_relay_shapes_gpu.py tests/test_flush_gpu.py tests/test_comm_gpu.py} \
    > gpurun_out/r06_env_tests.log 2>&1 || { tail -40 gpurun_out/r06_env_tests.log; exit 1; }
  tail -2 gpurun_out/r06_env_tests.log
fi
for v in "$@"; do
  n=$(echo "$v" | tr '/=' '__')
  env $(echo "$v" | tr ',' ' ') timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_kt_$n -o run \
    -- python3 tools/relay_only.py 10 > gpurun_out/r06_kt_$n.log 2>&1 || { tail -20 gpurun_out/r06_kt_$n.log; exit 3; }
  echo "$v $(tail -1 gpurun_out/r06_kt_$n.log)"
  python3 tools/kstats.py gpurun_out/r06_kt_$n
done
for rep in $( [ -z "$NO_AB" ] && echo 1 2 ); do
  for v in "$@"; do
    env $(echo "$v" | tr ',' ' ') timeout -k 10 150 python3 bench.py --steps 5 --no-cpu-baseline --no-c3 --no-c4 \
      --no-c5b --no-codel --no-tbucket --no-e2e 2> gpurun_out/r06_ab.err > gpurun_out/r06_ab.json || { tail -20 gpurun_out/r06_ab.err; exit 3; }
    python3 - "$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/r06_ab.json").readline()); r = d["relay"]; e = r["equeue"]
print(sys.argv[1], "relay ms/round", round(r["ms_per_round"], 4), "advance", round(e["advance_ms_per_round"], 4),
      "relay+merge", round(e["ms_per_round"], 4), "C2", round(d["ms_per_step"], 4), "ok", r.get("bit_exact_vs_cpu"))
PY
  done
done
