#!/bin/bash
# C2 build timing only (bench routing leg), alternating an environment toggle for an A/B of
# build-path changes: AB_VAR=NAME tools/c2_ab.sh [v1 v2 ...]  (default 0 1; each value twice, alternating)
cd "$(dirname "$0")/.."
var=${AB_VAR:-SHD_FLAGS_DMA}
vals=("$@"); [ ${#vals[@]} -eq 0 ] && vals=(0 1)
for v in "${vals[@]}" "${vals[@]}"; do
  env "$var=$v" timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-relay \
    --no-c3 --no-c4 --no-codel --no-tbucket 2>/dev/null > gpurun_out/c2ab.json || exit 3
  python3 - "$var=$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/c2ab.json").readline())
print(sys.argv[1].split("/")[-1], "C2 ms_per_step", round(d["ms_per_step"], 4), "kernel_ms", round(d["roofline"]["kernel_ms"], 4))
PY
done
