#!/bin/bash
# Relay tuning sweep over C5 rounds: tools/relay_sweep.sh "name:VAR=v,VAR=v name2:..." -- kernel
# stats per entry in gpurun_out/sw_<name>, the round time in gpurun_out/sw_<name>.log
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for e in $1; do
  name=${e%%:*}; vars=${e#*:}
  env ${vars//,/ } timeout -k 10 100 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sw_$name -o run -- python3 tools/relay_only.py 10 > gpurun_out/sw_$name.log 2>&1 || exit 1
done
